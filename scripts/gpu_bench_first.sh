#!/bin/bash
# First bench on the GPU box: a small-volume sanity run, then the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --size 96 --batch 1 --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err
rc=$?; echo "small rc=$rc"; tail -c 1500 gpurun_out/bench_small.json
[ $rc -eq 0 ] || { tail -20 gpurun_out/bench_small.err; exit $rc; }
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; echo "full rc=$rc"; tail -c 3000 gpurun_out/bench_full.json; tail -5 gpurun_out/bench_full.err
exit $rc
