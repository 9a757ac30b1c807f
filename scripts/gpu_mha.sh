#!/bin/bash
# MHA parity tests, the MHA micro-benchmark, and its rocprof kernel stats
tag=${1:-m}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_golden_gpu.py tests/test_composite_gpu.py -q \
    -k "mha or MHA or dropout or crossmodal or enc or composite" --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
r=$?; tail -5 gpurun_out/pytest_$tag.log; [ $r -eq 0 ] || exit $r
timeout -k 10 200 python scripts/bench_mha.py 10 > gpurun_out/bench_mha_$tag.json; r=$?; cat gpurun_out/bench_mha_$tag.json; [ $r -eq 0 ] || exit $r
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_mha_$tag -o mha -- python3 scripts/bench_mha.py 5 > /dev/null 2> gpurun_out/prof_mha_$tag.err
r=$?; echo "prof rc=$r"; exit $r
