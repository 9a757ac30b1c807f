#!/bin/bash
# Round evidence for the current tree: smoke, the GPU suite, the C3 bench line, a rocprofv3
# kernel-stats pass of the C3 bench, and the HBM counters (FETCH_SIZE / WRITE_SIZE, one per run) of
# the window-attention backward on the C3 micro-benchmark.  usage: gpu_evidence.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r3}
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
fatal() { [ "$1" -ge 124 ]; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/smoke_$TAG.log)"; fatal $rc && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu_$TAG.log | head; tail -1 gpurun_out/pytest_gpu_$TAG.log; fatal $rc && exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_c3_$TAG.json | cut -c1-700; fatal $rc && exit $rc
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof_c3_$TAG" -o k -- \
    python3 "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 > "$R/gpurun_out/prof_c3_$TAG.json" 2> "$R/gpurun_out/prof_c3_$TAG.err" )
rc=$?; echo "prof c3 rc=$rc"; fatal $rc && exit $rc
f=$(find gpurun_out/prof_c3_$TAG -name "*kernel_stats.csv" | head -1); head -8 "$f" | cut -c1-160
out="$R/gpurun_out/pmc_$TAG"; mkdir -p "$out"
for c in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "wattn_bwd_q4|wattn_fwd_bcs" -f csv \
      -d "$out/$c" -o w -- python3 "$R/scripts/bench_wattn.py" 3 > "$out/$c.log" 2>&1 )
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || { tail -3 "$out/$c.log"; exit $rc; }
done
exit 0
