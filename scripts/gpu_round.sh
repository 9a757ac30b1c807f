#!/bin/bash
# GPU-box sequence: parity tests, then the bench line.  Every GPU step has its own limit;
# the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
if [ "${2:-bench}" = "bench" ]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_$TAG.json; tail -5 gpurun_out/bench_$TAG.err
fi
exit $rc
