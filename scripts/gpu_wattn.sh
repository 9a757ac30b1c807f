#!/bin/bash
# Window-attention check on the GPU box: kernel parity tests, then the C3-shape micro-benchmark.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-wa}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "window" --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_wattn.py 5 > gpurun_out/bench_wattn_$TAG.json 2>&1
rc=$?; grep wattn gpurun_out/bench_wattn_$TAG.json
exit $rc
