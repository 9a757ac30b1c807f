#!/bin/bash
# window-attention parity (kernels + full-size) and the C3-shape micro-benchmark
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-wq}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fullsize_gpu.py -q -x -k "window or swin" \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_wattn.py 10 > gpurun_out/bench_wattn_$TAG.json 2>&1
rc=$?; echo "bench_wattn rc=$rc"; cat gpurun_out/bench_wattn_$TAG.json
exit $rc
