#!/bin/bash
# kernel parity (test_kernels_gpu + full-size) then the wattn / mha micro-benchmarks
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-k}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fullsize_gpu.py -q \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/bench_wattn.py 10 > gpurun_out/bench_wattn_$TAG.json 2>&1
r=$?; echo "bench_wattn rc=$r"; tail -1 gpurun_out/bench_wattn_$TAG.json; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python scripts/bench_mha.py 5 > gpurun_out/bench_mha_$TAG.json 2>&1
r=$?; echo "bench_mha rc=$r"; tail -1 gpurun_out/bench_mha_$TAG.json; [ $r -eq 0 ] || exit $r
exit $rc
