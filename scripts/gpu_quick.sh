#!/bin/bash
# Quick GPU check: kernel parity tests + the token-op and window-attention micro-benchmarks.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_kernels.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_kernels.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_tokenops.py > gpurun_out/bench_tokenops.json 2>&1
rc=$?; cat gpurun_out/bench_tokenops.json | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_wattn.py 5 > gpurun_out/bench_wattn.json 2>&1
rc=$?; tail -3 gpurun_out/bench_wattn.json
exit $rc
