#!/bin/bash
# MLP kernels on the GPU box: parity tests, then the C3-shape timing.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-mlp}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "mlp or token_linear or layernorm" --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_mlp.py > gpurun_out/bench_mlp_$TAG.json 2>&1
rc=$?; tail -2 gpurun_out/bench_mlp_$TAG.json
exit $rc
