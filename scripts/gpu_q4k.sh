#!/bin/bash
# Key-stationary window-attention backward session: op micro-benchmark, window-attention parity
# subset, A/B of the attention micro-benchmark against build/base.so, then gpu_r3.sh steps ($2).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-q4k}
if [ -x scripts/ubench_ops ] && [ ! -f gpurun_out/ubench_ops_$TAG.txt ]; then
  timeout -k 10 120 ./scripts/ubench_ops > gpurun_out/ubench_ops_$TAG.txt 2>&1; echo "ubench rc=$?"; cat gpurun_out/ubench_ops_$TAG.txt
fi
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "window_attention" \
  tests/test_fullsize_gpu.py::test_window_attention_c3_geometry_vs_fp64_oracle tests/test_golden_gpu.py > gpurun_out/pytest_wattn_$TAG.log 2>&1
rc=$?; echo "wattn parity rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_wattn_$TAG.log | tail -8
[ $rc -ne 0 ] && exit $rc
STEPS=${2:-ab,bench,profc3,suite,smoke}
exec_steps() { bash scripts/gpu_r3.sh $TAG "$STEPS"; }
exec_steps
