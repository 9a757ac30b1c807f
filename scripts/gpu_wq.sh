#!/bin/bash
# window-attention parity subset + alternating A/B micro-benchmark against a variant library
# usage: gpu_wq.sh VARIANT_SO [reps]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread \
    -k "window_attention or swinfusion3d" > gpurun_out/pt_wq.log 2>&1
r=$?; tail -4 gpurun_out/pt_wq.log; [ $r -eq 0 ] || exit $r
bash scripts/gpu_ab.sh "$1" ${2:-2}
