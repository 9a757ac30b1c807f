#!/bin/bash
# Quad (four-rows-per-lane) attention backward: parity of each variant library on the window
# attention cases, then alternating N=1 bench runs.  usage: gpu_q4.sh lib.so [lib.so ...]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in "$@"; do
  n=$(basename "$lib" .so)
  MMNI_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "${K:-window_attention}" -x -q \
      --timeout 120 --timeout-method thread > gpurun_out/q4_tests_$n.log 2>&1
  rc=$?; echo "$n tests rc=$rc"; tail -3 gpurun_out/q4_tests_$n.log; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_bench_ab.sh "$@"
