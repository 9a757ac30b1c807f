#!/bin/bash
# window-attention parity (kernels + full-size) and the micro-benchmark
tag=${1:-w}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fullsize_gpu.py tests/test_golden_gpu.py -q -x \
    -k "window or wattn or fullsize or c3 or swin or golden" --timeout 200 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
r=$?; tail -4 gpurun_out/pytest_$tag.log; [ $r -eq 0 ] || exit $r
timeout -k 10 120 python3 scripts/bench_wattn.py 10 > gpurun_out/bench_wattn_$tag.json; r=$?; cat gpurun_out/bench_wattn_$tag.json; exit $r
