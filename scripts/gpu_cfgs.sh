#!/bin/bash
# composite / golden tests, then the c4 and c5 benches (eager and whole-step graph)
tag=${1:-x}
timeout -k 10 400 python -u -m pytest tests/test_composite_gpu.py tests/test_golden_gpu.py tests/test_kernels_gpu.py -q -x \
    -k "composite or crossmodal or enc or mha or MHA or golden" --timeout 250 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
r=$?; tail -3 gpurun_out/pytest_$tag.log; [ $r -eq 0 ] || exit $r
for c in c4 c5; do
  for g in "" "--graph"; do
    bash scripts/gpu_bench_quick.sh ${tag}_$c${g:+g} $c $g | head -2 || exit 1
  done
done
