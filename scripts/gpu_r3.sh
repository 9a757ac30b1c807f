#!/bin/bash
# Round-3 GPU session: the new / changed parity tests verbose, then the whole GPU suite, smoke and
# the C3 bench line.  Each GPU step has its own limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r3a}
NEW=${NEW:-tests/test_configs_gpu.py tests/test_fullsize_gpu.py tests/test_kernels_gpu.py::test_swin_v2_attention_grads_are_deterministic}
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread $NEW > gpurun_out/pytest_new_$TAG.log 2>&1
rc=$?; echo "new tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|parity|C5|C1|2\^23|passed|failed" gpurun_out/pytest_new_$TAG.log | tail -40
[ $rc -eq 0 ] || exit $rc
[ "${2:-all}" = "new" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -5 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
exit $rc
