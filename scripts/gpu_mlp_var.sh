#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "mlp" --timeout 120 --timeout-method thread > gpurun_out/pytest_mlpv.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_mlpv.log; [ $rc -eq 0 ] || exit $rc
for lib in "$@"; do echo "== $lib"; MMNI_LIB=$PWD/$lib timeout -k 10 120 python scripts/bench_mlp.py 2>/dev/null | tail -1 || exit 1; done
