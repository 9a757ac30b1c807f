#!/bin/bash
# Time the window-attention micro-benchmark against each variant library given (MMNI_LIB).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in "$@"; do
  echo "== $lib"
  MMNI_LIB=$PWD/$lib MMNI_WATTN_ABL=$lib timeout -k 10 120 python scripts/bench_wattn.py 5 2>/dev/null | tail -1 || exit 1
done
