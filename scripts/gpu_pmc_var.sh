#!/bin/bash
# LDS counters of the window-attention backward for each variant library (MMNI_LIB), one pass each.
# usage: bash scripts/gpu_pmc_var.sh <tag> lib1.so lib2.so ...
R="$GRAFT_REPO_ROOT"
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
out="$R/gpurun_out/pmc_var_$tag"
mkdir -p "$out"
for lib in "$@"; do
  n=$(basename "$lib" .so)
  MMNI_LIB="$R/$lib" timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_BUSY_CYCLES \
      --kernel-include-regex "wattn_bwd" -f csv -d "$out/$n" -o w -- python3 "$R/scripts/bench_wattn.py" 2 > "$out/$n.log" 2>&1
  rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$out/$n.log"; exit $rc; }
done
