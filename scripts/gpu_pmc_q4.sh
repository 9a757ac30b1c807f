#!/bin/bash
# SQ counters and HBM traffic of the merged window-attention backward (wattn_bwd_q4m / q4k) for the
# current library and build/base.so (the round-2 kernel: per-step readlane + global dk/dv stores,
# DPP reduction stages as separate moves), on the C3 micro-benchmark shape.  One counter pass per
# rocprofv3 run (FETCH_SIZE and WRITE_SIZE cannot share a pass).  usage: gpu_pmc_q4m.sh TAG
R="$GRAFT_REPO_ROOT"
TAG=${1:-q4m}
out="$R/gpurun_out/pmc_q4_$TAG"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
run() {  # variant lib pass counters...
  local v=$1 lib=$2 n=$3; shift 3
  MMNI_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "wattn_bwd_q4" -f csv \
      -d "$out/$v/$n" -o w -- python3 "$R/scripts/bench_wattn.py" 3 > "$out/$v/$n.log" 2>&1
  local rc=$?; echo "$v $n rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$out/$v/$n.log"; exit $rc; }
}
for v in new base; do
  lib=""; [ $v = base ] && lib="$R/build/base.so"
  mkdir -p "$out/$v"
  run $v "$lib" p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS
  run $v "$lib" p2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_SMEM
  run $v "$lib" p3 FETCH_SIZE
  run $v "$lib" p4 WRITE_SIZE
  python3 "$R/scripts/pmc_table.py" "$out/$v" > "$out/$v/table.txt" 2>&1
  echo "== $v"; cat "$out/$v/table.txt"
done
exit 0
