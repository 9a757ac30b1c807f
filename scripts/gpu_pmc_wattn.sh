#!/bin/bash
# SQ counters on the window-attention micro-benchmark, one pass per counter group (8 SQ slots
# each).  usage: bash scripts/gpu_pmc_wattn.sh <tag>
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
out="$R/gpurun_out/pmc_wattn${1:+_$1}"
mkdir -p "$out"
timeout -k 10 120 rocprofv3 -L > "$out/avail.txt" 2>&1 || true
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "wattn" -f csv -d "$out/$n" -o w -- \
      python3 "$R/scripts/bench_wattn.py" 2 > "$out/$n.log" 2>&1
  local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$out/$n.log"; exit $rc; }
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS
run p2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM
run p3 SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SMEM SQ_INST_CYCLES_SMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_EXP SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT
