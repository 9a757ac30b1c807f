#!/bin/bash
# SQ / TA counters on the MLP micro-benchmark, one pass per counter group.
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
out="$R/gpurun_out/pmc_mlp${1:+_$1}"
mkdir -p "$out"
run() {
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "mlp_" -f csv -d "$out/$n" -o w -- \
      python3 "$R/scripts/bench_mlp.py" > "$out/$n.log" 2>&1
  local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$out/$n.log"; exit $rc; }
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS
run p2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU_TRANS_F32
run p3 SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_THREAD_CYCLES_VALU TA_TA_BUSY_sum TA_BUSY_max
