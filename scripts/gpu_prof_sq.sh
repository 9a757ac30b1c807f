#!/bin/bash
# two SQ counter passes over a micro-benchmark. usage: gpu_prof_sq.sh TAG KERNEL_REGEX SCRIPT [ARGS...]
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
TAG=$1; RX=$2; shift 2
out="$R/gpurun_out/prof_sq_$TAG"
mkdir -p "$out"
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$RX" -f csv -d "$out/$n" -o w -- \
      python3 "$R/$SCRIPT" $ARGS > "$out/$n.log" 2>&1
  local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$out/$n.log"; exit $rc; }
}
SCRIPT=$1; shift; ARGS="$*"
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS
run p2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_VMEM
python3 "$R/scripts/pmc_table.py" "$out" > "$out/sq_table.txt" 2>&1
cat "$out/sq_table.txt"
exit 0
