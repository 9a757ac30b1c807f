#!/bin/bash
# rocprofv3 kernel stats + two SQ counter passes on the window-attention micro-benchmark.
# usage: gpu_prof_wattn.sh TAG [kernel-regex]
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
TAG=${1:-p}; RX=${2:-wattn}
out="$R/gpurun_out/prof_wattn_$TAG"
mkdir -p "$out"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d "$out/trace" -o w -- python3 "$R/scripts/bench_wattn.py" 3 \
    > "$out/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$out/trace.log"; exit $rc; }
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$RX" -f csv -d "$out/$n" -o w -- \
      python3 "$R/scripts/bench_wattn.py" 2 > "$out/$n.log" 2>&1
  local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$out/$n.log"; exit $rc; }
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS
run p2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM
python3 "$R/scripts/pmc_table.py" "$out" > "$out/sq_table.txt" 2>&1
find "$out/trace" -name "*kernel_stats.csv" -exec cat {} \;
exit 0
