#!/bin/bash
# SQ counters on the window-attention micro-benchmark (two passes, 8 SQ slots each).
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
out="$R/gpurun_out/pmc_wattn${1:+_$1}"
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS \
    --kernel-include-regex "wattn" -f csv -d "$out/p1" -o w -- python3 "$R/scripts/bench_wattn.py" 2 > "$out/p1.log" 2>&1
rc=$?; echo "p1 rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$out/p1.log"; exit $rc; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM \
    --kernel-include-regex "wattn" -f csv -d "$out/p2" -o w -- python3 "$R/scripts/bench_wattn.py" 2 > "$out/p2.log" 2>&1
rc=$?; echo "p2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$out/p2.log"; exit $rc; }
