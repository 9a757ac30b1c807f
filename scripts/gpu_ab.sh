#!/bin/bash
# A/B of libmmni.so builds on the window-attention micro-benchmark, alternating: gpu_ab.sh LIB_B [reps]
B=$1; n=${2:-2}
for i in $(seq $n); do
  for lib in "" "$B"; do
    MMNI_LIB=$lib timeout -k 10 120 python3 scripts/bench_wattn.py 10 > gpurun_out/ab.json 2>&1
    r=$?; echo "${lib:-default} rc=$r $(tail -1 gpurun_out/ab.json | cut -c1-200)"; [ $r -eq 0 ] || exit $r
  done
done
