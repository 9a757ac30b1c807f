#!/bin/bash
# A/B of libmmni.so builds on a micro-benchmark, alternating: gpu_ab.sh LIB_B [reps] [script]
# (default script: the window-attention micro-benchmark)
B=$1; n=${2:-2}; script=${3:-scripts/bench_wattn.py}
for i in $(seq $n); do
  for lib in "" "$B"; do
    MMNI_LIB=$lib timeout -k 10 120 python3 $script 10 > gpurun_out/ab.json 2>&1
    r=$?; echo "${lib:-default} rc=$r $(tail -1 gpurun_out/ab.json | cut -c1-300)"; [ $r -eq 0 ] || exit $r
  done
done
