#!/bin/bash
# Alternate N=1 bench runs over variant libraries (MMNI_LIB), printing pairs/s and the attention
# kernel times of each.  usage: gpu_bench_ab.sh lib.so [lib.so ...]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in "$@"; do
  MMNI_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || exit 1
  cp gpurun_out/ab.json gpurun_out/ab_$(basename "$lib" .so).json
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); k=d['kernels']
print(sys.argv[1], d['value'], d['ms_per_step'], {x: k[x]['avg_ms'] for x in k if (x.startswith('wattn') and 'k0_C12' in x) or x.startswith('ln_mlp') or x.startswith('ln_linear_bwd_12x36') or x.startswith(tuple(sys.argv[2:]))})" "$lib" $AB_EXTRA
done
