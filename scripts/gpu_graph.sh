#!/bin/bash
# bench each config eager and with whole-step hipGraph capture
tag=$1; shift
out=gpurun_out/graph_$tag; mkdir -p $out
for c in "$@"; do
  for g in "" "--graph"; do
    n=${c}${g:+_graph}
    timeout -k 10 300 python3 bench.py --config $c $g --no-cpu-baseline > $out/$n.json 2> $out/$n.err
    r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || exit $r
    python3 -c "import json;d=json.loads(open('$out/$n.json').read().strip().splitlines()[-1]);print('$n',d['value'],d['ms_per_step'])"
  done
done
