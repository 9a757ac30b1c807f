#!/bin/bash
# one bench run (config $2, default c3) and a summary of its top kernels
tag=${1:-q}; cfg=${2:-c3}; shift 2 2>/dev/null
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --config $cfg --no-cpu-baseline "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
r=$?; [ $r -eq 0 ] || { tail -5 gpurun_out/bench_$tag.err; exit $r; }
python3 - "$tag" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(d["value"], d["unit"], d["ms_per_step"], "ms/step", d["roofline"]["kernel"], d["roofline"]["avg_ms"], d["roofline"]["frac"])
for t, n, a in sorted(((v["total_ms"], n, v["avg_ms"]) for n, v in d["kernels"].items()), reverse=True)[:8]:
    print(f"  {n:32s} {a:8.4f} ms avg  {t:9.2f} ms total")
PY
