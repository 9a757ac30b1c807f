#!/bin/bash
# Window-attention parity tests, the micro-benchmark, then FETCH_SIZE / WRITE_SIZE passes on the
# attention kernels of the micro-benchmark.  usage: gpu_wattn_traffic.sh TAG [variant.so ...]
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 1
TAG=$1; shift
bash scripts/gpu_wattn.sh "$TAG" || exit $?
[ $# -gt 0 ] && { bash scripts/gpu_abl.sh "$@" || exit $?; }
mkdir -p "$R/gpurun_out/tr_$TAG"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "wattn_(fwd|bwd)_pk2" -f csv -d "$R/gpurun_out/tr_$TAG/$c" -o w -- \
      python3 "$R/scripts/bench_wattn.py" 2 > "$R/gpurun_out/tr_$TAG/$c.log" 2>&1 || { echo "$c failed"; exit 1; }
done
python3 - "$R/gpurun_out/tr_$TAG" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(k, "%.1f MB" % (sum(v) / len(v) / 1024))
PY
