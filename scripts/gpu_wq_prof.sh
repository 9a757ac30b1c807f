#!/bin/bash
# per-kernel times of the window-attention micro-benchmark for the default and a variant library
# usage: gpu_wq_prof.sh VARIANT_SO [VARIANT_SO ...]
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for lib in "" "$@"; do
  tag=$( [ -z "$lib" ] && echo default || basename "$lib" .so )
  export MMNI_LIB=${lib:+$R/$lib}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/wqp_$tag" -o w -- python3 "$R/scripts/bench_wattn.py" 5 > "$R/gpurun_out/wqp_$tag.json" 2>&1
  r=$?; echo "$tag rc=$r"; [ $r -eq 0 ] || exit $r
  python3 - "$R/gpurun_out/wqp_$tag" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "wattn" in r["Name"] or "column_sum" in r["Name"]:
        print(f'   {r["Name"][:60]:60s} {int(r["Calls"]):5d} {float(r["AverageNs"])/1e3:9.1f} us')
PY
done
