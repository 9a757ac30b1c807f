#!/bin/bash
# Window-attention parity tests, the micro-benchmark for the main library and any variants given,
# then a rocprofv3 kernel-stats pass of the main library.  usage: gpu_wattn_prof.sh TAG [variant.so ...]
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 1
TAG=$1; shift
bash scripts/gpu_wattn.sh "$TAG" || exit $?
[ $# -gt 0 ] && { bash scripts/gpu_abl.sh "$@" || exit $?; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof_$TAG" -o w -- \
    python3 "$R/scripts/bench_wattn.py" 5 > "$R/gpurun_out/prof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
f=$(ls "$R"/gpurun_out/prof_$TAG/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && cut -d, -f1-4 "$f" | head -8
exit $rc
