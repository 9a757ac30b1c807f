#!/bin/bash
# rocprof kernel stats of one bench config (graph mode optional): gpu_prof_cfg.sh TAG CONFIG [bench args]
tag=$1; cfg=$2; shift 2
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof_$tag" -o k -- \
    python3 "$R/bench.py" --config $cfg --no-cpu-baseline "$@" > "$R/gpurun_out/prof_$tag.json" 2> "$R/gpurun_out/prof_$tag.err"
r=$?; echo "rc=$r"; tail -c 300 "$R/gpurun_out/prof_$tag.json"; exit $r
