#!/bin/bash
# rocprofv3 evidence for the bench: kernel trace + stats, then PMC passes (FETCH_SIZE and
# WRITE_SIZE in separate passes, MI355X_MICROARCH.md §rocprofv3 PMC slots) on the wattn kernels.
# usage: bash scripts/gpu_profile.sh <tag> [bench args...]
tag=${1:-r01}; shift
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
out="$R/gpurun_out/prof_$tag"
mkdir -p "$out"
args="--steps 2 --warmup 1 --no-cpu-baseline $*"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$out/trace" -o bench -- \
    python3 "$R/bench.py" $args > "$out/trace_bench.json" 2> "$out/trace.err"
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$out/trace.err"; exit $rc; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "wattn|mha_|conv3d|layernorm|linear_dw|column_sum|mlp_|token_linear|blk::" -f csv -d "$out/pmc_fetch" -o bench -- \
    python3 "$R/bench.py" $args > "$out/pmc_fetch_bench.json" 2> "$out/pmc_fetch.err"
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$out/pmc_fetch.err"; exit $rc; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "wattn|mha_|conv3d|layernorm|linear_dw|column_sum|mlp_|token_linear|blk::" -f csv -d "$out/pmc_write" -o bench -- \
    python3 "$R/bench.py" $args > "$out/pmc_write_bench.json" 2> "$out/pmc_write.err"
rc=$?; echo "pmc write rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$out/pmc_write.err"; exit $rc; }
find "$out" -name "*.csv" | head -20
