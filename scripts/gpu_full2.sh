#!/bin/bash
# Full GPU pass for a round milestone: smoke, parity suite, bench lines (c3 default + extra configs),
# rocprofv3 kernel stats of the c3 bench, FETCH_SIZE / WRITE_SIZE PMC passes on the attention kernels.
# usage: gpu_full2.sh TAG "c4 c2"
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r}; EXTRA=${2:-}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=10 \
    > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
[ $rc -le 1 ] || exit $rc
for c in c3 $EXTRA; do
  timeout -k 10 600 python bench.py --config $c > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err
  r=$?; echo "bench $c rc=$r"; tail -c 600 gpurun_out/bench_${TAG}_$c.json; echo; [ $r -eq 0 ] || exit $r
done
R="$GRAFT_REPO_ROOT"; out="$R/gpurun_out/prof_$TAG"; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
args="--steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$out/trace" -o bench -- python3 "$R/bench.py" $args \
    > "$out/trace_bench.json" 2> "$out/trace.err"
r=$?; echo "trace rc=$r"; [ $r -eq 0 ] || exit $r
for ctr in FETCH_SIZE:fetch WRITE_SIZE:write; do
  c=${ctr%%:*}; d=${ctr##*:}
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-include-regex "wattn|mha_|conv3d|mlp_|ln_linear|linear_bwd|token_linear|column_sum" \
      -f csv -d "$out/pmc_$d" -o bench -- python3 "$R/bench.py" $args > "$out/pmc_${d}_bench.json" 2> "$out/pmc_$d.err"
  r=$?; echo "pmc $c rc=$r"; [ $r -eq 0 ] || exit $r
done
exit $rc
