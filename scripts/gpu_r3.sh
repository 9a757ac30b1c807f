#!/bin/bash
# Round-3 GPU session.  Steps: the new / changed parity tests (verbose), the whole GPU suite, smoke,
# an A/B of the window-attention micro-benchmark against build/base.so (if present), the C3 bench
# line, a rocprof kernel-stats pass of C4 (eager).  Test failures are reported and the session goes
# on; a crash, abort or time-out (rc 124/134/137/139 or >128) ends it there.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r3}
STEPS=${2:-new,suite,smoke,ab,bench,profc4}
fatal() { [ "$1" -ge 124 ]; }
has() { [[ ",$STEPS," == *",$1,"* ]]; }
NEW=${NEW:-tests/test_configs_gpu.py tests/test_fullsize_gpu.py tests/test_kernels_gpu.py::test_swin_v2_attention_grads_are_deterministic tests/test_kernels_gpu.py::test_window_attention_grads_are_deterministic}
if has new; then
  timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread $NEW > gpurun_out/pytest_new_$TAG.log 2>&1
  rc=$?; echo "new tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|parity|C5|C1|2\^23|passed|failed|Error" gpurun_out/pytest_new_$TAG.log | tail -40
  fatal $rc && exit $rc
fi
if has suite; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu_$TAG.log | head; tail -3 gpurun_out/pytest_gpu_$TAG.log
  fatal $rc && exit $rc
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_$TAG.log
  fatal $rc && exit $rc
fi
if has ab && [ -f build/base.so ]; then
  for i in 1 2; do
    for lib in build/base.so ""; do
      MMNI_LIB=$lib timeout -k 10 120 python3 scripts/bench_wattn.py 10 > gpurun_out/ab_$TAG.json 2>&1
      r=$?; echo "${lib:-new} rc=$r $(tail -1 gpurun_out/ab_$TAG.json | cut -c1-400)"; fatal $r && exit $r
    done
  done
fi
if has encb; then
  timeout -k 10 300 python3 scripts/bench_encoder.py 20 > gpurun_out/encb_$TAG.json 2> gpurun_out/encb_$TAG.err
  rc=$?; echo "encoder bench rc=$rc"; cut -c1-150 gpurun_out/encb_$TAG.json; tail -2 gpurun_out/encb_$TAG.err
  fatal $rc && exit $rc
fi
if has bench; then
  timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; echo "bench rc=$rc"; python3 -c "
import json,sys; d=json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_ms'], d['roofline']['frac'])
k=sorted(d['kernels'].items(), key=lambda kv: -kv[1]['total_ms'])[:8]; print(k)" ; tail -2 gpurun_out/bench_$TAG.err
  fatal $rc && exit $rc
fi
if has benchc4; then
  timeout -k 10 600 python bench.py --config c4 --steps 10 --warmup 3 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err
  rc=$?; echo "bench c4 rc=$rc"; python3 -c "
import json; d=json.loads(open('gpurun_out/bench_c4_$TAG.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['config'].get('graph'), d['roofline']['kernel'], d['roofline']['avg_ms'])" ; tail -2 gpurun_out/bench_c4_$TAG.err
  fatal $rc && exit $rc
fi
if has benchc5; then
  timeout -k 10 600 python bench.py --config c5 --steps 10 --warmup 3 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err
  rc=$?; echo "bench c5 rc=$rc"; python3 -c "
import json; d=json.loads(open('gpurun_out/bench_c5_$TAG.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_ms'])" ; tail -2 gpurun_out/bench_c5_$TAG.err
  fatal $rc && exit $rc
fi
for c in c2 c3 c5; do
  if has bench$c; then
    timeout -k 10 600 python bench.py --config $c --steps 20 --warmup 5 > gpurun_out/bench_${c}_$TAG.json 2> gpurun_out/bench_${c}_$TAG.err
    rc=$?; echo "bench $c rc=$rc"; tail -1 gpurun_out/bench_${c}_$TAG.json | cut -c1-600; tail -2 gpurun_out/bench_${c}_$TAG.err
    fatal $rc && exit $rc
  fi
  if has prof$c; then
    R="$GRAFT_REPO_ROOT"
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof_${c}_$TAG" -o k -- \
        python3 "$R/bench.py" --config $c --no-cpu-baseline --steps 20 --warmup 5 > "$R/gpurun_out/prof_${c}_$TAG.json" 2> "$R/gpurun_out/prof_${c}_$TAG.err" )
    rc=$?; echo "prof $c rc=$rc"; fatal $rc && exit $rc
    f=$(find gpurun_out/prof_${c}_$TAG -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -c1-200
  fi
done
if has profc4; then
  R="$GRAFT_REPO_ROOT"
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof_c4_$TAG" -o k -- \
      python3 "$R/bench.py" --config c4 --eager --no-cpu-baseline --steps 3 --warmup 2 > "$R/gpurun_out/prof_c4_$TAG.json" 2> "$R/gpurun_out/prof_c4_$TAG.err" )
  rc=$?; echo "prof c4 rc=$rc"; fatal $rc && exit $rc
  f=$(find gpurun_out/prof_c4_$TAG -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -c1-200
fi
exit 0
