#!/bin/bash
# One GPU-box session: parity suite (all tests, per-test limit), bench lines for the given configs,
# optional SQ counter passes on the window-attention kernels.  Every GPU step has its own time limit;
# a crash / timeout (anything but pytest's "tests failed" status 1) ends the script.
# usage: gpu_session.sh TAG "c3 c2" [pmc]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-s}; CONFIGS=${2:-c3}; PMC=${3:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=15 \
    > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_$TAG.log
[ $rc -le 1 ] || exit $rc
for c in $CONFIGS; do
  timeout -k 10 600 python bench.py --config $c > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err
  r=$?; echo "bench $c rc=$r"; tail -c 1500 gpurun_out/bench_${TAG}_$c.json; tail -3 gpurun_out/bench_${TAG}_$c.err
  [ $r -eq 0 ] || exit $r
done
if [ -n "$PMC" ]; then
  bash scripts/gpu_pmc_wattn.sh $TAG || exit $?
fi
exit $rc
