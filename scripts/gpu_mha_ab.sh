cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r3i}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_golden_gpu.py -k "mha or MHA or cross or Transformer" > gpurun_out/pytest_mha_$TAG.log 2>&1; rc=$?; echo "mha tests rc=$rc"; tail -2 gpurun_out/pytest_mha_$TAG.log; [ $rc -ge 124 ] && exit $rc
for i in 1 2; do for lib in build/mha_old.so ""; do
  MMNI_LIB=$lib timeout -k 10 180 python3 scripts/bench_mha.py 5 > gpurun_out/mha_ab_$TAG.txt 2>&1; r=$?; echo "${lib:-new} rc=$r"; python3 scripts/mha_ab_line.py gpurun_out/mha_ab_$TAG.txt; [ $r -ge 124 ] && exit $r
done; done
timeout -k 10 300 bash scripts/gpu_prof_sq.sh mhab "mha_bwd_mfma" scripts/bench_mha.py 3 4096:84:bfloat16 | tail -40
exit 0
