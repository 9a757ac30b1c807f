# final-state check: smoke, GPU pytest, C3 bench (one call)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1
r=$?; echo "smoke rc=$r $(tail -1 gpurun_out/smoke_final.log)"; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_final.log 2>&1
r=$?; echo "pytest rc=$r $(tail -1 gpurun_out/pytest_final.log)"; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
r=$?; python3 -c "import json;d=json.loads(open('gpurun_out/bench_final.json').read().strip().splitlines()[-1]);print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])"; exit $r
