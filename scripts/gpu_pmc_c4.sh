#!/bin/bash
# HBM traffic of the C4 crossmodal-head kernels (encoder row GEMMs, LayerNorm backward, chunk sums,
# MHA split / forward / backward): FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes over one
# eager C4 step, summarised per (kernel, grid) with the gfx950 correction of MI355X_MICROARCH.md
# §HBM (bytes = 2 * FETCH_SIZE + WRITE_SIZE, in KB).  usage: gpu_pmc_c4.sh TAG
R="$GRAFT_REPO_ROOT"
TAG=${1:-c4}
out="$R/gpurun_out/pmc_c4_$TAG"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "enc::|mha_" -f csv -d "$out/$c" -o k -- \
      python3 "$R/bench.py" --config c4 --eager --no-cpu-baseline --steps 1 --warmup 1 > "$out/$c.log" 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$out/$c.log"; exit $rc; }
done
python3 - "$out" > "$out/summary.txt" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{d}/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            key = (r["Kernel_Name"].split("(")[0].replace("void ", "")[-48:], r.get("Grid_Size", r.get("Grid_Size_X", "")))
            agg[key][c].append(float(r["Counter_Value"]))
print(f"{'kernel':50s} {'grid':>8s} {'n':>4s} {'fetch_KB':>10s} {'write_KB':>10s} {'hbm_MB(2F+W)':>13s}")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1].get("FETCH_SIZE", [0]))):
    fk = sum(v["FETCH_SIZE"]) / max(1, len(v["FETCH_SIZE"]))
    wk = sum(v["WRITE_SIZE"]) / max(1, len(v["WRITE_SIZE"]))
    print(f"{k[0]:50s} {k[1]:>8s} {len(v['FETCH_SIZE']):4d} {fk:10.1f} {wk:10.1f} {(2 * fk + wk) / 1024:13.2f}")
PY
cat "$out/summary.txt" | head -60
exit 0
