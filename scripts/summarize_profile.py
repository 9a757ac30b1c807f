"""Turn a gpurun_out/prof_<tag> rocprofv3 directory into committed evidence under profiles/:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_pmc.json           per-kernel HBM bytes per launch from the FETCH_SIZE / WRITE_SIZE
                                    passes, corrected as MI355X_MICROARCH.md §HBM prescribes:
                                    bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE
                                    reads half of a wide coalesced stream)
  profiles/<tag>_profile.md         top kernels table
usage: python scripts/summarize_profile.py <tag>
"""
import collections
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench_key(name):
    """rocprof kernel name -> bench.py KernelTimer prefix (e.g. wattn_bwd_k0_C12)."""
    m = re.search(r"mmni::(wattn_(?:fwd|bwd))_kernel<(\d+), (\d+), (\d), \d+>", name)
    if m:
        return f"{m.group(1)}_k{m.group(4)}_C{m.group(2)}"
    m = re.search(r"mmni::(wattn_(?:fwd|bwd))_pk2?_kernel<(\d+), (\d), \d+>", name)
    if m:
        return f"{m.group(1)}_k{m.group(3)}_C{m.group(2)}"
    m = re.search(r"mmni::wattn_bwd[AB]_bc_kernel<6, 6, 6>|mmni::wattn_bwd[AB]_q4_kernel|mmni::wattn_bwd_q4m_kernel|mmni::wattn_bwd_q4k_kernel", name)
    if m:   # kind 0, C = 12, 6^3 windows: the merged backward (older rounds: passes A + B) = one call
        return "wattn_bwd_k0_C12"
    m = re.search(r"mmni::(mha_\w+?)_kernel<(\d+)>", name)
    if m:
        return f"{m.group(1)}_hd{m.group(2)}"
    m = re.search(r"mmni::(conv3d_\w+?)_kernel<(\d+), (\d+)", name)
    if m:
        return f"{m.group(1)}_{m.group(2)}x{m.group(3)}"
    m = re.search(r"mmni::(layernorm_(?:fwd|bwd))_kernel<(\d+)>", name)
    if m:
        return f"{m.group(1)}_C{m.group(2)}"
    m = re.search(r"mmni::linear_dw_kernel<(\d+), (\d+)>", name)
    if m:
        return f"linear_dw_tiles{m.group(1)}x{m.group(2)}"
    m = re.search(r"mmni::mlpk::(mlp_fwd|mlp_bwd)_kernel<(true|false)>", name)
    if m:
        return f"{'ln_' if m.group(2) == 'true' else ''}{m.group(1)}_12x48"
    m = re.search(r"mmni::mlpk::(mlp_fwd|mlp_bwd)_kernel", name)
    if m:
        return f"{m.group(1)}_12x48"
    m = re.search(r"mmni::blk::(ln_linear_fwd|ln_linear_bwd)_kernel<(\d+)>", name)
    if m:
        return f"{m.group(1)}_12x{m.group(2)}"
    m = re.search(r"mmni::blk::linear_bwd_kernel", name)
    if m:
        return "linear_bwd_12x12"
    m = re.search(r"mmni::token_linear_kernel<(\d+), (\d+), (\d), \d+>", name)
    if m:
        return f"token_linear_e{m.group(3)}_{m.group(1)}x{m.group(2)}"
    m = re.search(r"mmni::(wattn_absmax|wattn_dtable_convert|column_sum)_kernel", name)
    if m:
        return m.group(1)
    return None


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "bench_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"# rocprofv3 kernel stats ({tag})", "", f"total kernel time {total / 1e6:.1f} ms", "",
             "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
        lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.1f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
    pmc = {}
    for ctr, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write")):
        path = os.path.join(src, sub, "bench_counter_collection.csv")
        if not os.path.exists(path):
            continue
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] == ctr:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            pmc.setdefault(k, {})[ctr] = sum(v) / len(v)
            pmc[k]["launches"] = len(v)
    kernels = {}
    for name, d in pmc.items():
        key = bench_key(name) or name
        f, w = d.get("FETCH_SIZE"), d.get("WRITE_SIZE")
        hbm = (2 * f + w) * 1024 if f is not None and w is not None else None
        if key in kernels and hbm is not None and kernels[key]["hbm_bytes_per_launch"] is not None:
            # several kernels make one call (the row-broadcast backward's passes A and B): bytes add
            k = kernels[key]
            k["rocprof_name"] += " + " + name
            k["fetch_kb"] += f
            k["write_kb"] += w
            k["hbm_bytes_per_launch"] += hbm
            continue
        kernels[key] = dict(rocprof_name=name, fetch_kb=f, write_kb=w, hbm_bytes_per_launch=hbm,
                            launches=d.get("launches"))
    json.dump(dict(tag=tag, correction="bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 (MI355X_MICROARCH.md §HBM)",
                   kernels=kernels), open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
    lines += ["", "## HBM traffic per launch (PMC, corrected)", "", "| kernel | MB/launch |", "|---|---|"]
    for k, v in sorted(kernels.items(), key=lambda kv: -(kv[1]["hbm_bytes_per_launch"] or 0)):
        if v["hbm_bytes_per_launch"]:
            lines.append(f"| {k} | {v['hbm_bytes_per_launch'] / 1e6:.1f} |")
    open(os.path.join(dst, f"{tag}_profile.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:20]))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
