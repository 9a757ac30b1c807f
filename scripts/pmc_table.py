"""Summarise rocprofv3 counter CSVs (gpurun_out/pmc_*/p*/w_counter_collection.csv): mean value of
every counter per kernel (per dispatch).  usage: python scripts/pmc_table.py <dir>"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
agg = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"].split("(")[0][-48:], r["Counter_Name"])].append(float(r["Counter_Value"]))
kern = sorted({k for k, _ in agg})
for k in kern:
    print(k)
    for (kk, c), v in sorted(agg.items()):
        if kk == k:
            print(f"   {c:28s} {sum(v) / len(v):16.4g}")
