"""Median per-dispatch value of every PMC counter, per kernel, from rocprofv3
counter_collection CSVs.  usage: python scripts/pmc_summary.py DIR [DIR...]"""
import collections
import csv
import glob
import os
import statistics
import sys

vals = collections.defaultdict(list)
meta = {}
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][-60:]
            vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
            meta[k] = (r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Grid_Size"])
for k in sorted({k for k, _ in vals}):
    print(k, "vgpr/sgpr/lds/grid", meta[k])
    for (kk, c), v in sorted(vals.items()):
        if kk == k:
            print(f"   {c:24s} {statistics.median(v):14.0f}  (n={len(v)})")
