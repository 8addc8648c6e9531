"""Summarise scripts/probe_fetch_cal.py under rocprofv3 --pmc FETCH_SIZE:
FETCH_SIZE x 1024 / requested bytes per kernel (and per row length, in
launch order).  usage: fetch_cal_summary.py PMC_DIR PROBE_LOG"""
import csv
import glob
import json
import os
import statistics
import sys

d, log = sys.argv[1], sys.argv[2]
rec = json.loads([l for l in open(log) if l.startswith("{")][-1])
rows = []
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == "FETCH_SIZE"]
rows.sort(key=lambda r: int(r["Dispatch_Id"]))
wide = [float(r["Counter_Value"]) * 1024 for r in rows if "cal_wide" in r["Kernel_Name"]]
crow = [float(r["Counter_Value"]) * 1024 for r in rows if "cal_rows" in r["Kernel_Name"]]
out = {"wide_ratio": round(statistics.median(wide[1:]) / rec["wide_bytes"], 4), "rows": {}}
for k, (ln, b) in enumerate(rec["rows"].items()):
    v = statistics.median(crow[5 * k + 1: 5 * k + 5])
    out["rows"][ln] = {"fetch_over_span": round(v / b["span_bytes"], 4), "fetch_over_len": round(v / b["len_bytes"], 4)}
print(json.dumps(out))
