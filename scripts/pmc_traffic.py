"""Per-launch HBM traffic of the checksum kernel from rocprofv3 PMC passes.

usage: python scripts/pmc_traffic.py FETCH_DIR WRITE_DIR ALGO_BYTES [out.json]

FETCH_DIR / WRITE_DIR: `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE`
output directories (separate passes: FETCH_SIZE costs 3 TCC slots, WRITE_SIZE
2; MI355X_MICROARCH.md §rocprofv3 PMC slots).  Correction per the guide
(§HBM): FETCH_SIZE is in KiB and reads exactly 1/2 of a wide coalesced
stream's bytes on gfx950, so hbm_read = FETCH_SIZE x 1024 x 2;
hbm_write = WRITE_SIZE x 1024.  Writes profiles/traffic.json, which bench.py
reports as roofline.traffic.
"""
import csv
import glob
import json
import os
import re
import statistics
import sys


def counter(d, name):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name and "checksum_batch_kernel" in r["Kernel_Name"]:
                vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return vals


def main():
    fdir, wdir, algo = sys.argv[1], sys.argv[2], int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "profiles", "traffic.json")
    fs, ws = counter(fdir, "FETCH_SIZE"), counter(wdir, "WRITE_SIZE")
    res = {}
    for k, v in fs.items():
        targs = re.search(r"checksum_batch_kernel<(\d+), (\d+), (\d+), (true|false)>", k)
        mode = {"2": "VALIDATE", "1": "L4_FILL"}.get(targs.group(1), targs.group(1))
        key = f"checksum_batch_kernel<{mode},{targs.group(2)},{targs.group(3)},{'nt' if targs.group(4) == 'true' else 'rt'}>"
        rd = statistics.median(v) * 1024 * 2
        wr = statistics.median(ws.get(k, [0.0])) * 1024
        res[key] = {"hbm_bytes_per_launch": int(rd + wr), "read_bytes": int(rd), "write_bytes": int(wr),
                    "algorithmic_bytes": algo, "launches": len(v), "kernel": k,
                    "method": "median FETCH_SIZE x1024 x2 (gfx950 half-count) + WRITE_SIZE x1024, separate passes",
                    "source_dirs": [fdir, wdir]}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
