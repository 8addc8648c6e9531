"""Per-launch HBM traffic of the path's kernels from rocprofv3 PMC passes.

usage: python scripts/pmc_traffic.py FETCH_DIR WRITE_DIR ALGO_BYTES [KERNEL_SUBSTR] [out.json]
       [FETCH_PER_BYTE]

FETCH_DIR / WRITE_DIR: `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE`
output directories of the same bench command (separate passes: FETCH_SIZE
costs 3 TCC slots, WRITE_SIZE 2; MI355X_MICROARCH.md §rocprofv3 PMC slots).
Correction per the guide (§HBM): FETCH_SIZE is in KiB and reads exactly 1/2
of a wide coalesced stream's bytes on gfx950, so hbm_read = FETCH_SIZE x 1024
x 2; hbm_write = WRITE_SIZE x 1024.  KERNEL_SUBSTR (default
checksum_batch_kernel) picks the kernel; its record is merged into
profiles/traffic.json under the name the bench line reports
(wireguard_amd/traffic.py reads it back).
FETCH_PER_BYTE (default 0.5, the guide's wide-stream value) is what
FETCH_SIZE x 1024 reports per byte read in the kernel's own access pattern,
calibrated on a known byte count (scripts/probe_fetch_cal.py): 0.539 for
gro_batch_kernel's 16-lane rows over packets 64 KiB apart
(profiles/r4_probe_fetch_cal.json).  read = FETCH_SIZE x 1024 / FETCH_PER_BYTE.
"""
import csv
import glob
import json
import os
import re
import statistics
import sys


def counter(d, name, sub):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name and sub in r["Kernel_Name"]:
                vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return vals


def bench_key(k):
    """The kernel name as bench.py / gso_bench / udp_bench report it."""
    m = re.search(r"checksum_batch_kernel<(\d+), (\d+), (\d+), (true|false)", k)
    if m:
        mode = {"2": "VALIDATE", "1": "L4_FILL"}.get(m.group(1), m.group(1))
        return f"checksum_batch_kernel<{mode},{m.group(2)},{m.group(3)},{'nt' if m.group(4) == 'true' else 'rt'}>"
    m = re.search(r"gso_lds_kernel<(\d+), (\d+), (true|false)(?:, (\d+))?>", k)
    if m:  # round 5 added a fourth argument, parts per job (1: named as before)
        p = m.group(4) if m.group(4) and m.group(4) != "1" else None
        return f"gso_lds_kernel<{m.group(1)},{m.group(2)},{m.group(3)}" + (f",{p}>" if p else ">")
    m = re.search(r"gso_rows_kernel<(\d+), (true|false)(?:, (\d+))?>", k)
    if m:  # round 1 / early round 2 had a third template argument (block waves)
        return f"gso_rows_kernel<{m.group(1)},{m.group(2)}" + (f",{m.group(3)}>" if m.group(3) else ">")
    if "gro_batch_kernel" in k:
        return "gro_batch_kernel"
    m = re.search(r"udp_split_kernel<(\d+)>", k)
    if m:
        return f"udp_split_kernel<{m.group(1)}>"
    m = re.search(r"udp_coalesce_kernel<(\d+), (\d+)>", k)
    if m:
        return f"udp_coalesce_kernel<{m.group(1)},{m.group(2)}>"
    return k


def main():
    fdir, wdir, algo = sys.argv[1], sys.argv[2], int(sys.argv[3])
    sub = sys.argv[4] if len(sys.argv) > 4 else "checksum_batch_kernel"
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "profiles", "traffic.json")
    fpb = sys.argv[6] if len(sys.argv) > 6 else "0.5"
    if fpb.startswith("sized:"):
        return main_sized(fdir, wdir, fpb[len("sized:"):], algo, sub, out)
    fpb = float(fpb)
    fs, ws = counter(fdir, "FETCH_SIZE", sub), counter(wdir, "WRITE_SIZE", sub)
    try:
        with open(out) as f:
            res = json.load(f)
    except (OSError, ValueError):
        res = {}
    new = {}
    for k, v in fs.items():
        rd = statistics.median(v) * 1024 / fpb
        wr = statistics.median(ws.get(k, [0.0])) * 1024
        rec = {"hbm_bytes_per_launch": int(rd + wr), "read_bytes": int(rd), "write_bytes": int(wr),
               "algorithmic_bytes": algo, "launches": len(v), "kernel": k,
               "method": (f"median FETCH_SIZE x1024 / {fpb} (FETCH per byte of this access pattern"
                          + (", calibrated: profiles/r4_probe_fetch_cal.json" if fpb != 0.5 else
                             ", the guide's gfx950 wide-stream half-count") + ") + WRITE_SIZE x1024, separate passes"),
               "source_dirs": [fdir, wdir]}
        if fpb != 0.5:
            rec["read_bytes_wide_stream_correction"] = int(statistics.median(v) * 1024 * 2)
        key = bench_key(k)
        # one record per (kernel, launch size): a list once a kernel has several
        old = res.get(key)
        old = old if isinstance(old, list) else ([old] if old else [])
        old = [r for r in old if r.get("algorithmic_bytes") != algo] + [rec]
        res[key] = old[0] if len(old) == 1 else old
        new[key] = rec
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(new, indent=1))


def main_sized(fdir, wdir, sdir, algo, sub, out):
    """Round 5: read bytes from the L2's sized read requests (SIZED_DIR: a
    `--pmc TCC_EA0_RDREQ{,_128B,_64B,_32B}_sum` pass, scripts/pmc_sized.py:
    128 x RDREQ_128B + 64 x RDREQ_64B + 32 x RDREQ_32B, no per-pattern
    factor; checked against known byte counts, profiles/r5_probe_fetch_cal_sized.json)
    + WRITE_SIZE x 1024; the guide's FETCH_SIZE x 1024 x 2 beside it.
    usage: pmc_traffic.py FETCH_DIR WRITE_DIR ALGO KERNEL OUT sized:SIZED_DIR"""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import pmc_sized

    fs, ws = counter(fdir, "FETCH_SIZE", sub), counter(wdir, "WRITE_SIZE", sub)
    sized = {k: pmc_sized.summary(v) for k, v in pmc_sized.collect(sdir, sub).items()}
    try:
        with open(out) as f:
            res = json.load(f)
    except (OSError, ValueError):
        res = {}
    new = {}
    for k, sz in sized.items():
        rd = sz["read_bytes"]
        wr = statistics.median(ws.get(k, [0.0])) * 1024
        rec = {"hbm_bytes_per_launch": int(rd + wr), "read_bytes": int(rd), "write_bytes": int(wr),
               "algorithmic_bytes": algo, "launches": sz["launches"], "kernel": k,
               "method": "L2 sized read requests (128 x RDREQ_128B + 64 x RDREQ_64B + 32 x RDREQ_32B, median per "
                         "launch; scripts/pmc_sized.py) + WRITE_SIZE x1024, separate passes",
               "read_bytes_fetch_x2": int(statistics.median(fs.get(k, [0.0])) * 2048) if k in fs else None,
               "source_dirs": [sdir, wdir, fdir]}
        key = bench_key(k)
        old = res.get(key)
        old = old if isinstance(old, list) else ([old] if old else [])
        old = [r for r in old if r.get("algorithmic_bytes") != algo] + [rec]
        res[key] = old[0] if len(old) == 1 else old
        new[key] = rec
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(new, indent=1))


if __name__ == "__main__":
    main()
