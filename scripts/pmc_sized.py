"""HBM read bytes from the L2's sized memory-side read requests (NOT product
code): rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum
TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum (4 TCC slots, one pass).

rocprofv3's FETCH_SIZE is (BUBBLE x 128 + (RDREQ - BUBBLE - RDREQ_32B) x 64 +
RDREQ_32B x 32) / 1024 (its --list-avail expression): on gfx950 it tallies
128-byte requests at 64 bytes, which is why MI355X_MICROARCH.md calls it half
the bytes of a wide stream and leaves other access widths uncalibrated.  The
sized counters count each request once at its size, so
    read_bytes = 128 x RDREQ_128B + 64 x RDREQ_64B + 32 x RDREQ_32B
needs no per-pattern factor.  scripts/probe_fetch_cal.py checks it against
known byte counts (a wide stream and isolated rows 64 KiB apart: the bytes of
the 128-byte lines the rows touch).

usage: pmc_sized.py PMC_DIR [KERNEL_SUBSTR] -> one JSON line per kernel:
  median per launch of each counter, read_bytes, and the unsized remainder
  RDREQ - (128B + 64B + 32B) (0 when every request has one of the sizes).
       pmc_sized.py cal PMC_DIR PROBE_LOG -> the calibration probe's ratios."""
import csv
import glob
import json
import os
import statistics
import sys

NAMES = ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_32B_sum")


def collect(d, sub=""):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub not in r["Kernel_Name"] or r["Counter_Name"] not in NAMES:
                continue
            k = (r["Kernel_Name"], int(r["Dispatch_Id"]))
            per.setdefault(k, {})[r["Counter_Name"]] = per.get(k, {}).get(r["Counter_Name"], 0.0) + float(
                r["Counter_Value"])
    by_kernel = {}
    for (name, disp), c in sorted(per.items(), key=lambda kv: kv[0][1]):
        by_kernel.setdefault(name, []).append((disp, c))
    return by_kernel


def summary(launches):
    med = {n: statistics.median(c.get(n, 0.0) for _, c in launches) for n in NAMES}
    rd = 128 * med["TCC_EA0_RDREQ_128B_sum"] + 64 * med["TCC_EA0_RDREQ_64B_sum"] + 32 * med["TCC_EA0_RDREQ_32B_sum"]
    return {"launches": len(launches), **{n: med[n] for n in NAMES}, "read_bytes": int(rd),
            "unsized_requests": med["TCC_EA0_RDREQ_sum"] - med["TCC_EA0_RDREQ_128B_sum"] - med["TCC_EA0_RDREQ_64B_sum"]
            - med["TCC_EA0_RDREQ_32B_sum"]}


def cal(d, log):
    """scripts/probe_fetch_cal.py's launches (5 wide, then 5 per row pattern,
    in launch order): sized read bytes over the known byte counts."""
    rec = json.loads([l for l in open(log) if l.startswith("{")][-1])
    by = collect(d)
    wide = [c for name, ls in by.items() if "cal_wide" in name for _, c in ls]
    rows = sorted([(disp, c) for name, ls in by.items() if "cal_rows" in name for disp, c in ls])
    out = {"wide": {**summary([(0, c) for c in wide[1:]]), "bytes": rec["wide_bytes"]}, "rows": {}}
    out["wide"]["read_over_bytes"] = round(out["wide"]["read_bytes"] / rec["wide_bytes"], 4)
    for k, (key, b) in enumerate(rec["rows"].items()):
        s = summary(rows[5 * k + 1: 5 * k + 5])
        s.update({kk: b[kk] for kk in b})
        s["read_over_len"] = round(s["read_bytes"] / b["len_bytes"], 4)
        if "line128_bytes" in b:
            s["read_over_line128"] = round(s["read_bytes"] / b["line128_bytes"], 4)
            s["read_over_line64"] = round(s["read_bytes"] / b["line64_bytes"], 4)
        out["rows"][key] = s
    print(json.dumps(out))


def main():
    if sys.argv[1] == "cal":
        return cal(sys.argv[2], sys.argv[3])
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, launches in collect(d, sub).items():
        print(json.dumps({"kernel": name, **summary(launches)}))


if __name__ == "__main__":
    main()
