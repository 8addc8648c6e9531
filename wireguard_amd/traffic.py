"""Per-launch HBM traffic of the path's kernels, as the bench lines report it
(roofline.traffic): read from the committed profiles/traffic.json, which
scripts/pmc_traffic.py writes from separate rocprofv3 passes.  Round-5
records: reads from the L2's sized read requests (128 x TCC_EA0_RDREQ_128B +
64 x _64B + 32 x _32B, scripts/pmc_sized.py) + WRITE_SIZE x 1024, with the
guide's FETCH_SIZE x 1024 x 2 beside them (read_bytes_fetch_x2; within 1 %
for every kernel, profiles/r5_pmc/).  Bench-side bookkeeping only, not the
data path."""
from __future__ import annotations

import json
import os

TRAFFIC_FILE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                            "traffic.json")


def per_launch(kname: str, algo_bytes: int):
    """HBM bytes per launch of kernel `kname` for a launch of `algo_bytes`
    algorithmic bytes, or None when no matching PMC record is committed."""
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    recs = t.get(kname)
    for rec in (recs if isinstance(recs, list) else [recs]):  # one record per launch size
        if rec and rec.get("algorithmic_bytes") == algo_bytes:
            return rec["hbm_bytes_per_launch"]
    return None
