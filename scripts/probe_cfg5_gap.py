"""Why configs[4] (cfg5: 1 M mixed frames) runs at ~0.72 of 8 TB/s while cfg2
(64 k TCP4 frames) reaches ~0.88 and a flat read of cfg5's bytes 0.845
(profiles/r5_probe_flat_stream3.jsonl).  NOT product code: the product kernel
on batches that differ in one factor at a time -- batch size, rotation depth
(how much of the rotating set the 256 MiB Infinity Cache can hold), frame mix.
One JSON line per case."""
import json
import os
import sys

import numpy as np
import torch  # first: one HIP runtime per process

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wireguard_amd import synth  # noqa: E402
from wireguard_amd.tun import MODE_VALIDATE, Device  # noqa: E402

dev = Device(0)
torch.cuda.set_device(0)
CASES = [  # (frames, kinds, rotated copies)
    (65536, "tcp4", 4), (65536, "tcp4", 32), (65536, "mixed", 4), (65536, "mixed", 32),
    (1048576, "tcp4", 2), (1048576, "mixed", 2), (262144, "mixed", 8), (262144, "mixed", 2),
]
if os.environ.get("GAP_CASES"):  # e.g. "1048576:mixed:2,1048576:mixed:4"
    CASES = [(int(a), k, int(r)) for a, k, r in (c.split(":") for c in os.environ["GAP_CASES"].split(","))]
for n, kinds, R in CASES:
    arena_np, pkts_np, _ = synth.make_batch(n, 1500, kinds=kinds, seed=synth.SEED)
    nbytes = int(pkts_np["len"].astype(np.int64).sum())
    arenas = [torch.from_numpy(arena_np).to("cuda") for _ in range(R)]
    pkts = torch.from_numpy(pkts_np.view(np.uint8)).to("cuda")
    outs = [torch.empty(n * 2, dtype=torch.uint8, device="cuda") for _ in range(R)]
    strm = [torch.cuda.Stream(), torch.cuda.Stream()]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(strm[0])
    e1.record(strm[0])
    K = max(8, min(200, int(3e9 // nbytes)))
    for ns in (1, 2):
        def run(K):
            bl = dev.batch_list([(arenas[k % R], pkts, n, outs[k % R]) for k in range(K)])
            torch.cuda.synchronize()
            dev.checksum_batches(MODE_VALIDATE, bl, strm[:ns], e0, e1)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3 / K
        run(4)
        us = min(run(K) for _ in range(3))
        print(json.dumps({"frames": n, "kinds": kinds, "rotate": R, "rotating_MB": round(R * nbytes / 1e6),
                          "streams": ns, "launches": K, "us_per_launch": round(us, 2),
                          "frac_of_8TBps": round(nbytes / us / 1e3 / 8000, 4)}), flush=True)
    del arenas, outs, pkts
    torch.cuda.empty_cache()
