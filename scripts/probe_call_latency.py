#!/usr/bin/env python3
"""Median latency of the per-call (host buffer) entry points on one packet /
one Write batch: wgcs_checksum_valid on a 1500-B TCP/IPv4 frame and
wgcs_checksum on 1480 bytes, next to the C oracle (checker) for the same call.
Prints one JSON line."""
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import oracle  # noqa: E402  (checker / CPU timing only)
from wireguard_amd import synth  # noqa: E402
from wireguard_amd.tun import Device  # noqa: E402


def med(fn, reps=300):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e6


dev = Device(0)
arena, pkts, _ = synth.make_batch(1, 1500, kinds="tcp4")
pk = arena[:1500].copy()
L, h = dev.lib, dev.h
v = C.c_int(0)
out = C.c_uint16(0)
for _ in range(20):
    L.wgcs_checksum_valid(h, pk.ctypes.data, 1500, 20, 6, 0, C.byref(v))
assert v.value == 1
res = {
    "checksum_valid_us": round(med(lambda: L.wgcs_checksum_valid(h, pk.ctypes.data, 1500, 20, 6, 0, C.byref(v))), 1),
    "checksum_us": round(med(lambda: L.wgcs_checksum(h, pk[20:].ctypes.data, 1480, 0, C.byref(out))), 1),
}
OL = oracle.lib()
if hasattr(OL, "or_checksum_valid"):
    res["oracle_checksum_valid_us"] = round(med(lambda: OL.or_checksum_valid(pk.ctypes.data, 1500, 20, 6, 0)), 2)
print(json.dumps(res), flush=True)
dev.close()
