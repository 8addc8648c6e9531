#!/usr/bin/env python3
"""Where a ring request's time goes (NOT product code; round 6, VERDICT r5
item 4).  Run with WGCS_LIB pointing at a -DWGCS_RING_STAMPS build: after
every call, workgroup b's stamps (s_memrealtime, 10-ns ticks from the moment
the workgroup read the request) = {body issued, every wave drained, stores
released, idle before}.  The host's wall latency minus the device span is the
poll's detection time plus the completion's trip back.  Median over REPS
calls; one JSON line per request kind."""
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from wireguard_amd import synth  # noqa: E402
from wireguard_amd.tun import Device, Ring  # noqa: E402

REPS = int(os.environ.get("REPS", "300"))
dev = Device(0)
ring = Ring(dev, idle_us=1_000_000)
L, rh = dev.lib, ring.h
L.wgcs_ring_debug_stamps.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_uint32)]
nb = ring.info().get("blocks", 3)
st = (C.c_uint32 * 4)()


def run(tag, fn):
    for _ in range(30):
        fn()
    wall, per = [], [[] for _ in range(nb)]
    for _ in range(REPS):
        t0 = time.perf_counter()
        fn()
        wall.append((time.perf_counter() - t0) * 1e6)
        for b in range(nb):
            L.wgcs_ring_debug_stamps(rh, b, st)
            per[b].append([x * 0.01 for x in st])  # ticks -> us
    out = {"probe": "ring_stamps", "call": tag, "reps": REPS, "wall_us": round(statistics.median(wall), 2)}
    for b in range(nb):
        cols = list(zip(*per[b]))
        out[f"wg{b}"] = {k: round(statistics.median(c), 2) for k, c in zip(("issued", "drained", "released"), cols)}
    print(json.dumps(out), flush=True)


arena, pkts, _ = synth.make_batch(1, 1500, kinds="tcp4")
ppk = dev.host_alloc(1536)
ppk[:1500] = arena[:1500]
v = C.c_int(0)
run("checksum_valid_pinned", lambda: L.wgcs_ring_checksum_valid(rh, ppk.ctypes.data, 1500, 20, 6, 0, C.byref(v)))

vp = synth.make_super_packet(65535, 1460)
n = len(vp)
prb = dev.host_alloc(n + 64)
prb[:n] = np.frombuffer(bytearray(vp), np.uint8)
nbuf, bsz, off = 64, 2048, 16
slab = dev.host_alloc(nbuf * bsz)
u8p = C.POINTER(C.c_uint8)
sarr = (u8p * nbuf)(*[C.cast(slab.ctypes.data + i * bsz, u8p) for i in range(nbuf)])
lens = (C.c_size_t * nbuf)(*[bsz] * nbuf)
sizes = (C.c_int * nbuf)()
cnt = C.c_int(0)
run("virtio_read_direct", lambda: L.wgcs_ring_handle_virtio_read(rh, prb.ctypes.data, n, sarr, lens, nbuf, sizes, off,
                                                                 C.byref(cnt)))
assert cnt.value == 45
ring.close()
for p in (ppk, prb, slab):
    dev.host_free(p)
dev.close()
