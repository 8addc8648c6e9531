#!/usr/bin/env python3
"""Per-call latency at the reference's call granularity (NOT product code;
VERDICT r5 item 4): one checksumValid of a 1500-B TCP/IPv4 frame and one
handleVirtioRead of a 65,535-B TSO read into 64 buffers of 2,048 B, through
  - the per-call entry points (a kernel launch + completion wait per call),
  - the resident ring (wgcs_ring_*), with the request bytes in ordinary memory
    (copied into the ring's staging) and in wgcs_host_alloc memory (read in
    place, as a Go caller with a pinned readBuf would),
  - the C oracle (the CPU restatement of the Go code, one core, via ctypes:
    ~0.3 us of call overhead included).
Median over `reps` calls after a warmup; every result is checked once
against the oracle.  Prints one JSON line."""
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
from wireguard_amd.tun import Device, Ring  # noqa: E402

REPS = int(os.environ.get("REPS", "400"))


def med(fn, reps=REPS, warm=30):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return {"median_us": round(statistics.median(ts) * 1e6, 2), "p10_us": round(ts[len(ts) // 10] * 1e6, 2),
            "p90_us": round(ts[len(ts) * 9 // 10] * 1e6, 2)}


dev = Device(0)
ring = Ring(dev, idle_us=1_000_000)
L, h, rh = dev.lib, dev.h, ring.h
OL = oracle.lib()
res = {"probe": "ring_calls", "reps": REPS}

# ---- checksumValid, 1500-B TCP/IPv4
arena, pkts, _ = synth.make_batch(1, 1500, kinds="tcp4")
pk = arena[:1500].copy()
ppk = dev.host_alloc(1536)
ppk[:1500] = pk
v = C.c_int(0)
SKIP_CS = os.environ.get("PROBE_SKIP_CS") == "1"  # virtio reads only (no inline requests before them)
assert SKIP_CS or ring.checksum_valid(pk, 20, 6, False) and ring.checksum_valid(ppk[:1500], 20, 6, False)
res["checksum_valid"] = {} if SKIP_CS else {
    "per_call_launch": med(lambda: L.wgcs_checksum_valid(h, pk.ctypes.data, 1500, 20, 6, 0, C.byref(v))),
    "ring_copied": med(lambda: L.wgcs_ring_checksum_valid(rh, pk.ctypes.data, 1500, 20, 6, 0, C.byref(v))),
    "ring_pinned": med(lambda: L.wgcs_ring_checksum_valid(rh, ppk.ctypes.data, 1500, 20, 6, 0, C.byref(v))),
    "oracle_1core": med(lambda: OL.or_checksum_valid(pk.ctypes.data, 1500, 20, 6, 0)),
}

# ---- handleVirtioRead, 65,535-B TSO read (45 segments of MSS 1460) into 64 x 2,048-B buffers
vp = synth.make_super_packet(65535, 1460)
n = len(vp)
rb = np.frombuffer(bytearray(vp), np.uint8).copy()
prb = dev.host_alloc(n + 64)
prb[:n] = rb
nb, bsz, off = 64, 2048, 16
bufs = [np.zeros(bsz, np.uint8) for _ in range(nb)]
u8p = C.POINTER(C.c_uint8)
arr = (u8p * nb)(*[C.cast(b.ctypes.data, u8p) for b in bufs])
lens = (C.c_size_t * nb)(*[bsz] * nb)
sizes = (C.c_int * nb)()
cnt = C.c_int(0)

# one checked call of each transport (the readBuf edits are idempotent for a split)
for fn in ("wgcs_handle_virtio_read",):
    rbo = rb.copy()
    bo = [np.zeros(bsz, np.uint8) for _ in range(nb)]
    rc_o, n_o, sz_o = oracle.handle_virtio_read(rbo, bo, off)
    for tag, call in (("per_call", lambda: L.wgcs_handle_virtio_read(h, rb.ctypes.data, n, arr, lens, nb, sizes, off,
                                                                     C.byref(cnt))),
                      ("ring_pinned", lambda: L.wgcs_ring_handle_virtio_read(rh, prb.ctypes.data, n, arr, lens, nb,
                                                                             sizes, off, C.byref(cnt)))):
        for b in bufs:
            b[:] = 0
        rc = call()
        assert rc == rc_o and cnt.value == n_o and list(sizes)[:n_o] == sz_o[:n_o], (tag, rc, rc_o)
        assert all(np.array_equal(bufs[i], bo[i]) for i in range(nb)), tag
# the Read buffers as one pinned slab on a fixed stride: segments written in place
slab = dev.host_alloc(nb * bsz)
sarr = (u8p * nb)(*[C.cast(slab.ctypes.data + i * bsz, u8p) for i in range(nb)])
rc = L.wgcs_ring_handle_virtio_read(rh, prb.ctypes.data, n, sarr, lens, nb, sizes, off, C.byref(cnt))
assert rc == 0 and cnt.value == 45
assert all(np.array_equal(slab[i * bsz:(i + 1) * bsz], bo[i]) for i in range(nb))
res["handle_virtio_read"] = {
    "ring_pinned_direct": med(lambda: L.wgcs_ring_handle_virtio_read(rh, prb.ctypes.data, n, sarr, lens, nb, sizes,
                                                                     off, C.byref(cnt))),
    "bytes": n, "segments": 45,
    "per_call_launch": med(lambda: L.wgcs_handle_virtio_read(h, rb.ctypes.data, n, arr, lens, nb, sizes, off,
                                                             C.byref(cnt))),
    "ring_copied": med(lambda: L.wgcs_ring_handle_virtio_read(rh, rb.ctypes.data, n, arr, lens, nb, sizes, off,
                                                              C.byref(cnt))),
    "ring_pinned": med(lambda: L.wgcs_ring_handle_virtio_read(rh, prb.ctypes.data, n, arr, lens, nb, sizes, off,
                                                              C.byref(cnt))),
    "oracle_1core": med(lambda: OL.or_handle_virtio_read_cap(rb.ctypes.data, n, n, arr, lens, nb, sizes, off,
                                                              C.byref(cnt))),
}
res["ring"] = ring.info()
print(json.dumps(res), flush=True)
ring.close()
dev.host_free(ppk)
dev.host_free(prb)
dev.host_free(slab)
dev.close()
