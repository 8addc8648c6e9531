"""Print the differing byte positions between the GPU GSO split and the oracle
for a handful of super-packets (debug aid, GPU box)."""
import sys

import torch  # noqa: F401  (one HIP runtime per process)
import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "oracle")
import oracle
from wireguard_amd import synth
from wireguard_amd.tun import Device

dev = Device(0)
cases = [(65535, 1460, False, False, 16), (20000, 1460, False, False, 3), (9000, 1, False, False, 16),
         (4001, 1000, True, True, 16), (1500, 1460, False, True, 16)]
for total, gso, v6, udp, off in cases:
    vp = synth.make_super_packet(total, gso, seed=total + gso, v6=v6, udp=udp)
    rb_o = np.frombuffer(bytearray(vp), dtype=np.uint8).copy()
    rb_p = rb_o.copy()
    n = 128
    bo = [np.full(65535, 0xA5, np.uint8) for _ in range(n)]
    bp = [np.full(65535, 0xA5, np.uint8) for _ in range(n)]
    rc_o, n_o, sz_o = oracle.handle_virtio_read(rb_o, bo, off)
    sz_p = [0] * n
    n_p, err = dev.handle_virtio_read(rb_p, bp, sz_p, off)
    print(f"case total={total} gso={gso} v6={v6} udp={udp} off={off}: rc_o={rc_o} n_o={n_o} n_p={n_p} err={err}")
    bad = 0
    for i in range(n):
        d = np.nonzero(bo[i] != bp[i])[0]
        if len(d):
            bad += 1
            if bad <= 4:
                pos = (d - off).tolist()
                print(f"  seg {i} size o={sz_o[i]} p={sz_p[i]}: {len(d)} diffs at pkt pos {pos[:24]}"
                      f" o={bo[i][d[:8]].tolist()} p={bp[i][d[:8]].tolist()}")
    print(f"  {bad} bad segments")
