import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests")); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import numpy as np, torch
import oracle
from wireguard_amd import synth
from wireguard_amd.tun import Device
dev = Device(0)
for (total, gso, v6, udp) in [(65535, 1460, False, False), (65535, 1460, True, False), (1500, 1460, False, False)]:
    vp = synth.make_super_packet(total, gso, seed=total + gso, v6=v6, udp=udp)
    rb_o = np.frombuffer(bytearray(vp), dtype=np.uint8).copy(); rb_p = rb_o.copy()
    bo = [np.full(65535, 0xA5, np.uint8) for _ in range(128)]; bp = [b.copy() for b in bo]
    rc_o, n_o, sz_o = oracle.handle_virtio_read(rb_o, bo, 16)
    sz_p = [0] * 128
    n_p, err = dev.handle_virtio_read(rb_p, bp, sz_p, 16)
    print("case", total, gso, v6, udp, "n", n_o, n_p, "err", rc_o, err)
    bad = 0
    for i in range(n_o):
        d = np.nonzero(bp[i] != bo[i])[0]
        if len(d):
            bad += 1
            if bad <= 4:
                print(" seg", i, "size", sz_o[i], sz_p[i], "diff at", d[:12].tolist(), "n", len(d), "got", bp[i][d[:6]].tolist(), "want", bo[i][d[:6]].tolist())
    print(" bad segments", bad)
dev.close()
