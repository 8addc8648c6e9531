"""Generate tests/golden/golden.json -- committed golden vectors for the hot path.

Outputs come from the oracle (oracle/wg_oracle.c, the C restatement of the
reference's tun/checksum.go + tun/gro.go), cross-checked here against the
independent closed form and the RFC 1071 / IPv4-header /
pseudo-header known answers.  The reference itself ships no vectors and cannot
run in this image (Go toolchain absent), so these fixtures pin the oracle
against regressions and let the GPU box check the product without building
anything but the product.  Inputs are seeded (numpy PCG64).

usage: python tests/golden/make_golden.py   (rewrites golden.json)
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
from wireguard_amd import synth  # noqa: E402

SEED = 20261015


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def fold_vectors(rng):
    out = []
    inits = [0, 0xFFFF, 2**64 - 1, 1, 0x1234567890ABCDEF]
    for n in list(range(0, 66)) + [127, 128, 129, 255, 256, 257, 1023, 1500]:
        for pat in ("rand", "zero", "ff"):
            b = {"rand": rng.integers(0, 256, n, dtype=np.uint8).tobytes(), "zero": b"\0" * n, "ff": b"\xff" * n}[pat]
            ini = inits[(n + len(pat)) % len(inits)]
            c = oracle.checksum(b, ini)
            assert c == oracle.closed_form_checksum(b, ini)
            out.append({"hex": b.hex(), "init": hex(ini), "checksum": c, "nofold": hex(oracle.checksum_nofold(b, ini))})
    return out


def rows(p):
    """wgcs_pkt rows as [off, len, csum_start, csum_offset, proto, flags]."""
    off = synth.pkt_off(p)
    return [[int(off[i]), int(x["len"]), int(x["csum_start"]), int(x["csum_offset"]), int(x["proto"]), int(x["flags"])]
            for i, x in enumerate(p)]


def frame_vectors():
    arena, pkts, kinds = synth.make_batch(48, 1501, kinds="mixed", seed=SEED, stride=1505)
    bad, _, _ = synth.make_batch(16, 1501, kinds="mixed", seed=SEED + 1, stride=1505, valid=False)
    arena = np.concatenate([arena[: 48 * 1505], bad[: 16 * 1505], np.zeros(64, np.uint8)])
    p2 = np.zeros(64, pkts.dtype)
    p2[:48] = pkts
    _, pb, _ = synth.make_batch(16, 1501, kinds="mixed", seed=SEED + 1, stride=1505, valid=False)
    synth.set_pkt_off(pb, synth.pkt_off(pb) + np.uint64(48 * 1505))
    p2[48:] = pb
    rec = {
        "arena_hex": arena.tobytes().hex(),
        "pkts": rows(p2),
    }
    for name, mode in (("validate", 2), ("fill", 1), ("partial", 3), ("fold", 0)):
        rec[name] = [int(v) for v in oracle.checksum_batch(mode, arena.copy(), p2)]
    p4 = p2.copy()
    p4 = p4[(p4["flags"] & 1) == 0]
    rec["ip4hdr_pkts"] = rows(p4)
    rec["ip4hdr"] = [int(v) for v in oracle.checksum_batch(4, arena.copy(), p4)]
    return rec


def gso_vectors():
    cases = [
        dict(total=6000, gso=1460, v6=False, udp=False, flags=0x19, nbufs=128, bufsize=2000, offset=16),
        dict(total=5000, gso=1000, v6=True, udp=True, flags=0x10, nbufs=128, bufsize=1200, offset=10),
        dict(total=9000, gso=1460, v6=False, udp=False, flags=0x18, nbufs=3, bufsize=1600, offset=16),  # too many
        dict(total=3001, gso=999, v6=True, udp=False, flags=0x10, nbufs=8, bufsize=1100, offset=3),
    ]
    out = []
    for k, c in enumerate(cases):
        vp = synth.make_super_packet(c["total"], c["gso"], seed=SEED + k, v6=c["v6"], udp=c["udp"], tcp_flags=c["flags"])
        rb = np.frombuffer(bytearray(vp), np.uint8).copy()
        bufs = [np.zeros(c["bufsize"], np.uint8) for _ in range(c["nbufs"])]
        rc, n, sizes = oracle.handle_virtio_read(rb, bufs, c["offset"])
        written = c["nbufs"] if rc == -3 else n
        out.append(dict(c, input_hex=vp.hex(), rc=rc, n=n, sizes=sizes[:written],
                        segments_sha256=[sha(bufs[i][c["offset"]: c["offset"] + sizes[i]]) for i in range(written)],
                        readbuf_sha256=sha(rb)))
    # GSO_NONE with NEEDS_CSUM at an odd csumStart
    rng = np.random.default_rng(SEED)
    pkt = rng.integers(0, 256, 777, dtype=np.uint8).tobytes()
    vp = bytes([1, 0, 0, 0, 0, 0, 21, 0, 16, 0]) + pkt
    rb = np.frombuffer(bytearray(vp), np.uint8).copy()
    bufs = [np.zeros(1000, np.uint8)]
    rc, n, sizes = oracle.handle_virtio_read(rb, bufs, 16)
    out.append(dict(total=777, gso=0, nbufs=1, bufsize=1000, offset=16, input_hex=vp.hex(), rc=rc, n=n,
                    sizes=sizes[:1], segments_sha256=[sha(bufs[0][16: 16 + sizes[0]])], readbuf_sha256=sha(rb)))
    return out


def gro_vectors():
    def split(vp, seg):
        rb = np.frombuffer(bytearray(vp), np.uint8).copy()
        bufs = [np.zeros(seg + 100, np.uint8) for _ in range(64)]
        rc, n, sizes = oracle.handle_virtio_read(rb, bufs, 16)
        return [bufs[i][16: 16 + sizes[i]].tobytes() for i in range(n)]
    a = split(synth.make_super_packet(40 + 6 * 1000, 1000, seed=SEED), 1000)
    b = split(synth.make_super_packet(48 + 4 * 800, 800, seed=SEED + 1, v6=True, udp=True), 800)
    c = split(synth.make_super_packet(60 + 3 * 500, 500, seed=SEED + 2, v6=True, tcp_flags=0x18), 500)
    bad = bytearray(a[4]); bad[-1] ^= 1
    pkts = [a[1], a[0], b[0], a[2], c[0], b[1], a[3], bytes(bad), c[1], b[2], a[5], c[2], b[3]]
    bufs = []
    lens = []
    for p in pkts:
        buf = np.zeros(65535, np.uint8)
        buf[16: 16 + len(p)] = np.frombuffer(p, np.uint8)
        bufs.append(buf)
        lens.append(16 + len(p))
    rc, tw, order, nl = oracle.handle_gro(bufs, lens, 16, True)
    return dict(packets_hex=[p.hex() for p in pkts], offset=16, can_udp_gro=True, rc=rc, to_write=tw, order=order,
                lens=nl, written_sha256=[sha(bufs[order[i]][6: nl[i]]) for i in tw])


def main():
    rng = np.random.default_rng(SEED)
    kat = {
        "rfc1071": {"hex": "0001f203f4f5f6f7", "checksum": oracle.checksum(bytes.fromhex("0001f203f4f5f6f7"))},
        "ipv4_header": {"hex": "450000730000400040110000c0a80001c0a800c7", "complement": 0xB861},
        "pseudo": {"src": "c0a80001", "dst": "c0a800c7", "proto": 17, "len": 0x5F, "nofold": "0x80c101c800000000",
                   "checksum": 0x8289},
    }
    assert kat["rfc1071"]["checksum"] == 0xDDF2
    g = {"generator": "tests/golden/make_golden.py", "seed": SEED, "kat": kat, "fold": fold_vectors(rng),
         "frames": frame_vectors(), "gso": gso_vectors(), "gro": gro_vectors()}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(g, f, separators=(",", ":"))
    print(os.path.getsize(os.path.join(HERE, "golden.json")), "bytes")


if __name__ == "__main__":
    main()
