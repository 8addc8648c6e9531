"""The GSO header-fuzz corpus shared by the GPU parity test
(tests/test_gpu_gso.py::test_fuzz_headers) and the CPU cross-check of the two
oracle restatements (tests/test_py_restatement.py): the same seeded cases in
the same order."""
import numpy as np

from wireguard_amd import synth

SENT = 0xA5


def fuzz_header(rng, base: bytearray, raw: bool):
    """Mutate the virtio header / IP version / TCP data offset of a valid
    super-packet: any header geometry handleVirtioRead or gsoSplit accepts,
    including IP headers shorter than 20 / 40 bytes, headers over 240 bytes,
    checksum fields outside the header, wrapped uint16 positions."""
    b = bytearray(base)
    plen = len(b) - 10
    f = lambda a, v: b.__setitem__(slice(a, a + 2), int(v % 65536).to_bytes(2, "little"))  # noqa: E731
    if rng.random() < 0.2:
        b[0] = int(rng.integers(0, 256))
    if rng.random() < 0.3:
        b[1] = int(rng.choice([0, 1, 4, 5, int(rng.integers(0, 256))]))
    cs = int(rng.choice([int.from_bytes(b[6:8], "little"), int(rng.integers(0, 64)), int(rng.integers(0, 400)),
                         int(rng.integers(65500, 65536))], p=[0.25, 0.35, 0.35, 0.05]))
    f(6, cs)
    if rng.random() < 0.8 and plen >= 2:
        at = int(rng.integers(0, min(plen - 1, 600))) if rng.random() < 0.7 else int(rng.integers(0, plen - 1))
        f(8, at - cs)
    else:
        f(8, int(rng.integers(0, 65536)))
    if rng.random() < 0.5:
        f(2, int(rng.choice([cs + 8, cs + 20, int(rng.integers(0, 600)), int(rng.integers(0, 65536))])))
    if rng.random() < 0.4:
        f(4, int(rng.choice([0, 1, 7, int(rng.integers(1, 3000)), 65535])))
    if rng.random() < 0.3:
        b[10] = (int(rng.choice([4, 6, int(rng.integers(0, 16))])) << 4) | (b[10] & 0xF)
    if 10 + cs + 12 < len(b) and rng.random() < 0.5:
        b[10 + cs + 12] = int(rng.choice([0x50, 0x80, 0xF0, int(rng.integers(0, 256))]))
    if rng.random() < 0.25:
        b = b[: int(rng.integers(10, len(b) + 1))]
    return bytes(b)



def fuzz_cases(raw: bool):
    """Yields (vp, nbufs, bufsize, fill, offset, hdr, is_v6): 1,100
    handleVirtioRead cases (raw False) or 1,500 gsoSplit cases with the
    caller's header hdr (raw True; hdr / is_v6 are None otherwise)."""
    rng = np.random.default_rng(17 + raw)
    bases = [bytearray(synth.make_super_packet(t, g, seed=t, v6=v6, udp=u))
             for t, g, v6, u in [(8000, 1000, False, False), (3000, 500, True, False), (6000, 1448, False, True),
                                 (2500, 700, True, True), (1200, 100, False, False), (20000, 1460, False, False)]]
    for trial in range(1500 if raw else 1100):
        vp = fuzz_header(rng, bases[trial % len(bases)], raw)
        nbufs = int(rng.choice([4, 16, 64]))
        bufsize = int(rng.choice([2000, 9000, 65535]))
        fill = int(rng.choice([SENT, 0x00, 0xFF]))
        offset = int(rng.choice([16, 10, 3, 0]))
        if raw:
            h = tuple([vp[0], vp[1]] + [int.from_bytes(vp[k:k + 2], "little") for k in (2, 4, 6, 8)])
            yield vp, nbufs, bufsize, fill, offset, h, bool(rng.integers(0, 2))
        else:
            yield vp, nbufs, bufsize, fill, offset, None, None


def short_cases(raw: bool, count: int = 400):
    """Packets shorter than their pseudo-header addresses (< 20 B IPv4, < 40 B
    IPv6) whose split still runs, followed by 0-48 bytes of the read buffer's
    spare capacity: gsoSplit's address slices (gro.go:1471-1477) read the
    spare bytes, or panic past them.  Yields (buf, n_read, nbufs, bufsize,
    fill, offset, hdr, is_v6): buf[:n_read] is the read (virtio header first
    unless raw), buf[n_read:] the spare capacity."""
    rng = np.random.default_rng(29 + raw)
    for _ in range(count):
        v6 = bool(rng.integers(0, 2))
        plen = int(rng.integers(12, 40 if v6 else 20))
        pkt = rng.integers(0, 256, plen, dtype=np.uint8)
        pkt[0] = (0x60 if v6 else 0x45) | (pkt[0] & 0x0F if v6 else 0)
        tcp = bool(rng.integers(0, 2)) and (raw or v6)
        cs = int(rng.integers(0, min(plen - 1, 20 if tcp and not raw else plen - 1)))
        if raw:
            hdr_len = int(rng.integers(cs, plen))
        else:
            hdr_len = cs + 20 if tcp else cs + 8
            if tcp:
                if cs + 12 < plen:
                    pkt[cs + 12] = 0x50
                else:
                    tcp = False
                    hdr_len = cs + 8
        at = int(rng.integers(0, plen - 1))
        co = (at - cs) % 65536
        gso = int(rng.integers(1, 12))
        gtype = (4 if v6 else 1) if tcp else 5
        vh = bytes([1, gtype]) + b"".join(int(x).to_bytes(2, "little") for x in (hdr_len, gso, cs, co))
        spare = rng.integers(0, 256, int(rng.choice([0, 3, 8, 20, 28, 48])), dtype=np.uint8).tobytes()
        body = pkt.tobytes() if raw else vh + pkt.tobytes()
        h = (1, gtype, hdr_len, gso, cs, co)
        yield (body + spare, len(body), 16, int(rng.choice([200, 60])), int(rng.choice([SENT, 0])),
               int(rng.choice([16, 0, 3])), h if raw else None, v6 if raw else None)


def short_valid_cases(count: int = 600):
    """checksumValid on packets shorter than their addresses (or than iphLen),
    with 0-40 bytes of spare capacity after them: (buf, n, iph_len, proto,
    is_v6), the packet being buf[:n] and buf[n:] its spare capacity."""
    rng = np.random.default_rng(31)
    for _ in range(count):
        v6 = bool(rng.integers(0, 2))
        n = int(rng.integers(0, 48 if v6 else 28))
        spare = int(rng.choice([0, 1, 4, 12, 24, 40]))
        buf = rng.integers(0, 256, n + spare, dtype=np.uint8).tobytes()
        iph = int(rng.choice([0, 8, 20, 40, int(rng.integers(0, 64))]))
        yield buf, n, iph, int(rng.choice([6, 17, int(rng.integers(0, 256))])), v6
