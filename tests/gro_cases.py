"""GRO header-field fuzz corpus (test infrastructure): Write calls whose
packets carry mutated IPv4 / IPv6 / TCP / UDP header fields -- the fields
handleGRO's candidate checks and the can-coalesce predicates read
(gro.go:392-544 ipHeadersCanCoalesce / tcpPacketsCanCoalesce /
udpPacketsCanCoalesce, :784-800 and :1280-1324 the candidate tests): TOS,
TTL, DF/MF and fragment offset, IP options, total / payload length, next
header, hop limit, traffic class and flow label, TCP flags, data offset,
ack, window and options, the UDP length; truncated packets and trailing
bytes.  Most mutated packets get valid checksums again, some do not.  Shared
by the CPU cross-check of the two restatements and the GPU parity tests."""
import struct

import numpy as np

import oracle

OFFSET = 16


def _fix(pkt: bytearray, v6: bool) -> None:
    """Recompute the IPv4 header checksum and the L4 checksum (pseudo header
    over the addresses, the packet's protocol byte and len - iphLen)."""
    if v6:
        iph, proto = 40, pkt[6]
        src, dst = bytes(pkt[8:24]), bytes(pkt[24:40])
    else:
        iph, proto = (pkt[0] & 0xF) * 4, pkt[9]
        if iph < 20 or iph > len(pkt):
            return
        pkt[10:12] = b"\0\0"
        pkt[10:12] = ((~oracle.checksum(bytes(pkt[:iph]), 0)) & 0xFFFF).to_bytes(2, "big")
        src, dst = bytes(pkt[12:16]), bytes(pkt[16:20])
    at = iph + (16 if proto == 6 else 6)
    if at + 2 > len(pkt):
        return
    pkt[at:at + 2] = b"\0\0"
    ph = oracle.pseudo_header_nofold(src, dst, proto, len(pkt) - iph)
    pkt[at:at + 2] = ((~oracle.checksum(bytes(pkt[iph:]), ph)) & 0xFFFF).to_bytes(2, "big")


def packet(v6, udp, src, dst, sport, dport, seq, payload, *, flags=0x10, ack=7, tcp_opts=b"", ip_opts=b"",
           tos=0, ttl=64, ipflags=0x4000, ipid=0x1234, tc=0, flow=0, hop=64, win=65535):
    if udp:
        l4 = bytearray(struct.pack("!HHHH", sport, dport, 8 + len(payload), 0) + payload)
        proto = 17
    else:
        th = 20 + len(tcp_opts)
        l4 = bytearray(struct.pack("!HHIIBBHHH", sport, dport, seq & 0xFFFFFFFF, ack & 0xFFFFFFFF, (th // 4) << 4,
                                   flags, win, 0, 0) + tcp_opts + payload)
        proto = 6
    if v6:
        ip = bytearray(struct.pack("!IHBB", (6 << 28) | (tc << 20) | flow, len(l4), proto, hop) + src + dst)
    else:
        ihl = 5 + len(ip_opts) // 4
        ip = bytearray(struct.pack("!BBHHHBBH4s4s", 0x40 | ihl, tos, ihl * 4 + len(l4), ipid, ipflags, ttl, proto, 0,
                                   src, dst) + ip_opts)
    pkt = ip + l4
    _fix(pkt, v6)
    return bytes(pkt)


def _mutate(rng, pkt: bytes, v6: bool, udp: bool) -> bytes:
    b = bytearray(pkt)
    iph = 40 if v6 else 20
    m = int(rng.integers(0, 16))
    if m == 0:
        if v6:
            b[1] ^= 0x10                                          # traffic class
        else:
            b[1] ^= int(rng.integers(1, 256))                     # TOS
    elif m == 1:
        b[7 if v6 else 8] = int(rng.integers(0, 256))             # hop limit / TTL
    elif m == 2 and not v6:
        b[6] = int(rng.choice([0x00, 0x20, 0x60, 0x40, 0x41]))   # DF / MF / fragment offset
        b[7] = int(rng.choice([0, 0, 1, 0xFF]))
    elif m == 2:
        b[3] ^= int(rng.integers(1, 256))                         # flow label
    elif m == 3:
        d = int(rng.choice([-9, -1, 1, 4, 100]))                  # total / payload length
        at = 4 if v6 else 2
        v = (int.from_bytes(b[at:at + 2], "big") + d) & 0xFFFF
        b[at:at + 2] = v.to_bytes(2, "big")
    elif m == 4:
        b[6 if v6 else 9] = int(rng.choice([6, 17, 1, 41, 0]))    # next header / protocol
    elif m == 5 and not udp:
        b[iph + 13] = int(rng.choice([0x02, 0x04, 0x01, 0x11, 0x19, 0x20, 0x30, 0x40, 0x80, 0x18, 0x00]))
    elif m == 6 and not udp:
        b[iph + 12] = int(rng.choice([0x40, 0x60, 0xF0, 0x00, 0x50]))  # data offset
    elif m == 7 and not udp:
        b[iph + 8:iph + 12] = int(rng.integers(0, 2**32)).to_bytes(4, "big")  # ack
    elif m == 8 and not udp:
        b[iph + 14:iph + 16] = int(rng.integers(0, 65536)).to_bytes(2, "big")  # window
    elif m == 8:
        d = int(rng.choice([-1, 1, 8]))                           # UDP length
        v = (int.from_bytes(b[iph + 4:iph + 6], "big") + d) & 0xFFFF
        b[iph + 4:iph + 6] = v.to_bytes(2, "big")
    elif m == 9:
        b = b[: int(rng.integers(1, max(2, len(b))))]            # truncated
    elif m == 10:
        b += bytes(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8))  # trailing bytes
    elif m == 11:
        b[(8 if v6 else 12) + int(rng.integers(0, 4))] ^= 1      # source address
    elif m == 12 and not v6:
        b[4:6] = int(rng.integers(0, 65536)).to_bytes(2, "big")  # IPv4 id
    elif m == 13:
        b[0] = (b[0] & 0x0F) | (int(rng.choice([4, 6, 5, 0])) << 4)  # IP version
    elif m == 14 and not udp:
        b[iph + 18:iph + 20] = int(rng.integers(1, 65536)).to_bytes(2, "big")  # urgent pointer
    else:
        b[-1] ^= 0x5A                                             # payload byte (checksum now wrong)
        return bytes(b)
    if rng.random() < 0.85 and m not in (9,):
        _fix(b, v6 and (b[0] >> 4) == 6)
    return bytes(b)


def _flow(rng, n, mss, v6, udp, k):
    src = bytes(rng.integers(0, 256, 16 if v6 else 4, dtype=np.uint8))
    dst = bytes(rng.integers(0, 256, 16 if v6 else 4, dtype=np.uint8))
    seq0 = int(rng.integers(0, 2**32))
    ip_opts = bytes([1, 1, 1, 0]) if (not v6 and rng.random() < 0.15) else b""
    tcp_opts = bytes([1, 1, 8, 10]) + bytes(8) if (not udp and rng.random() < 0.2) else b""
    tos, ttl = int(rng.choice([0, 0, 0x10])), int(rng.choice([64, 64, 1]))
    out = []
    for j in range(n):
        ln = mss if j < n - 1 or rng.random() < 0.6 else int(rng.integers(1, mss + 1))
        pay = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
        flags = 0x18 if (j == n - 1 and rng.random() < 0.4) else 0x10
        out.append(packet(v6, udp, src, dst, 3000 + k, 51820, seq0 + j * mss, pay, flags=flags, ip_opts=ip_opts,
                          tcp_opts=tcp_opts, tos=tos, ttl=ttl))
    return out


def field_fuzz_calls(count: int = 150, seed: int = 4242):
    """[(pkts, cap, can_udp, lens_override)] Write calls, as the GRO GPU tests take them."""
    rng = np.random.default_rng(seed)
    calls = []
    for c in range(count):
        pk = []
        for f in range(int(rng.integers(1, 5))):
            v6, udp = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
            pk += [(p, v6, udp) for p in _flow(rng, int(rng.integers(1, 24)), int(rng.choice([200, 536, 1448])),
                                                v6, udp, 10 * c + f)]
        pk = pk[:128]
        out = []
        for p, v6, udp in pk:
            out.append(_mutate(rng, p, v6, udp) if rng.random() < 0.2 else p)
        noise = rng.random(len(out)) * (2.0 if c % 4 == 0 else 0.2)
        out = [out[i] for i in np.argsort(np.arange(len(out)) * 0.1 + noise)]
        cap = 65535 if c % 5 else (lambda n, e=int(rng.integers(0, 3000)): OFFSET + n + e)
        calls.append((out, cap, bool(c % 6), None))
    return calls


def long_run_calls(seed: int = 9090):
    """[(pkts, cap, can_udp, lens_override)] long in-order TCP flows (65-128
    packets, so a flow spans more than one 64-packet window of the kernel's
    wave-wide append run) broken at and around the window edges: a short
    payload, PSH, a bad checksum, a changed TOS / ack / TTL, a missing or a
    repeated segment, the item's capacity running out, other flows
    interleaved so a window holds non-members too.  Calls 40-59: UDP flows
    (UDP GRO walks them the same way)."""
    rng = np.random.default_rng(seed)
    calls = []
    spots = [0, 1, 31, 62, 63, 64, 65, 66, 100, 126, 127]
    kinds = ["short", "psh", "badsum", "tos", "ack", "ttl", "gap", "dup", "none"]
    for c in range(60):
        v6, udp = bool(c % 2), c >= 40
        n = int(rng.integers(65, 129))
        mss = int(rng.choice([200, 536, 1448]))
        src = bytes(rng.integers(0, 256, 16 if v6 else 4, dtype=np.uint8))
        dst = bytes(rng.integers(0, 256, 16 if v6 else 4, dtype=np.uint8))
        seq0 = int(rng.integers(0, 2**32))
        brk = {int(rng.choice(spots)) % n: kinds[(c + k) % len(kinds)] for k in range(int(rng.integers(1, 4)))}
        pk, seq = [], seq0
        for j in range(n):
            kind = brk.get(j, "")
            ln = int(rng.integers(1, mss)) if kind == "short" else mss
            pay = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
            if kind == "gap":
                seq += mss
            if kind == "dup":
                seq -= mss
            p = packet(v6, udp, src, dst, 5000, 51820, seq, pay, flags=0x18 if kind == "psh" else 0x10,
                       ack=9 if kind == "ack" else 7, tos=0x10 if kind == "tos" else 0, tc=1 if kind == "tos" else 0,
                       ttl=3 if kind == "ttl" else 64, hop=3 if kind == "ttl" else 64)
            if kind == "badsum":
                p = p[:-1] + bytes([p[-1] ^ 0x5A])
            pk.append(p)
            seq += ln
        if c % 4 == 3:  # another flow interleaved, every third slot
            other = _flow(rng, 128 - n if n < 128 else 0, mss, v6, udp, 777 + c)
            mixed = []
            for j, p in enumerate(pk):
                mixed.append(p)
                if j % 3 == 2 and other:
                    mixed.append(other.pop(0))
            pk = (mixed + other)[:128]
        cap = 65535 if c % 5 else 200000
        calls.append((pk, cap, True, None))
    return calls
