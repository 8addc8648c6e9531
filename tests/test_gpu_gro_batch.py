"""GPU parity: the device-resident batch of Tun.Write calls
(wgcs_handle_gro_batch, one workgroup per call) vs the oracle's handleGRO per
call -- status, toWrite, the slice headers after the prepend swaps and
appends, and every byte of every buffer (tun/tun.go:654-700,
gro.go:1326-1367).  The calls are the write-stager cases (mixed TCP/UDP,
v4/v6, PSH, prepends, capacity limits, UDP GRO off, invalid offsets, bad
checksums) plus one call per edge case."""
import numpy as np
import pytest
import torch

import oracle
from wireguard_amd.tun import GRO_BUF_DTYPE, GRO_CALL_DTYPE, GRO_CAN_UDP

from test_gpu_gro import flow
from test_gpu_wstager import OFFSET, _calls, _mk

pytestmark = pytest.mark.gpu


def _run(dev, calls):
    """calls: [(pkts, cap, can_udp, lens_override)] -> per call (status,
    to_write, bufs_out) and the final arena, next to the oracle's buffers."""
    host_bufs, lens_all, meta = [], [], []
    for pkts, cap, can_udp, lo in calls:
        bufs, lens = _mk(pkts, cap, OFFSET, lo)
        meta.append((len(host_bufs), len(bufs), can_udp))
        host_bufs += bufs
        lens_all += lens
    offs, pos = [], 0
    for b in host_bufs:
        offs.append(pos)
        pos += (len(b) + 15) // 16 * 16 + 16
    arena = np.zeros(pos + 64, np.uint8)
    for o, b in zip(offs, host_bufs):
        arena[o: o + len(b)] = b
    gb = np.zeros(len(host_bufs), GRO_BUF_DTYPE)
    gb["off"] = offs
    gb["len"] = lens_all
    gb["cap"] = [len(b) for b in host_bufs]
    gc = np.zeros(len(calls), GRO_CALL_DTYPE)
    for c, (first, n, can_udp) in enumerate(meta):
        gc[c] = (first, n, OFFSET, GRO_CAN_UDP if can_udp else 0)
    d_arena = torch.from_numpy(arena).cuda()
    d_bufs = torch.from_numpy(gb.view(np.uint8)).cuda()
    d_calls = torch.from_numpy(gc.view(np.uint8)).cuda()
    st = torch.zeros(len(calls), dtype=torch.int32, device="cuda")
    nw = torch.zeros(len(calls), dtype=torch.int32, device="cuda")
    tw = torch.full((len(host_bufs),), -7, dtype=torch.int32, device="cuda")
    dev.handle_gro_batch(d_arena, d_bufs, d_calls, len(calls), st, nw, tw)
    torch.cuda.synchronize()
    return (meta, offs, host_bufs, lens_all, arena, d_arena.cpu().numpy(), d_bufs.cpu().numpy().view(GRO_BUF_DTYPE),
            st.cpu().numpy(), nw.cpu().numpy(), tw.cpu().numpy())


def _check(dev, calls):
    meta, offs, host_bufs, lens_all, arena0, arena, gb, st, nw, tw = _run(dev, calls)
    compared = 0
    for c, (first, n, can_udp) in enumerate(meta):
        bo = [host_bufs[first + i].copy() for i in range(n)]
        lo = lens_all[first: first + n]
        rc, tw_o, order, nl = oracle.handle_gro(bo, list(lo), OFFSET, can_udp)
        assert st[c] == rc, (c, st[c], rc)
        if rc == 0:
            assert nw[c] == len(tw_o), c
            assert list(tw[first: first + nw[c]]) == list(tw_o), c
        for i in range(n):  # slice headers: buffer at position i and its length
            g = gb[first + i]
            assert g["off"] == offs[first + order[i]], (c, i)
            assert g["len"] == nl[i], (c, i, g["len"], nl[i])
        for j in range(n):  # every byte of every buffer, by buffer identity
            o = offs[first + j]
            got = arena[o: o + len(bo[j])]
            if not np.array_equal(got, bo[j]):
                diff = np.flatnonzero(got != bo[j])
                bad = int(diff[0])
                pos = order.index(j)
                raise AssertionError(
                    f"call {c} buffer {j} (now at position {pos}, len {lo[j]} -> {nl[pos]}, cap {len(bo[j])}, "
                    f"to_write {pos in tw_o}, {len(diff)} bytes differ in [{bad}, {int(diff[-1])}]): "
                    f"got {got[bad:bad + 8].tobytes().hex()} want {bo[j][bad:bad + 8].tobytes().hex()} "
                    f"orig {host_bufs[first + j][bad:bad + 8].tobytes().hex()}; lens {lo[:12]}")
        compared += 1
    return compared


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gro_batch_matches_handle_gro(dev, seed):
    calls = _calls(seed)
    assert _check(dev, calls) == len(calls)


def edge_calls():
    f4 = flow(8, seg=1448, seed=7)
    f6 = flow(8, seg=1000, v6=True, seed=8)
    u4 = flow(8, seg=1200, udp=True, seed=9)
    rev = list(reversed(f4))  # a prepend chain
    calls = [
        (f4, 65535, True, None),
        (rev, 65535, True, None),
        (f4 + f6 + u4, 65535, True, None),
        (u4, 65535, False, None),                       # UDP GRO off: every packet written as-is
        (f4[:1], 65535, True, None),                    # one packet
        (f4, lambda n: OFFSET + n, True, None),         # no spare capacity: nothing merges
        (f4, 65535, True, {0: OFFSET}),                 # invalid offset on the first buffer
        (f4 + u4, 65535, True, {5: 3}),                 # invalid offset part-way (len < offset)
        ([bytes(40)] * 4 + f4, 65535, True, None),      # non-candidates first
    ]
    return calls


def test_gro_batch_edge_calls(dev):
    calls = edge_calls()
    assert _check(dev, calls) == len(calls)


def bad_checksum_calls():
    rng = np.random.default_rng(5)
    calls = []
    for k in range(12):
        fs = [flow(int(rng.integers(2, 10)), seg=int(rng.choice([536, 1448])), v6=bool(k & 1), udp=bool(k & 2),
                   seed=100 + 10 * k + j, last_flags=int(rng.choice([0x10, 0x18]))) for j in range(3)]
        pk = [p for f in fs for p in f]
        for _ in range(int(rng.integers(0, 4))):
            i = int(rng.integers(0, len(pk)))
            b = bytearray(pk[i])
            b[int(rng.integers(20, len(b)))] ^= 0x41
            pk[i] = bytes(b)
        order = np.argsort(rng.random(len(pk)) + np.arange(len(pk)) * 0.05)
        calls.append(([pk[i] for i in order], 65535, True, None))
    return calls


def test_gro_batch_bad_checksums_and_flags(dev):
    calls = bad_checksum_calls()
    assert _check(dev, calls) == len(calls)


def test_gro_batch_rejects_oversized_call(dev):
    f = flow(4, seed=11)
    calls = [(f * 65, 65535, True, None)]  # 260 buffers > WGCS_GRO_MAX_CALL
    meta, offs, host_bufs, lens_all, arena0, arena, gb, st, nw, tw = _run(dev, calls)
    assert st[0] == -1 and nw[0] == 0  # WGCS_ERR_INVALID_ARG, nothing touched
    assert np.array_equal(arena, arena0)


def host_scenario_calls():
    """Every scenario of tests/test_gpu_gro.py (the host-path GRO tests) as
    one call each."""
    rng = np.random.default_rng(11)
    s_pre = flow(6, seed=3)
    s_bad = flow(8, seed=5)
    for k in (0, 3, 7):
        b = bytearray(s_bad[k]); b[-1] ^= 0x5A; s_bad[k] = bytes(b)
    u_bad = flow(6, udp=True, seed=6)
    b = bytearray(u_bad[2]); b[-2] ^= 1; u_bad[2] = bytes(b)
    flows = [flow(int(rng.integers(1, 10)), seg=int(rng.choice([536, 1000, 1448])), v6=bool(k % 2),
                  udp=bool(k % 3 == 0), seed=100 + k, last_flags=int(rng.choice([0x10, 0x18]))) for k in range(10)]
    icmp = bytearray(flows[0][0]); icmp[9] = 1
    opts = bytearray(flows[1][0] if not flows[1][0][0] >> 4 == 6 else flows[0][0]); opts[0] = 0x46
    frag = bytearray(flows[0][0]); frag[6] = 0x20
    batch = [p for f in flows for p in f] + [bytes(icmp), bytes(opts), bytes(frag)]
    order = np.argsort(rng.random(len(batch)) + np.arange(len(batch)) * 0.05)
    mixed = [batch[i] for i in order]
    for _ in range(5):
        k = int(rng.integers(0, len(mixed)))
        b = bytearray(mixed[k]); b[-1] ^= 0x11; mixed[k] = bytes(b)
    a, u, o = flow(6, seed=21, last_flags=0x18), flow(4, udp=True, seed=22), flow(4, seed=23)
    inv = [a[0], a[1], u[0], o[1], o[0], a[2], u[1], a[3], o[2], a[4], u[2], a[5], o[3], u[3]]
    ic2 = bytearray(a[0]); ic2[9] = 1
    inv.insert(3, bytes(ic2))
    big = []
    for k in range(16):
        big += flow(8, seg=1400, v6=bool(k % 2), udp=bool(k % 4 == 3), seed=200 + k)
    perm = np.random.default_rng(12).permutation(len(big))
    calls = [
        (flow(8), 65535, True, None),
        (flow(12, seg=1200, seed=7), 65535, True, None),
        (flow(12, seg=1200, v6=True, seed=7), 65535, True, None),
        (flow(12, seg=1200, udp=True, seed=7), 65535, True, None),
        (flow(12, seg=1200, v6=True, udp=True, seed=7), 65535, True, None),
        ([s_pre[2], s_pre[1], s_pre[0], s_pre[3], s_pre[5], s_pre[4]], 65535, True, None),
        (flow(5, seg=1000, seed=4, last_flags=0x18), 65535, True, None),
        (flow(3, seg=700, seed=4) + flow(3, seg=1000, seed=4), 65535, True, None),
        (s_bad, 65535, True, None),
        (u_bad, 65535, True, None),
        (flow(6, seg=1000, seed=8), lambda n: OFFSET + n + 1500, True, None),
        (flow(4, udp=True, seed=9), 65535, False, None),
        (mixed, 65535, True, None),
        ([big[i] for i in perm], 65535, True, None),
        (big, 65535, True, None),
    ] + [(inv, 65535, True, {bad_at: OFFSET}) for bad_at in (1, 5, 9, 13)]
    return calls


def test_gro_batch_host_test_scenarios(dev):
    """Every scenario of tests/test_gpu_gro.py as one call each, all in one launch."""
    calls = host_scenario_calls()
    assert _check(dev, calls) == len(calls)


def _tcp_pkt(src, dst, sport, dport, seq, flags, opts, payload, v6):
    """One TCP segment with options and valid IPv4 / TCP checksums (oracle
    checksum functions: test infrastructure)."""
    import struct

    th = 20 + len(opts)
    tcp = bytearray(struct.pack("!HHIIBBHHH", sport, dport, seq & 0xFFFFFFFF, 7, (th // 4) << 4, flags, 65535, 0, 0)
                    + opts + payload)
    if v6:
        ip = bytearray(struct.pack("!IHBB", 0x60000000, len(tcp), 6, 64) + src + dst)
    else:
        ip = bytearray(struct.pack("!BBHHHBBH4s4s", 0x45, 0, 20 + len(tcp), 0x1234, 0x4000, 64, 6, 0, src, dst))
        ip[10:12] = ((~oracle.checksum(bytes(ip), 0)) & 0xFFFF).to_bytes(2, "big")
    c = (~oracle.checksum(bytes(tcp), oracle.pseudo_header_nofold(src, dst, 6, len(tcp)))) & 0xFFFF
    tcp[16:18] = c.to_bytes(2, "big")
    return bytes(ip + tcp)


def _opt_flow(rng, nseg, mss, v6, same_opts, seed):
    src = bytes(rng.integers(0, 256, 16 if v6 else 4, dtype=np.uint8))
    dst = bytes(rng.integers(0, 256, 16 if v6 else 4, dtype=np.uint8))
    sport, dport = 1000 + seed, 51820
    seq0 = int(rng.integers(0, 2**32))
    out = []
    for k in range(nseg):
        ts = 1000 if same_opts else 1000 + k
        opts = bytes([1, 1, 8, 10]) + ts.to_bytes(4, "big") + (99).to_bytes(4, "big")  # NOP NOP TS
        flags = 0x18 if k == nseg - 1 and rng.random() < 0.5 else 0x10
        out.append(_tcp_pkt(src, dst, sport, dport, seq0 + k * mss, flags, opts,
                            bytes(rng.integers(0, 256, mss, dtype=np.uint8)), v6))
    return out


def tcp_options_calls():
    """Random Write calls mixing TCP flows with timestamp options (equal
    options coalesce, changing ones do not: gro.go:442-448), flows without
    options, UDP, reordering (prepends), tight capacities and corrupted
    checksums."""
    rng = np.random.default_rng(2024)
    calls = []
    for k in range(40):
        flows = []
        for j in range(int(rng.integers(1, 6))):
            kind = int(rng.integers(0, 4))
            n = int(rng.integers(1, 20))
            mss = int(rng.choice([536, 1000, 1448]))
            if kind == 0:
                flows.append(_opt_flow(rng, n, mss, bool(rng.integers(0, 2)), True, 10 * k + j))
            elif kind == 1:
                flows.append(_opt_flow(rng, n, mss, bool(rng.integers(0, 2)), False, 10 * k + j))
            else:
                flows.append(flow(n, seg=mss, v6=bool(rng.integers(0, 2)), udp=kind == 3, seed=5000 + 10 * k + j,
                                  last_flags=int(rng.choice([0x10, 0x18]))))
        pk = [p for f in flows for p in f][:128]
        noise = rng.random(len(pk)) * (3.0 if k % 3 == 0 else 0.3)  # sometimes heavy reordering
        pk = [pk[i] for i in np.argsort(np.arange(len(pk)) * 0.1 + noise)]
        for _ in range(int(rng.integers(0, 3))):
            i = int(rng.integers(0, len(pk)))
            b = bytearray(pk[i]); b[-1] ^= 0x24; pk[i] = bytes(b)
        cap = 65535 if k % 4 else (lambda n, e=int(rng.integers(0, 4000)): OFFSET + n + e)
        calls.append((pk, cap, bool(k % 5), None))
    return calls


def _udp_pkt(src, dst, sport, dport, payload, v6):
    """One UDP datagram with valid IPv4 / UDP checksums (oracle checksum
    functions: test infrastructure)."""
    import struct

    udp = bytearray(struct.pack("!HHHH", sport, dport, 8 + len(payload), 0) + payload)
    if v6:
        ip = bytearray(struct.pack("!IHBB", 0x60000000, len(udp), 17, 64) + src + dst)
    else:
        ip = bytearray(struct.pack("!BBHHHBBH4s4s", 0x45, 0, 20 + len(udp), 0x1234, 0x4000, 64, 17, 0, src, dst))
        ip[10:12] = ((~oracle.checksum(bytes(ip), 0)) & 0xFFFF).to_bytes(2, "big")
    c = (~oracle.checksum(bytes(udp), oracle.pseudo_header_nofold(src, dst, 17, len(udp)))) & 0xFFFF
    udp[6:8] = c.to_bytes(2, "big")
    return bytes(ip + udp)


def _seq_flow(rng, nseg, mss, v6, udp=False, psh_at=(), seq0=None):
    src = bytes(rng.integers(0, 256, 16 if v6 else 4, dtype=np.uint8))
    dst = bytes(rng.integers(0, 256, 16 if v6 else 4, dtype=np.uint8))
    seq0 = int(rng.integers(0, 2**32)) if seq0 is None else seq0
    out = []
    for k in range(nseg):
        pay = bytes(rng.integers(0, 256, mss, dtype=np.uint8))
        if udp:
            out.append(_udp_pkt(src, dst, 4000, 51820, pay, v6))
        else:
            out.append(_tcp_pkt(src, dst, 4000, 51820, seq0 + k * mss, 0x18 if k in psh_at else 0x10, b"", pay, v6))
    return out


def quirk_calls():
    """Write calls that reach the reference's integer-width quirks and PSH
    rules: capacities above 64 KiB, so an item grows past the uint16
    lhsLen = gsoSize * (numMerged + 1) (gro.go:468, it wraps and the next
    segment no longer looks adjacent) and past uint16 total / payload / UDP
    lengths (apply*, gro.go:1124-1138, :1206-1232); a PSH segment in the middle
    of a flow (nothing appends after it, gro.go:474-478; it still appends
    itself, :724-729); the sequence number wrapping 2^32."""
    rng = np.random.default_rng(77)
    big = 200000
    return [
        (_seq_flow(rng, 8, 1000, False, psh_at=(3,)), 65535, True, None),
        (_seq_flow(rng, 8, 1000, True, psh_at=(0, 5)), 65535, True, None),
        (_seq_flow(rng, 100, 1448, False), big, True, None),
        (_seq_flow(rng, 128, 536, True), big, True, None),
        (_seq_flow(rng, 100, 1400, False, udp=True), big, True, None),
        (_seq_flow(rng, 60, 1200, True, udp=True), big, True, None),
        (list(reversed(_seq_flow(rng, 60, 1448, False))), big, True, None),
        (_seq_flow(rng, 20, 1448, False, seq0=2**32 - 5 * 1448 - 7), 65535, True, None),
        (list(reversed(_seq_flow(rng, 20, 1000, True, seq0=2**32 - 700))), 65535, True, None),
    ]


def test_gro_batch_quirk_calls(dev):
    calls = quirk_calls()
    assert _check(dev, calls) == len(calls)


def test_gro_batch_tcp_options_fuzz(dev):
    """The options fuzz calls in one launch: the register fast path falls back
    to the LDS path for every one of these."""
    calls = tcp_options_calls()
    assert _check(dev, calls) == len(calls)


def test_gro_batch_bench_call_shapes(dev):
    """The gro_device bench's call shapes (one 128-packet flow, prepend chains,
    a shuffled batch) against the oracle, every byte, in one launch."""
    from wireguard_amd.gro_bench import CALL_SHAPES, CAP, shape_batch

    calls = [(shape_batch(dev, s), CAP, True, None) for s in CALL_SHAPES]
    assert _check(dev, calls) == len(calls)


def test_gro_batch_field_fuzz(dev):
    """The header-field fuzz calls (tests/gro_cases.py: mutated TOS, TTL,
    fragment bits, lengths, protocol, TCP flags / data offset / ack / window,
    UDP length, truncated packets, trailing bytes) in one launch."""
    import gro_cases

    calls = gro_cases.field_fuzz_calls()
    assert _check(dev, calls) == len(calls)


def test_gro_batch_long_runs(dev):
    """Long in-order flows broken at and around the 64-packet window edges of
    the kernel's wave-wide append run (tests/gro_cases.py long_run_calls), in
    one launch, every byte against the oracle."""
    import gro_cases

    calls = gro_cases.long_run_calls()
    assert _check(dev, calls) == len(calls)
