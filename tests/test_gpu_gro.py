"""GPU parity: handleGRO (tun/gro.go:1326-1367) -- GPU-validated, GPU-coalesced
product vs the oracle restatement: error code, toWrite, the prepend swaps of
bufs, the Go-slice lengths and every byte handed to the TUN fd
(bufs[i][offset-10:len] for i in toWrite)."""
import numpy as np
import pytest

import oracle
from wireguard_amd import synth

pytestmark = pytest.mark.gpu
OFFSET = 16


def _split(vp, seg):
    rb = np.frombuffer(bytearray(vp), np.uint8).copy()
    n = (len(vp) + seg) // max(seg, 1) + 2
    bufs = [np.zeros(seg + 200, np.uint8) for _ in range(n)]
    rc, cnt, sizes = oracle.handle_virtio_read(rb, bufs, 16)
    assert rc == 0, rc
    return [bufs[i][16: 16 + sizes[i]].tobytes() for i in range(cnt)]


def flow(nseg, seg=1000, v6=False, udp=False, seed=0, last_flags=0x10):
    ih = 40 if v6 else 20
    lh = 8 if udp else 20
    vp = synth.make_super_packet(ih + lh + nseg * seg, seg, seed=seed, v6=v6, udp=udp, tcp_flags=last_flags)
    return _split(vp, seg)


def run_both(dev, pkts, cap=65535, can_udp=True, offset=OFFSET, lens_override=None):
    def mk():
        bufs, lens = [], []
        for p in pkts:
            b = np.full(cap if isinstance(cap, int) else cap(len(p)), 0x5A, np.uint8)
            b[offset: offset + len(p)] = np.frombuffer(p, np.uint8)
            bufs.append(b)
            lens.append(offset + len(p))
        if lens_override:
            for i, ln in lens_override.items():
                lens[i] = ln
        return bufs, lens
    bo, lo = mk()
    bp, lp = mk()
    rc, tw_o, order_o, lens_o = oracle.handle_gro(bo, lo, offset, can_udp)
    tw_p, order_p, lens_p, err = dev.handle_gro(bp, lp, offset, can_udp)
    rc_p = 0 if err is None else err.code
    assert rc_p == rc
    if rc:
        # the loop stopped part-way (gro.go:1335-1337): toWrite so far, the
        # slice headers and every byte of every buffer as the reference leaves them
        assert (tw_p, order_p, lens_p) == (tw_o, order_o, lens_o)
        for i in range(len(bo)):
            assert np.array_equal(bo[i], bp[i]), f"bufs[{i}] differs after the error"
        return
    assert tw_p == tw_o
    assert order_p == order_o, "prepend swaps differ"
    assert lens_p == lens_o
    for i in tw_o:
        a = bo[order_o[i]][offset - 10: lens_o[i]]
        b = bp[order_p[i]][offset - 10: lens_p[i]]
        assert np.array_equal(a, b), f"written bytes of bufs[{i}] differ"
    return tw_o


def test_in_order_tcp4(dev):
    tw = run_both(dev, flow(8))
    assert tw == [0]


@pytest.mark.parametrize("v6,udp", [(False, False), (True, False), (False, True), (True, True)])
def test_single_flow_kinds(dev, v6, udp):
    run_both(dev, flow(12, seg=1200, v6=v6, udp=udp, seed=7))


def test_out_of_order_prepend(dev):
    s = flow(6, seed=3)
    run_both(dev, [s[2], s[1], s[0], s[3], s[5], s[4]])


def test_psh_and_short_last(dev):
    s = flow(5, seg=1000, seed=4, last_flags=0x18)  # PSH on the last segment only
    run_both(dev, s)
    # a short last segment (GSO tail) then more data -> cannot append after it
    s2 = flow(3, seg=700, seed=4) + flow(3, seg=1000, seed=4)
    run_both(dev, s2)


def test_invalid_checksums(dev):
    s = flow(8, seed=5)
    for k in (0, 3, 7):
        b = bytearray(s[k]); b[-1] ^= 0x5A; s[k] = bytes(b)
    run_both(dev, s)
    u = flow(6, udp=True, seed=6)
    b = bytearray(u[2]); b[-2] ^= 1; u[2] = bytes(b)
    run_both(dev, u)


def test_insufficient_capacity(dev):
    s = flow(6, seg=1000, seed=8)
    run_both(dev, s, cap=lambda n: OFFSET + n + 1500)  # room for one more segment only


def test_udp_gro_disabled(dev):
    run_both(dev, flow(4, udp=True, seed=9), can_udp=False)


def test_mixed_batch(dev):
    rng = np.random.default_rng(11)
    flows = [flow(int(rng.integers(1, 10)), seg=int(rng.choice([536, 1000, 1448])), v6=bool(k % 2),
                  udp=bool(k % 3 == 0), seed=100 + k, last_flags=int(rng.choice([0x10, 0x18])))
             for k in range(10)]
    # non-candidates: ICMP, IPv4 with options, a fragment
    icmp = bytearray(flows[0][0]); icmp[9] = 1
    opts = bytearray(flows[1][0] if not flows[1][0][0] >> 4 == 6 else flows[0][0]); opts[0] = 0x46
    frag = bytearray(flows[0][0]); frag[6] = 0x20
    batch = [p for f in flows for p in f] + [bytes(icmp), bytes(opts), bytes(frag)]
    # interleave flows, mild reordering
    order = np.argsort(rng.random(len(batch)) + np.arange(len(batch)) * 0.05)
    pkts = [batch[i] for i in order]
    for _ in range(5):
        k = int(rng.integers(0, len(pkts)))
        b = bytearray(pkts[k]); b[-1] ^= 0x11; pkts[k] = bytes(b)
    run_both(dev, pkts)


def test_invalid_offset(dev):
    s = flow(3)
    run_both(dev, s, offset=5)
    tw_p, _, _, err = dev.handle_gro([np.zeros(100, np.uint8)], [10], 12, True)
    assert err is not None and err.code == -4


@pytest.mark.parametrize("bad_at", [1, 5, 9, 13])
def test_invalid_offset_after_coalescing(dev, bad_at):
    """An invalid offset on a later buffer: the earlier buffers have already
    been coalesced (appends, prepend swaps, PSH, zero virtio headers of no-op
    packets) but never applied -- the reference's state at the error."""
    a = flow(6, seed=21, last_flags=0x18)
    u = flow(4, udp=True, seed=22)
    o = flow(4, seed=23)
    pkts = [a[0], a[1], u[0], o[1], o[0], a[2], u[1], a[3], o[2], a[4], u[2], a[5], o[3], u[3]]
    icmp = bytearray(a[0]); icmp[9] = 1
    pkts.insert(3, bytes(icmp))
    run_both(dev, pkts, lens_override={bad_at: OFFSET})  # len(bufs[bad_at]) == offset: offset > len-1


def test_batch_size_128(dev):
    """conn.BatchSize = 128 packets per Write (conn/conn.go:12-15)."""
    rng = np.random.default_rng(12)
    pkts = []
    for k in range(16):
        pkts += flow(8, seg=1400, v6=bool(k % 2), udp=bool(k % 4 == 3), seed=200 + k)
    perm = rng.permutation(len(pkts))
    run_both(dev, [pkts[i] for i in perm])
    run_both(dev, pkts)


def test_tcp_options_host_path(dev):
    """wgcs_handle_gro (host planner) on flows with TCP timestamp options:
    equal options coalesce, changing ones do not (gro.go:442-448)."""
    from test_gpu_gro_batch import _opt_flow

    rng = np.random.default_rng(77)
    for k in range(6):
        fa = _opt_flow(rng, 7, 1000, bool(k & 1), True, 2 * k)
        fb = _opt_flow(rng, 5, 1448, bool(k & 2), False, 2 * k + 1)
        pk = fa + fb + flow(4, seed=300 + k)
        order = np.argsort(rng.random(len(pk)) * (2.0 if k > 2 else 0.2) + np.arange(len(pk)) * 0.1)
        run_both(dev, [pk[i] for i in order])


def test_quirk_calls_host_path(dev):
    """The integer-width / PSH quirk calls (test_gpu_gro_batch.quirk_calls:
    capacities above 64 KiB, a mid-flow PSH, sequence numbers wrapping 2^32)
    through the per-call host path (wgcs_handle_gro)."""
    from test_gpu_gro_batch import quirk_calls

    for pkts, cap, can_udp, lo in quirk_calls():
        run_both(dev, pkts, cap=cap, can_udp=can_udp, lens_override=lo)


def test_field_fuzz_host_path(dev):
    """The header-field fuzz calls (tests/gro_cases.py) through the per-call
    host path (wgcs_handle_gro)."""
    import gro_cases

    for pkts, cap, can_udp, lo in gro_cases.field_fuzz_calls(count=60):
        run_both(dev, pkts, cap=cap, can_udp=can_udp, lens_override=lo)
