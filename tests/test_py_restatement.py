"""CPU cross-check of the two oracle restatements: the C
oracle (oracle/wg_oracle.c, which every GPU parity test compares against) and
oracle/py_restatement.py, a second restatement written from the Go text
(tun/checksum.go, tun/gro.go, tun/tun.go:514-632) that shares no code with
it.  Zero mismatches on:
  - checksumNoFold / checksum: random and carry-saturating inputs, both the
    step-by-step ADC chain and the one-sum form of py_restatement;
  - handleVirtioRead and gsoSplit: the GPU tests' 2,600-case header-fuzz
    corpus (tests/gso_cases.py) plus the GPU GSO test configurations --
    status, count, sizes, the readBuf mutation and every byte of every buffer;
  - handleGRO: the GPU tests' Write-call corpora (write-stager calls, edge
    calls, bad checksums, the host-path scenarios, the TCP-options fuzz) --
    status, toWrite, the slice headers after prepend swaps and every byte.
Where both restatements report a Go panic (OUT_OF_RANGE) only the status is
compared: the reference's state after a panic is undefined."""
import numpy as np
import pytest

import gso_cases
import oracle
import py_restatement as py
from wireguard_amd import synth

OOR = py.ERR_OUT_OF_RANGE


def test_checksum_forms_agree():
    rng = np.random.default_rng(99)
    inits = [0, 1, 0xFFFF, 0xFFFFFFFF, 2**64 - 1, 2**63, 0x0123456789ABCDEF]
    cases = []
    for n in list(range(0, 140)) + [255, 256, 257, 1023, 1500, 4096 + 7]:
        cases.append(bytes(rng.integers(0, 256, n, dtype=np.uint8)))
        cases.append(b"\xff" * n)  # every add carries: the chain's saturating case
    cases.append(b"\x00" * 300)
    for b in cases:
        for ini in inits + [int(rng.integers(0, 2**63)) * 2 + 1]:
            want = oracle.checksum_nofold(b, ini)
            assert py.checksum_no_fold(b, ini) == want, (len(b), ini)
            assert py.checksum(b, ini) == oracle.checksum(b, ini) == oracle.closed_form_checksum(b, ini)
    for b in cases[:60]:
        for ini in inits:
            assert py.checksum_no_fold_adc(b, ini) == py.checksum_no_fold(b, ini), (len(b), ini)


def test_pseudo_header_and_valid_kats():
    # RFC 1071 §3 and an IPv4 header KAT, as the C oracle's tests pin them
    assert py.checksum(bytes([0x00, 0x01, 0xF2, 0x03, 0xF4, 0xF5, 0xF6, 0xF7]), 0) == 0xDDF2
    arena, pkts, _ = synth.make_batch(64, 1500, kinds="mixed")
    for p in pkts:
        off = int(p["off_lo"])
        pkt = py.Slice(arena[off: off + 1500].copy())
        v6 = bool(p["flags"] & 1)
        assert py.checksum_valid(pkt, int(p["csum_start"]), int(p["proto"]), v6)
        assert oracle.checksum_valid(bytes(pkt.view()), int(p["csum_start"]), int(p["proto"]), v6)
        pkt[1499] ^= 1
        assert not py.checksum_valid(pkt, int(p["csum_start"]), int(p["proto"]), v6)


def _gso_compare(run_c, run_py, nbufs, bufsize, fill):
    bc = [np.full(bufsize, fill, np.uint8) for _ in range(nbufs)]
    bp = [b.copy() for b in bc]
    (rc_c, n_c, sz_c), rb_c = run_c(bc)
    (rc_p, n_p, sz_p), rb_p = run_py(bp)
    assert rc_p == rc_c, (rc_p, rc_c)
    if rc_c == OOR:
        return "panic"
    assert n_p == n_c
    assert sz_p == sz_c
    assert np.array_equal(rb_p, rb_c), "readBuf mutation"
    for i in range(nbufs):
        assert np.array_equal(bp[i], bc[i]), f"buffer {i}"
    return "compared"


def _virtio_runner(vp, nbufs, bufsize, offset, fill):
    def run_c(bufs):
        rb = np.frombuffer(bytearray(vp), np.uint8).copy()
        return oracle.handle_virtio_read(rb, bufs, offset), rb

    def run_py(bufs):
        rb = np.frombuffer(bytearray(vp), np.uint8).copy()
        return py.run_handle_virtio_read(rb, bufs, offset), rb

    return _gso_compare(run_c, run_py, nbufs, bufsize, fill)


def _raw_runner(rbytes, hdr, is_v6, nbufs, bufsize, offset, fill):
    def run_c(bufs):
        rb = np.frombuffer(bytearray(rbytes), np.uint8).copy()
        return oracle.gso_split(rb, hdr, bufs, offset, is_v6), rb

    def run_py(bufs):
        rb = np.frombuffer(bytearray(rbytes), np.uint8).copy()
        return py.run_gso_split(rb, hdr, bufs, offset, is_v6), rb

    return _gso_compare(run_c, run_py, nbufs, bufsize, fill)


@pytest.mark.parametrize("raw", [False, True])
def test_gso_fuzz_corpus(raw):
    """The 1,100 handleVirtioRead + 1,500 gsoSplit fuzz headers of the GPU
    test: zero mismatches between the two restatements."""
    seen = {"compared": 0, "panic": 0}
    for vp, nbufs, bufsize, fill, offset, h, is_v6 in gso_cases.fuzz_cases(raw):
        if raw:
            seen[_raw_runner(vp[10:], h, is_v6, nbufs, bufsize, offset, fill)] += 1
        else:
            seen[_virtio_runner(vp, nbufs, bufsize, offset, fill)] += 1
    assert seen["compared"] >= 550 and sum(seen.values()) == (1500 if raw else 1100), seen


@pytest.mark.parametrize("v6,udp", [(False, False), (True, False), (False, True), (True, True)])
def test_gso_configs(v6, udp):
    """The GPU GSO test's super-packet configurations (all full splits), the
    TooMany cases, FIN/PSH flags and empty bufs."""
    for total, gso in [(65535, 1460), (1500, 1460), (9000, 1), (4001, 1000), (65535, 65000)]:
        vp = synth.make_super_packet(total, gso, seed=total + gso, v6=v6, udp=udp)
        assert _virtio_runner(vp, 128 if gso > 1 else 9000, 65535 if gso > 1 else 100, 16, 0xA5) == "compared"
    vp = synth.make_super_packet(65535, 1460, v6=v6, udp=udp)
    for nbufs in (0, 1, 5):
        assert _virtio_runner(vp, nbufs, 2000, 16, 0xA5) == "compared"
    for flags in (0x10, 0x19, 0x01):
        vp = synth.make_super_packet(10000, 1460, v6=v6, udp=udp, tcp_flags=flags)
        assert _virtio_runner(vp, 16, 2000, 10, 0x00) == "compared"


def test_gso_none_corpus():
    """GSO_NONE with NEEDS_CSUM at every kind of uint16 csumStart / csumOffset
    (the GPU test_gso_none_paths generator)."""
    rng = np.random.default_rng(4)
    seen = {"compared": 0, "panic": 0}
    for trial in range(120):
        plen = int(rng.integers(1, 3000)) if trial % 3 else int(rng.integers(3000, 65536))
        pkt = rng.integers(0, 256, size=plen, dtype=np.uint8)
        pkt[0] = 0x45
        cs = int(rng.integers(0, plen))
        co = (int(rng.integers(0, plen - 1)) - cs) % 65536 if plen >= 2 and rng.random() < 0.8 \
            else int(rng.integers(0, 65536))
        hdr = np.zeros(10, np.uint8)
        hdr[0] = int(rng.integers(0, 2))
        hdr[6:8] = np.frombuffer(np.uint16(cs).tobytes(), np.uint8)
        hdr[8:10] = np.frombuffer(np.uint16(co).tobytes(), np.uint8)
        bufsize = int(rng.choice([65535 + 16, plen + 16, plen + 15, 100]))
        seen[_virtio_runner(hdr.tobytes() + pkt.tobytes(), 4, bufsize, 16, 0xA5)] += 1
    assert seen["compared"] > 60, seen


def _gro_calls():
    from test_gpu_gro_batch import (bad_checksum_calls, edge_calls, host_scenario_calls, quirk_calls,
                                    tcp_options_calls)
    from test_gpu_wstager import _calls

    calls = []
    for seed in (1, 2, 3, 6, 8):
        calls += _calls(seed)
    return (calls + edge_calls() + bad_checksum_calls() + host_scenario_calls() + tcp_options_calls() +
            quirk_calls())


def test_gro_call_corpus():
    """Every Write call of the GPU GRO corpora through both restatements."""
    from test_gpu_wstager import OFFSET, _mk

    calls = _gro_calls()
    assert len(calls) >= 190
    merged = prepends = errs = 0
    for c, (pkts, cap, can_udp, lo) in enumerate(calls):
        bc, lens = _mk(pkts, cap, OFFSET, lo)
        bp = [b.copy() for b in bc]
        rc_c, tw_c, order_c, nl_c = oracle.handle_gro(bc, list(lens), OFFSET, can_udp)
        rc_p, tw_p, order_p, nl_p = py.run_handle_gro(bp, list(lens), OFFSET, can_udp)
        assert (rc_p, tw_p, order_p, nl_p) == (rc_c, tw_c, order_c, nl_c), c
        for j in range(len(bc)):
            assert np.array_equal(bp[j], bc[j]), (c, j)
        merged += sum(1 for i in range(len(lens)) if nl_c[i] > lens[order_c[i]])
        prepends += order_c != list(range(len(lens)))
        errs += rc_c != 0
    assert merged > 300 and prepends > 10 and errs >= 5, (merged, prepends, errs)


def test_gro_empty_and_invalid_offsets():
    assert py.run_handle_gro([], [], 16, True) == (0, [], [], [])
    b = [np.zeros(100, np.uint8)]
    assert py.run_handle_gro(b, [5], 16, True)[0] == py.ERR_INVALID_OFFSET
    assert py.run_handle_gro(b, [50], 9, True)[0] == py.ERR_INVALID_OFFSET


@pytest.mark.parametrize("raw", [False, True])
def test_gso_short_packets_spare_capacity(raw):
    """Packets shorter than their pseudo-header addresses, read from a buffer
    with spare capacity (tests/gso_cases.py short_cases): both restatements
    read the addresses from the spare bytes, or panic past cap(readBuf)."""
    seen = {"compared": 0, "panic": 0}
    for buf, n_read, nbufs, bufsize, fill, offset, h, is_v6 in gso_cases.short_cases(raw):
        def run_c(bufs):
            rb = np.frombuffer(bytearray(buf), np.uint8).copy()
            if raw:
                return oracle.gso_split(rb, h, bufs, offset, is_v6, n_read=n_read), rb
            return oracle.handle_virtio_read(rb, bufs, offset, n_read=n_read), rb

        def run_py(bufs):
            rb = np.frombuffer(bytearray(buf), np.uint8).copy()
            if raw:
                return py.run_gso_split(rb, h, bufs, offset, is_v6, n_read=n_read), rb
            return py.run_handle_virtio_read(rb, bufs, offset, n_read=n_read), rb

        seen[_gso_compare(run_c, run_py, nbufs, bufsize, fill)] += 1
    assert seen["compared"] >= 100 and seen["panic"] >= 20, seen


def test_checksum_valid_short_packets_spare_capacity():
    """checksumValid's address slices read up to cap(pkt) (gro.go:558-563):
    both restatements agree on short packets with spare capacity, including
    where Go panics (past cap, or iphLen > len)."""
    seen = {"valid": 0, "invalid": 0, "panic": 0}
    for buf, n, iph, proto, v6 in gso_cases.short_valid_cases():
        c = oracle.checksum_valid(buf, iph, proto, v6, n=n)
        try:
            p = py.checksum_valid(py.Slice(np.frombuffer(bytearray(buf), np.uint8), 0, n), iph, proto, v6)
        except py.GoPanic:
            p = py.ERR_OUT_OF_RANGE
        assert c == p, (n, len(buf), iph, proto, v6, c, p)
        seen["panic" if c is not True and c is not False else ("valid" if c else "invalid")] += 1
    assert seen["panic"] >= 100 and seen["invalid"] >= 100, seen


@pytest.mark.parametrize("corpus", ["field_fuzz_calls", "long_run_calls"])
def test_gro_field_fuzz_corpus(corpus):
    """The GRO header-field fuzz calls (tests/gro_cases.py): mutated TOS, TTL,
    fragment bits, lengths, protocol, TCP flags / data offset / ack / window,
    UDP length, truncation, trailing bytes; and the long in-order flows broken
    around 64-packet boundaries -- both restatements agree on status, toWrite,
    slice headers and every buffer byte."""
    import gro_cases
    from test_gpu_wstager import _mk

    calls = getattr(gro_cases, corpus)()
    merged = writes = 0
    for c, (pkts, cap, can_udp, lo) in enumerate(calls):
        bc, lens = _mk(pkts, cap, gro_cases.OFFSET, lo)
        bp = [b.copy() for b in bc]
        rc_c, tw_c, order_c, nl_c = oracle.handle_gro(bc, list(lens), gro_cases.OFFSET, can_udp)
        rc_p, tw_p, order_p, nl_p = py.run_handle_gro(bp, list(lens), gro_cases.OFFSET, can_udp)
        assert (rc_p, tw_p, order_p, nl_p) == (rc_c, tw_c, order_c, nl_c), c
        for j in range(len(bc)):
            assert np.array_equal(bp[j], bc[j]), (c, j)
        merged += sum(1 for i in range(len(lens)) if nl_c[i] > lens[order_c[i]])
        writes += len(tw_c)
    assert merged > 40 and writes > 100, (merged, writes)
