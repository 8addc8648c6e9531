"""GPU parity: outer-UDP message batching (splitMessages / coalesceMessages,
conn/bind.go:542-662) through the C ABI vs the oracle -- every buffer byte,
N, Addr, nPackets / nMsgs, status code and control message.

Host-call API (wgcs_split_messages / wgcs_coalesce_messages) on seeded random
recvmmsg / Send batches, then the device-resident batch API on many batches
at once, compared batch by batch."""
import numpy as np
import pytest

import oracle
from conn_cases import Msg, clone_msgs, coalesce_case, gro_cmsg, split_case
from wireguard_amd import conn

pytestmark = pytest.mark.gpu


def _code(err):
    return 0 if err is None else err.code


# ------------------------------------------------------------------ host API
@pytest.mark.parametrize("seed", range(40))
def test_split_messages_host(dev, seed):
    rng = np.random.default_rng(5000 + seed)
    n_msgs = int(rng.choice([128, 128, 8, 16, 3]))
    first = None if n_msgs == 128 else int(rng.integers(0, n_msgs))
    buf_len = int(rng.choice([65535, 65535, 4096, 1500]))
    msgs, first = split_case(rng, n_msgs=n_msgs, first=first, buf_len=buf_len)
    mo, mp = clone_msgs(msgs), clone_msgs(msgs)
    npk_o, rc_o = oracle.split_messages(mo, first)
    npk_p, err = conn.split_messages(dev, mp, first)
    assert (npk_p, _code(err)) == (npk_o, rc_o)
    for k in range(n_msgs):
        assert mp[k].n == mo[k].n, k
        assert mp[k].addr == mo[k].addr, k
        assert np.array_equal(mp[k].buf, mo[k].buf), k


def test_split_messages_host_readat_126(dev):
    """The receive path's exact shape: 2 GRO datagrams at 126/127."""
    rng = np.random.default_rng(7)
    msgs, first = split_case(rng, n_msgs=128, kinds=("gro",))
    assert first == 126
    mo, mp = clone_msgs(msgs), clone_msgs(msgs)
    npk_o, rc_o = oracle.split_messages(mo, first)
    assert rc_o == 0 and npk_o > 0
    npk, err = conn.split_messages(dev, mp, first)
    assert err is None and npk == npk_o
    for k in range(128):
        assert mp[k].n == mo[k].n and np.array_equal(mp[k].buf, mo[k].buf), k


@pytest.mark.parametrize("seed", range(40))
def test_coalesce_messages_host(dev, seed):
    rng = np.random.default_rng(6000 + seed)
    bufs, lens, src, v6, oob_cap = coalesce_case(rng)
    bo = [b.copy() for b in bufs]
    bp = [b.copy() for b in bufs]
    mo = [Msg(np.zeros(1, np.uint8), oob_cap) for _ in bufs]
    mp = [conn.Message(None, oob_cap) for _ in bufs]
    nm_o = oracle.coalesce_messages(mo, bo, lens, src, "ep", v6)
    nm_p = conn.coalesce_messages(dev, mp, bp, lens, src, "ep", v6)
    assert nm_p == nm_o
    for m in range(nm_o):
        fo = next(j for j, b in enumerate(bo) if b is mo[m].buf)
        fp = next(j for j, b in enumerate(bp) if b is mp[m].buf)
        assert fp == fo and mp[m].buf_len == mo[m].buf_len, m
        assert mp[m].oob_len == mo[m].oob_len and np.array_equal(mp[m].oob, mo[m].oob), m
    for j in range(len(bufs)):
        assert np.array_equal(bp[j], bo[j]), j


def test_coalesce_messages_host_empty(dev):
    assert conn.coalesce_messages(dev, [], [], [], b"", "ep", False) == 0


# --------------------------------------------------------- device batch API
def _split_batch_ref(msgs_list, first):
    outs = []
    for msgs in msgs_list:
        mo = clone_msgs(msgs)
        npk, rc = oracle.split_messages(mo, first)
        outs.append((npk, rc, mo))
    return outs


def _split_batch_check(dev, cases, n_msgs, first, buf_len, in_stride):
    import torch

    B = len(cases)
    ns = n_msgs - first
    h_in = np.zeros((B * ns, in_stride), dtype=np.uint8)
    n_in = np.zeros(B * n_msgs, dtype=np.int32)
    gso = np.zeros(B * n_msgs, dtype=np.int32)
    for b, msgs in enumerate(cases):
        for s, m in enumerate(msgs):
            n_in[b * n_msgs + s] = m.n
            if s >= first:
                h_in[b * ns + s - first, :buf_len] = m.buf
                g, rc = oracle.get_gso_size(m.oob[: m.nn].tobytes())
                gso[b * n_msgs + s] = rc if rc else g
    out_stride = 65536
    d_in = torch.from_numpy(h_in).cuda()
    d_n = torch.from_numpy(n_in).cuda()
    d_g = torch.from_numpy(gso).cuda()
    d_out = torch.zeros((B * n_msgs, out_stride), dtype=torch.uint8, device="cuda")
    d_nout = torch.zeros(B * n_msgs, dtype=torch.int32, device="cuda")
    d_src = torch.zeros(B * n_msgs, dtype=torch.int32, device="cuda")
    d_cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
    d_st = torch.zeros(B, dtype=torch.int32, device="cuda")
    rc = dev.lib.wgcs_split_messages_batch(dev.h, d_in.data_ptr(), in_stride, buf_len, d_n.data_ptr(), d_g.data_ptr(),
                                           n_msgs, first, B, d_out.data_ptr(), out_stride, d_nout.data_ptr(),
                                           d_src.data_ptr(), d_cnt.data_ptr(), d_st.data_ptr(), None)
    assert rc == 0
    dev.sync()
    out, nout, src = d_out.cpu().numpy(), d_nout.cpu().numpy(), d_src.cpu().numpy()
    cnt, st = d_cnt.cpu().numpy(), d_st.cpu().numpy()
    for b, (npk, rco, mo) in enumerate(_split_batch_ref(cases, first)):
        assert (cnt[b], st[b]) == (npk, rco), b
        for k in range(n_msgs):
            q = b * n_msgs + k
            assert nout[q] == mo[k].n, (b, k)
            if k < npk:
                assert mo[k].addr == f"addr{src[q]}", (b, k)
                assert np.array_equal(out[q, : mo[k].n], mo[k].buf[: mo[k].n]), (b, k)
            else:
                assert src[q] == -1


@pytest.mark.parametrize("seed,in_stride", [(0, 65536), (1, 65536), (2, 65536), (3, 65541), (4, 65664 + 56)])
def test_split_messages_batch(dev, seed, in_stride):
    """Landing slots on 128-B lines and off them (odd strides): the rows that
    share a source line through LDS see every phase of it."""
    rng = np.random.default_rng(7000 + seed)
    n_msgs, first, buf_len = 128, 126, 65535
    cases = [split_case(rng, n_msgs=n_msgs, first=first, buf_len=buf_len)[0] for _ in range(16)]
    _split_batch_check(dev, cases, n_msgs, first, buf_len, in_stride)


@pytest.mark.parametrize("in_stride", [65536, 65539])
def test_split_messages_batch_gso_edges(dev, in_stride):
    """gsoSize at the edges of the kernel's shared-line path (round 6: rows of
    one message share 128-B source lines for 128 <= gsoSize <= 1,650, others
    copy directly): 127 / 128 / 129, 1,649 / 1,650 / 1,651, 3,000, with short
    tails and with several messages' packets in one 16-row block."""
    rng = np.random.default_rng(7100 + in_stride)
    n_msgs, first, buf_len = 128, 124, 65535
    gs = (127, 128, 129, 1649, 1650, 1651, 3000, 1452)
    cases = []
    for b in range(12):
        msgs = []
        for s in range(n_msgs):
            m = Msg(rng.integers(0, 256, buf_len, dtype=np.uint8))
            m.addr = f"addr{s}"
            msgs.append(m)
        for s in range(first, n_msgs):
            g = gs[(b * 4 + s) % len(gs)]
            segs = int(rng.integers(1, max(2, min(40, 60000 // g))))
            n = min(g * segs - int(rng.integers(0, g)), buf_len)
            m = msgs[s]
            m.n = max(n, 1)
            ctl = gro_cmsg(g)
            m.oob[: len(ctl)] = np.frombuffer(ctl, dtype=np.uint8)
            m.nn = len(ctl)
        cases.append(msgs)
    _split_batch_check(dev, cases, n_msgs, first, buf_len, in_stride)


@pytest.mark.parametrize("seed", range(3))
def test_coalesce_messages_batch(dev, seed):
    import torch

    rng = np.random.default_rng(8000 + seed)
    B, max_bufs, stride = 12, 128, 65536
    cases = [coalesce_case(rng, nbufs=int(rng.integers(1, max_bufs + 1))) for _ in range(B)]
    v6 = bool(rng.integers(2))
    h = np.zeros((B * max_bufs, stride), dtype=np.uint8)
    lens = np.zeros(B * max_bufs, dtype=np.int32)
    caps = np.zeros(B * max_bufs, dtype=np.int32)
    nb = np.zeros(B, dtype=np.int32)
    for b, (bufs, ln, _, _, _) in enumerate(cases):
        nb[b] = len(bufs)
        for j, buf in enumerate(bufs):
            q = b * max_bufs + j
            h[q, : len(buf)] = buf
            lens[q] = ln[j]
            caps[q] = len(buf)
    d = torch.from_numpy(h).cuda()
    d_lens, d_caps, d_nb = (torch.from_numpy(x).cuda() for x in (lens, caps, nb))
    d_nm = torch.zeros(B, dtype=torch.int32, device="cuda")
    d_first, d_len, d_gso = (torch.zeros(B * max_bufs, dtype=torch.int32, device="cuda") for _ in range(3))
    rc = dev.lib.wgcs_coalesce_messages_batch(dev.h, d.data_ptr(), stride, 65535, d_caps.data_ptr(),
                                              d_lens.data_ptr(), d_nb.data_ptr(), max_bufs, B, int(v6),
                                              d_nm.data_ptr(), d_first.data_ptr(), d_len.data_ptr(),
                                              d_gso.data_ptr(), None)
    assert rc == 0
    dev.sync()
    got, nm = d.cpu().numpy(), d_nm.cpu().numpy()
    first, mlen, gso = d_first.cpu().numpy(), d_len.cpu().numpy(), d_gso.cpu().numpy()
    for b, (bufs, ln, src, _, _) in enumerate(cases):
        bo = [x.copy() for x in bufs]
        mo = [Msg(np.zeros(1, np.uint8), 64) for _ in bufs]
        nmo = oracle.coalesce_messages(mo, bo, ln, b"", "ep", v6)
        assert nm[b] == nmo, b
        for m in range(nmo):
            q = b * max_bufs + m
            f = next(j for j, x in enumerate(bo) if x is mo[m].buf)
            assert (first[q], mlen[q]) == (f, mo[m].buf_len), (b, m)
            g = int.from_bytes(mo[m].oob[16:18].tobytes(), "little") if mo[m].oob_len == 24 else -1
            assert gso[q] == g, (b, m)
        for j, x in enumerate(bo):
            assert np.array_equal(got[b * max_bufs + j, : len(x)], x), (b, j)
