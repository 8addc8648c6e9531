"""GPU parity of wgcs_checksum_batches (many independent batches enqueued by
one call, dealt over streams, optional bracket events): every batch's results
equal the oracle's, whatever the stream count, mode or batch sizes, and bad
stream lists are refused before anything is enqueued."""
import numpy as np
import pytest
import torch

import oracle
from wireguard_amd import synth
from wireguard_amd.tun import MODE_FOLD, MODE_L4_FILL, MODE_VALIDATE, WgcsError

pytestmark = pytest.mark.gpu


def _batches(n_batches, seed):
    out = []
    rng = np.random.default_rng(seed)
    for k in range(n_batches):
        n = int(rng.integers(0, 700))
        flen = int(rng.choice([64, 576, 1500, 4000]))
        arena, pkts, _ = synth.make_batch(max(n, 1), flen, kinds="mixed", seed=seed * 100 + k)
        out.append((arena, pkts[:n]))
    return out


@pytest.mark.parametrize("mode", [MODE_VALIDATE, MODE_L4_FILL, MODE_FOLD])
@pytest.mark.parametrize("n_streams", [0, 1, 2, 3])
def test_batches_match_oracle(dev, mode, n_streams):
    host = _batches(7, seed=10 + mode * 4 + n_streams)
    d = []
    for arena, pkts in host:
        d_arena = torch.from_numpy(arena).cuda()
        d_pkts = torch.from_numpy(pkts.view(np.uint8).copy()).cuda() if len(pkts) else torch.zeros(16, dtype=torch.uint8,
                                                                                                      device="cuda")
        ini = np.arange(len(pkts), dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        d_ini = torch.from_numpy(ini.view(np.uint8).copy()).cuda() if mode == MODE_FOLD and len(pkts) else None
        d_out = torch.full((max(len(pkts), 1) * 2,), 0xEE, dtype=torch.uint8, device="cuda")
        d.append((d_arena, d_pkts, len(pkts), d_out, d_ini, ini))
    bl = dev.batch_list([(a, p, n, o, i) for a, p, n, o, i, _ in d])
    streams = [torch.cuda.Stream() for _ in range(n_streams)]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    e1.record()
    torch.cuda.synchronize()
    dev.checksum_batches(mode, bl, streams, e0, e1)
    torch.cuda.synchronize()
    assert e0.elapsed_time(e1) >= 0.0
    for (arena, pkts), (_, _, n, d_out, _, ini) in zip(host, d):
        if n == 0:
            continue
        want = oracle.checksum_batch(mode, arena, pkts, ini if mode == MODE_FOLD else None)
        dt = np.uint8 if mode == MODE_VALIDATE else np.uint16
        got = d_out.cpu().numpy().view(dt)[:n]
        assert np.array_equal(got, want)


def test_batches_reject_bad_stream_list(dev):
    arena, pkts, _ = synth.make_batch(8, 1500, kinds="tcp4")
    d_arena = torch.from_numpy(arena).cuda()
    d_pkts = torch.from_numpy(pkts.view(np.uint8).copy()).cuda()
    d_out = torch.zeros(16, dtype=torch.uint8, device="cuda")
    bl = dev.batch_list([(d_arena, d_pkts, 8, d_out)])
    with pytest.raises(WgcsError) as ei:
        dev.checksum_batches(MODE_VALIDATE, bl, [torch.cuda.Stream() for _ in range(17)])
    assert ei.value.code == -1
    bad = dev.batch_list([(d_arena, 0, 8, d_out)])  # NULL descriptors with n > 0
    with pytest.raises(WgcsError):
        dev.checksum_batches(MODE_VALIDATE, bad, [])
    torch.cuda.synchronize()
    assert int(d_out.sum().item()) == 0  # nothing was enqueued
