"""GPU parity at BASELINE.json's full sizes, through size-independent
properties (the oracle checks a random sample of each batch bit-exactly):

* cfg2 / cfg3 / cfg5 batches: VALIDATE accepts every synthetic frame and
  rejects exactly the frames that were corrupted on the device; L4_FILL
  reproduces every stored checksum field; an in-place FILL after zeroing the
  fields restores the arena byte for byte (idempotence).
* cfg4 GSO: every produced segment passes VALIDATE (the split kernel's
  checksums checked by the checksum kernel), the segments' payloads
  concatenate back to each super-packet's payload, and sampled jobs match the
  oracle's handleVirtioRead byte for byte.
"""
import numpy as np
import pytest

import oracle
from wireguard_amd import shard, synth
from wireguard_amd.tun import GSO_JOB_DTYPE, MODE_L4_FILL, MODE_VALIDATE, PKT_DTYPE, pkt_off, set_pkt_off

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def S():
    """torch's current stream: kernels are ordered with the torch ops around them."""
    return torch.cuda.current_stream()


def _field_pos(pkts):
    return pkt_off(pkts).astype(np.int64) + pkts["csum_start"].astype(np.int64) + pkts["csum_offset"].astype(np.int64)


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3", "cfg5"])
def test_checksum_batch_properties(dev, cfg):
    n, flen, kinds = {"cfg2": (65536, 1500, "tcp4"), "cfg3": (65536, 9000, "tcp4"),
                      "cfg5": (1048576, 1500, "mixed")}[cfg]
    arena_np, pkts_np, _, _, _ = shard.make_global_shard(n, 0, 1, flen, kinds)
    arena = torch.from_numpy(arena_np).cuda()
    pkts = torch.from_numpy(pkts_np.view(np.uint8)).cuda()
    out = torch.zeros(2 * n, dtype=torch.uint8, device="cuda")
    dev.checksum_batch(MODE_VALIDATE, arena, pkts, n, out, stream=S())
    torch.cuda.synchronize()
    assert bool(out[:n].all().item()), "every synthetic frame must validate"

    # L4_FILL reproduces the stored big-endian fields
    dev.checksum_batch(MODE_L4_FILL, arena, pkts, n, out, stream=S())
    torch.cuda.synchronize()
    got = out.cpu().numpy().view("<u2")[:n]
    fp = _field_pos(pkts_np)
    want = (arena_np[fp].astype(np.uint16) << 8) | arena_np[fp + 1]
    assert np.array_equal(got, want)

    # sampled bit-exact parity with the oracle
    rng = np.random.default_rng(7)
    sample = np.sort(rng.choice(n, size=min(n, 2048), replace=False))
    sub = pkts_np[sample].copy()
    assert np.array_equal(got[sample], oracle.checksum_batch(MODE_L4_FILL, arena_np, sub))

    # corrupt 97 frames on the device: VALIDATE rejects exactly those
    bad = np.sort(rng.choice(n, size=97, replace=False))
    pos = pkt_off(pkts_np)[bad].astype(np.int64) + rng.integers(0, flen, size=97)
    idx = torch.from_numpy(pos).cuda()
    arena[idx] ^= torch.tensor(0x5A, dtype=torch.uint8, device="cuda")
    dev.checksum_batch(MODE_VALIDATE, arena, pkts, n, out, stream=S())
    torch.cuda.synchronize()
    v = out[:n].cpu().numpy()
    assert set(np.nonzero(v == 0)[0].tolist()) == set(bad.tolist())
    arena[idx] ^= torch.tensor(0x5A, dtype=torch.uint8, device="cuda")

    # zero the fields, FILL in place: the arena comes back byte for byte
    fpt = torch.from_numpy(fp).cuda()
    arena[fpt] = 0
    arena[fpt + 1] = 0
    dev.checksum_batch(MODE_L4_FILL, arena, pkts, n, out, inplace=True, stream=S())
    torch.cuda.synchronize()
    assert torch.equal(arena.cpu(), torch.from_numpy(arena_np))


@pytest.mark.parametrize("max_segs", [64, 128])  # 128: len(bufs) of the reference's Read (bench.py cfg4)
def test_gso_cfg4_properties(dev, max_segs):
    n_jobs, total, gso, stride, offset = 256, 65535, 1460, 1536, 16
    vps = [synth.make_super_packet(total, gso, seed=synth.SEED + k) for k in range(n_jobs)]
    jlen = len(vps[0])
    arena_np = np.frombuffer(b"".join(vps), np.uint8).copy()
    jobs = np.zeros(n_jobs, GSO_JOB_DTYPE)
    jobs["off"] = np.arange(n_jobs, dtype=np.uint64) * np.uint64(jlen)
    jobs["len"] = jlen
    d_arena = torch.from_numpy(arena_np).cuda()
    d_jobs = torch.from_numpy(jobs.view(np.uint8)).cuda()
    d_out = torch.zeros(n_jobs * max_segs * stride, dtype=torch.uint8, device="cuda")
    d_sizes = torch.zeros(n_jobs * max_segs, dtype=torch.int32, device="cuda")
    d_count = torch.zeros(n_jobs, dtype=torch.int32, device="cuda")
    d_status = torch.zeros(n_jobs, dtype=torch.int32, device="cuda")
    dev.gso_split_batch(d_arena, d_jobs, n_jobs, d_out, stride, offset, max_segs, d_sizes, d_count, d_status,
                        stream=S())
    torch.cuda.synchronize()
    count = d_count.cpu().numpy()
    assert (d_status.cpu().numpy() == 0).all() and (count == 45).all()
    sizes = d_sizes.cpu().numpy().reshape(n_jobs, max_segs)
    assert (sizes[:, 45:] == 0).all()  # slots past the last segment untouched
    assert not bool(d_out.view(n_jobs, max_segs, stride)[:, 45:, :].any().item())

    # every produced segment validates (checksum kernel over the split kernel's output)
    slots = [(j, i) for j in range(n_jobs) for i in range(45)]
    segs = np.zeros(len(slots), PKT_DTYPE)
    set_pkt_off(segs, [(j * max_segs + i) * stride + offset for j, i in slots])
    segs["len"] = [sizes[j, i] for j, i in slots]
    segs["csum_start"] = 20
    segs["csum_offset"] = 16
    segs["proto"] = 6
    d_segs = torch.from_numpy(segs.view(np.uint8)).cuda()
    valid = torch.zeros(len(slots), dtype=torch.uint8, device="cuda")
    dev.checksum_batch(MODE_VALIDATE, d_out, d_segs, len(slots), valid, stream=S())
    torch.cuda.synchronize()
    assert bool(valid.all().item())

    out_np = d_out.cpu().numpy()
    # payloads concatenate back to the super-packet payload (header 40 B)
    for j in range(0, n_jobs, 17):
        pay = b"".join(out_np[(j * max_segs + i) * stride + offset + 40:
                              (j * max_segs + i) * stride + offset + sizes[j, i]].tobytes() for i in range(45))
        assert pay == vps[j][10 + 40:]
    # sampled jobs bit-exact vs the oracle's handleVirtioRead
    for j in (0, 1, 127, 255):
        bo = [np.zeros(stride, np.uint8) for _ in range(max_segs)]
        rc, cnt, sz = oracle.handle_virtio_read(np.frombuffer(bytearray(vps[j]), np.uint8).copy(), bo, offset)
        assert rc == 0 and cnt == 45
        for i in range(45):
            base = (j * max_segs + i) * stride
            assert sz[i] == sizes[j, i]
            assert np.array_equal(out_np[base + offset: base + offset + sz[i]], bo[i][offset: offset + sz[i]])
