"""Multi-process (gloo, world_size 2, CPU) coverage of the N>1 path: the shard
assignment, shard generation and the max-over-ranks timing reduction that
bench.py uses on the GPUs.  The per-rank compute here is the oracle (the GPU
kernel is the same code on every rank); the point is that the union of the
shards is exactly the single-process batch and every rank's results agree
with it, with no collective on the data path."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from wireguard_amd import shard, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, chunk, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    arena, pkts, kinds, lo, hi = shard.make_global_shard(n_total, rank, world, 1500, "mixed", chunk=chunk)
    valid = oracle.checksum_batch(2, arena, pkts)
    fill = oracle.checksum_batch(1, arena, pkts)
    t = shard.max_over_ranks(float(rank + 1) * 0.5, dist)
    dist.barrier()
    q.put((rank, lo, hi, valid.tobytes(), fill.tobytes(), t, arena[:64].tobytes()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_batch_equals_single_process(world):
    n_total, chunk = 3000, 1024
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, chunk, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # whole batch in one process
    a1, p1, k1, lo1, hi1 = shard.make_global_shard(n_total, 0, 1, 1500, "mixed", chunk=chunk)
    v1 = oracle.checksum_batch(2, a1, p1)
    f1 = oracle.checksum_batch(1, a1, p1)
    assert [(r[1], r[2]) for r in res] == [shard.shard_range(n_total, r, world) for r in range(world)]
    assert b"".join(r[3] for r in res) == v1.tobytes()
    assert b"".join(r[4] for r in res) == f1.tobytes()
    assert v1.all()
    assert all(r[5] == 0.5 * world for r in res)  # every rank sees the slowest rank's time
    assert res[1][6] == a1[(res[1][1]) * 1500:(res[1][1]) * 1500 + 64].tobytes()


def test_shard_ranges_cover_exactly():
    for n in (0, 1, 7, 65536, 1048576):
        for w in (1, 2, 3, 8):
            rs = [shard.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def _worker_mixed(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    arena, pkts, lo, hi = shard.mixed_len_shard(n_total, rank, world)
    valid = oracle.checksum_batch(2, arena, pkts)
    nbytes = int(pkts["len"].astype(np.int64).sum())
    t = torch.tensor([nbytes], dtype=torch.int64)
    dist.all_reduce(t)  # bench-side bookkeeping only (aggregate bytes), not data path
    q.put((rank, lo, hi, valid.tobytes(), nbytes, int(t.item())))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_mixed_length_shards_are_byte_balanced(world):
    """Mixed 64..9000-byte frames: the shards are cut by byte prefix sum, each
    rank's byte count is within one frame of total/world, and the union of the
    ranks' results is the single-process result."""
    n_total = 2000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_mixed, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    arena, pkts, _, lens = shard.make_mixed_len_batch(n_total)
    total = int(lens.sum())
    assert all(r[5] == total for r in res)
    assert res[0][1] == 0 and res[-1][2] == n_total and all(res[i][2] == res[i + 1][1] for i in range(world - 1))
    for r in res:
        assert abs(r[4] - total / world) <= max(lens), (r[4], total / world)
    by_bytes = max(abs(r[4] - total / world) for r in res)
    by_count = max(abs(int(lens[lo:hi].sum()) - total / world)
                   for lo, hi in (shard.shard_range(n_total, r, world) for r in range(world)))
    assert by_bytes <= by_count
    v1 = oracle.checksum_batch(2, arena, pkts)
    assert b"".join(r[3] for r in res) == v1.tobytes() and v1.all()


def test_byte_shards_cover_exactly():
    rng = np.random.default_rng(3)
    for n in (0, 1, 7, 1000):
        lens = rng.integers(1, 9001, size=n)
        for w in (1, 2, 3, 8):
            rs = [shard.shard_range_bytes(lens, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            if n:
                b = [int(lens[l:h].sum()) for l, h in rs]
                assert max(abs(x - lens.sum() / w) for x in b) <= lens.max()
    assert shard.shard_range_bytes(np.full(1048576, 1500), 3, 8) == shard.shard_range(1048576, 3, 8)


def test_shard_is_independent_of_world_size():
    n = 5000
    a2, p2, _, lo, hi = shard.make_global_shard(n, 1, 2, 1500, "mixed", chunk=1024)
    a4, p4, _, lo4, hi4 = shard.make_global_shard(n, 2, 4, 1500, "mixed", chunk=1024)
    assert lo == lo4
    m = hi4 - lo4
    assert np.array_equal(a2[: m * 1500], a4[: m * 1500])
    assert synth.PKT_DTYPE == p2.dtype
