"""GPU, N > 1 processes: the product's HIP path run by 2 ranks (one process
each, gloo for the bench-side bookkeeping, both on cuda:0 of the 1-GPU box)
on byte-balanced shards of a mixed-length batch -- the union of the ranks'
results equals the oracle on the whole batch.  No collective touches the data
(SURVEY.md §8(e))."""
import os
import socket

import numpy as np
import pytest

import oracle
from wireguard_amd import shard, synth

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, n_total, q):
    import torch  # noqa: F401  (one HIP runtime per process)
    import torch.distributed as dist

    from wireguard_amd.tun import MODE_L4_FILL, MODE_VALIDATE, Device

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = Device(0)
    arena, pkts, lo, hi = shard.mixed_len_shard(n_total, rank, world)
    v = dev.checksum_batch_host(MODE_VALIDATE, arena, pkts)
    f = dev.checksum_batch_host(MODE_L4_FILL, arena, pkts)
    dev.close()
    dist.barrier()
    q.put((rank, lo, hi, v.tobytes(), f.tobytes()))
    dist.destroy_process_group()


def test_two_ranks_hip_path_on_byte_shards():
    import torch.multiprocessing as mp

    world, n_total = 2, 3000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    arena, pkts, _, _ = shard.make_mixed_len_batch(n_total)
    assert b"".join(r[3] for r in res) == oracle.checksum_batch(2, arena, pkts).tobytes()
    assert b"".join(r[4] for r in res) == oracle.checksum_batch(1, arena.copy(), pkts).tobytes()


def test_cfg1_batch(dev):
    """BASELINE.json configs[0]: 1,024 x 1500-B UDP/IPv4 frames -- VALIDATE,
    L4_FILL and IP4HDR on the GPU vs the oracle, bit-exact."""
    from wireguard_amd.tun import MODE_IP4HDR, MODE_L4_FILL, MODE_VALIDATE

    arena, pkts, _ = synth.make_batch(1024, 1500, kinds="udp4")
    for mode in (MODE_VALIDATE, MODE_L4_FILL, MODE_IP4HDR):
        got = dev.checksum_batch_host(mode, arena.copy(), pkts)
        want = oracle.checksum_batch(mode, arena.copy(), pkts)
        assert np.array_equal(got, want), mode
    assert dev.checksum_batch_host(MODE_VALIDATE, arena, pkts).all()


def _rccl_rank(port, q):
    """bench.py's N > 1 bookkeeping on RCCL, one rank: init with device_id (as
    bench.py binds one GPU per rank), barrier, the device-tensor max over
    ranks, and the device-resident checksum path in between."""
    import torch
    import torch.distributed as dist

    from wireguard_amd.tun import MODE_VALIDATE, Device

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    dev = Device(0)
    arena, pkts, _ = synth.make_batch(512, 1500, kinds="tcp4")
    d_arena = torch.from_numpy(arena).cuda()
    d_pkts = torch.from_numpy(pkts.view(np.uint8)).cuda()
    out = torch.zeros(len(pkts), dtype=torch.uint8, device="cuda")
    dist.barrier()
    dev.checksum_batch(MODE_VALIDATE, d_arena, d_pkts, len(pkts), out)
    torch.cuda.synchronize()
    dist.barrier()
    m = shard.max_over_ranks(1.25, dist)  # device tensor all_reduce(MAX) on RCCL
    ok = bool(out.all().item())
    dev.close()
    dist.destroy_process_group()
    q.put((m, ok))


def test_rccl_single_rank_bookkeeping():
    """The RCCL calls bench.py makes at N > 1 (init_process_group("nccl",
    device_id=...), barrier, all_reduce MAX of a cuda tensor), exercised on the
    1-GPU box with one rank; the 8-GPU runs use the same calls with 8."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_rank, args=(_free_port(), q))
    p.start()
    m, ok = q.get(timeout=180)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert m == 1.25 and ok
