"""Packet-level sharding across the GPUs of one node.

Per-packet checksums and per-super-packet GSO splits are independent, so a
batch is cut into contiguous packet ranges, one per rank (one process per
GPU), with NO collective on the data path.  torch.distributed is used only
for the bench's barrier and its max-over-ranks timing reduction.

Global batches are generated in fixed 65,536-packet chunks, each seeded by
its chunk index, so a rank's shard is byte-identical to the same packet range
of the whole batch whatever the world size (parity across N).
"""
from __future__ import annotations

import os

import numpy as np

from . import synth

CHUNK = 65536


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced [lo, hi) packet range of `rank` out of `world`."""
    assert 0 <= rank < world
    return n * rank // world, n * (rank + 1) // world


def shard_range_bytes(lens, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [lo, hi) packet range of `rank` balanced by BYTES (mixed
    lengths): the cuts are the packet boundaries nearest to the prefix-sum
    targets k * total / world, so each rank's bytes differ from total / world
    by at most one packet.  Equal lengths give shard_range."""
    assert 0 <= rank < world
    cum = np.concatenate([[0], np.cumsum(np.asarray(lens, dtype=np.int64))])
    total = int(cum[-1])

    def cut(r):
        if r == 0:
            return 0
        if r == world:
            return len(cum) - 1
        t = total * r // world
        i = int(np.searchsorted(cum, t, side="left"))
        if i > 0 and t - cum[i - 1] < cum[i] - t:
            i -= 1
        return i

    return cut(rank), cut(rank + 1)


LEN_CHOICES = (64, 576, 1280, 1500, 4096, 9000)


def make_mixed_len_batch(n: int, seed: int = synth.SEED):
    """n seeded frames of mixed kinds AND mixed lengths (LEN_CHOICES), packed
    back to back; returns (arena, pkts, kinds, lens)."""
    rng = np.random.default_rng(seed)
    lens = rng.choice(np.array(LEN_CHOICES, np.int64), size=n)
    kinds = rng.integers(0, 4, size=n)
    kinds[(lens < 64)] = synth.KIND_UDP4
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    arena = np.zeros(int(lens.sum()) + 64, np.uint8)
    for L in np.unique(lens):
        idx = np.nonzero(lens == L)[0]
        fr = synth.build_frames(kinds[idx], int(L), rng)
        for j, i in enumerate(idx):
            arena[int(offs[i]): int(offs[i]) + int(L)] = fr[j]
    pkts = synth.describe(kinds, lens, offs)
    return arena, pkts, kinds, lens


def mixed_len_shard(n_total: int, rank: int, world: int, seed: int = synth.SEED):
    """Rank's byte-balanced shard of make_mixed_len_batch(n_total): (arena,
    pkts rebased to the shard's arena, lo, hi)."""
    arena, pkts, _, lens = make_mixed_len_batch(n_total, seed)
    lo, hi = shard_range_bytes(lens, rank, world)
    from .tun import pkt_off, set_pkt_off

    offs = pkt_off(pkts)
    a0 = int(offs[lo]) if lo < n_total else len(arena) - 64
    a1 = int(offs[hi - 1]) + int(lens[hi - 1]) if hi > lo else a0
    sub = pkts[lo:hi].copy()
    set_pkt_off(sub, offs[lo:hi] - np.uint64(a0))
    return np.concatenate([arena[a0:a1], np.zeros(64, np.uint8)]), sub, lo, hi


def make_global_shard(n_total: int, rank: int, world: int, frame_len: int = 1500, kinds: str = "mixed",
                      seed: int = synth.SEED, chunk: int = CHUNK):
    """Packets [lo, hi) of the seeded global batch of n_total frames.
    Returns (arena, pkts, kinds, lo, hi) with offsets local to the arena."""
    lo, hi = shard_range_bytes(np.full(n_total, frame_len, np.int64), rank, world)
    m = hi - lo
    arena = np.zeros(m * frame_len + 64, np.uint8)
    chunks = list(range(lo // chunk, (hi + chunk - 1) // chunk))

    def one(c):  # chunk c's frames that fall in [lo, hi), written straight into the shard's arena
        cn = min(chunk, n_total - c * chunk)
        a, _, k = synth.make_batch(cn, frame_len, kinds=kinds, seed=seed + c, pad=0)
        s0 = max(lo - c * chunk, 0)
        s1 = min(hi - c * chunk, cn)
        d0 = c * chunk + s0 - lo
        arena[d0 * frame_len: (d0 + s1 - s0) * frame_len] = a[s0 * frame_len: s1 * frame_len]
        return k[s0:s1]

    # chunks are independent (each seeded by its index): numpy releases the GIL
    # in the bulk of the work, so a few threads cut the 1M-frame build ~3x
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(max_workers=max(1, min(8, len(chunks), len(os.sched_getaffinity(0))))) as ex:
        kparts = list(ex.map(one, chunks))
    k = np.concatenate(kparts) if kparts else np.zeros(0, np.int64)
    pkts = synth.describe(k, frame_len, np.arange(m, dtype=np.uint64) * np.uint64(frame_len))
    return arena, pkts, k, lo, hi


def dist_env():
    """(world, rank, local_rank) from the torchrun environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def gather_floats(value: float, dist, device=None) -> list[float]:
    """Every rank's `value`, in rank order (bench bookkeeping, not data path):
    each rank fills its own slot of a zero vector and one SUM all-reduce
    combines them."""
    if dist is None:
        return [float(value)]
    import torch

    if device is None:
        device = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.zeros(dist.get_world_size(), dtype=torch.float64, device=device)
    t[dist.get_rank()] = float(value)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(x) for x in t.cpu().tolist()]


def parse_cpulist(s: str) -> set[int]:
    """Linux cpulist text ("0-3,8,10-11") -> set of CPU ids."""
    cpus: set[int] = set()
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            cpus.update(range(int(a), int(b) + 1))
        else:
            cpus.add(int(part))
    return cpus


def gpu_local_cpus(props, sysfs: str = "/sys/bus/pci/devices") -> tuple[set[int] | None, str]:
    """NUMA-local CPUs of the GPU whose torch device properties are `props`
    (pci_domain_id / pci_bus_id / pci_device_id), from the PCI device's
    local_cpulist; (None, why) when it cannot be found."""
    try:
        bdf = f"{int(props.pci_domain_id):04x}:{int(props.pci_bus_id):02x}:{int(props.pci_device_id):02x}.0"
    except (AttributeError, TypeError, ValueError):
        return None, "device properties carry no PCI address"
    path = os.path.join(sysfs, bdf, "local_cpulist")
    try:
        with open(path) as f:
            return parse_cpulist(f.read()), bdf
    except OSError:
        return None, f"{path} unreadable"


def bind_numa_local(torch, device: int, apply: bool = True) -> dict:
    """Bind every thread of this process to the CPUs NUMA-local to GPU
    `device` (intersected with the CPUs the process may use), so the pinned
    host memory the end-to-end leg allocates afterwards is first touched on
    the GPU's socket.  In-process (os.sched_setaffinity on each task of
    /proc/self/task): never an exec.  Returns what was done, for the line."""
    allowed = set(os.sched_getaffinity(0))
    local, where = gpu_local_cpus(torch.cuda.get_device_properties(device))
    info = {"allowed_cpus": len(allowed), "pci": where}
    if local is None:
        info["applied"] = False
        return info
    both = sorted(allowed & local)
    info["numa_local_cpus"] = len(local)
    info["bound_cpus"] = len(both)
    if not both or not apply:
        info["applied"] = False
        if not both:
            info["why_not"] = "no NUMA-local CPU inside this process's cpuset"
        return info
    tids = [int(t) for t in os.listdir("/proc/self/task")] if os.path.isdir("/proc/self/task") else [0]
    for tid in tids:
        try:
            os.sched_setaffinity(tid, both)
        except OSError:  # a thread that exited meanwhile
            pass
    info["applied"] = True
    return info


def max_over_ranks(value: float, dist, device=None) -> float:
    """The slowest rank's time (the bench's timing reduction; not data path)."""
    if dist is None:
        return value
    import torch

    if device is None:  # RCCL reduces device tensors; gloo (CPU tests, rehearsals) host tensors
        device = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
