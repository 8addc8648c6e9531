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


def make_global_shard(n_total: int, rank: int, world: int, frame_len: int = 1500, kinds: str = "mixed",
                      seed: int = synth.SEED, chunk: int = CHUNK):
    """Packets [lo, hi) of the seeded global batch of n_total frames.
    Returns (arena, pkts, kinds, lo, hi) with offsets local to the arena."""
    lo, hi = shard_range(n_total, rank, world)
    parts, kparts = [], []
    c0 = lo // chunk
    for c in range(c0, (hi + chunk - 1) // chunk):
        cn = min(chunk, n_total - c * chunk)
        a, p, k = synth.make_batch(cn, frame_len, kinds=kinds, seed=seed + c, pad=0)
        s0 = max(lo - c * chunk, 0)
        s1 = min(hi - c * chunk, cn)
        parts.append(a[s0 * frame_len: s1 * frame_len])
        kparts.append(k[s0:s1])
    arena = np.concatenate(parts + [np.zeros(64, np.uint8)])
    k = np.concatenate(kparts) if kparts else np.zeros(0, np.int64)
    m = hi - lo
    pkts = synth.describe(k, frame_len, np.arange(m, dtype=np.uint64) * np.uint64(frame_len))
    return arena, pkts, k, lo, hi


def dist_env():
    """(world, rank, local_rank) from the torchrun environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


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
