"""Multi-GPU sharding of a frame batch: one process per GPU.

A global batch of N frames is partitioned round-robin — frame i lives on rank
i mod W at local index i div W — so every rank digests an independent shard
with no data-path collective. The only collective is the gather of the 8-byte
digests + 1-byte verdicts to rank 0 (torch.distributed "nccl" = RCCL over
xGMI on MI355X; "gloo" for the CPU tests), after which rank 0 restores global
frame order. Frames are independent (eth/crc.go:12 — CRC791 is per call), so
sharded results are element-wise identical to single-GPU results.
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np


def local_indices(n_global: int, world: int, rank: int) -> np.ndarray:
    """Global frame indices owned by `rank`: rank, rank + W, rank + 2W, ..."""
    return np.arange(rank, n_global, world, dtype=np.int64)


def shard_count(n_global: int, world: int, rank: int) -> int:
    return (n_global - rank + world - 1) // world if rank < n_global else 0


def shard_batch(buf: np.ndarray, offsets: np.ndarray, lengths: np.ndarray, world: int, rank: int):
    """Host-side shard of a packed batch: (buf, offsets, lengths) holding only this rank's frames,
    repacked contiguously (the 4-byte alignment of each frame start is kept)."""
    idx = local_indices(len(lengths), world, rank)
    ln = lengths[idx].astype(np.int64)
    step = (ln + 3) // 4 * 4
    off = np.zeros(len(idx), dtype=np.int64)
    if len(idx) > 1:
        off[1:] = np.cumsum(step[:-1])
    total = int(off[-1] + step[-1]) if len(idx) else 0
    out = np.zeros(total + 16, dtype=np.uint8)
    for j, i in enumerate(idx):
        o, L = int(offsets[i]), int(lengths[i])
        out[off[j] : off[j] + L] = buf[o : o + L]
    return out, off, lengths[idx].astype(np.int32)


def gather_digests(words, status, world: int, rank: int, n_global: int, group=None, async_op: bool = False):
    """Gather every rank's (n_local, 2) int32 digest words and (n_local,) uint8 verdicts to rank 0.

    Shards differ by at most one frame, so each is padded to ceil(N / W) rows for the
    fixed-size collective. Returns (handles, finish) where finish() -> (words, status)
    in GLOBAL frame order on rank 0 (None elsewhere); with async_op=False the gather
    has already completed.
    """
    import torch
    import torch.distributed as dist

    m = (n_global + world - 1) // world
    n_local = words.shape[0]
    if n_local < m:
        pw = torch.zeros((m, 2), dtype=words.dtype, device=words.device)
        pw[:n_local] = words
        ps = torch.zeros((m,), dtype=status.dtype, device=status.device)
        ps[:n_local] = status
        words, status = pw, ps
    gw = [torch.empty_like(words) for _ in range(world)] if rank == 0 else None
    gs = [torch.empty_like(status) for _ in range(world)] if rank == 0 else None
    h = [dist.gather(words, gw, dst=0, group=group, async_op=async_op),
         dist.gather(status, gs, dst=0, group=group, async_op=async_op)]

    def finish():
        if async_op:
            for x in h:
                x.wait()
        if rank != 0:
            return None
        # interleave: global frame j*W + r = local frame j of rank r
        w = torch.stack(gw, dim=1).reshape(world * m, 2)[:n_global]
        s = torch.stack(gs, dim=1).reshape(world * m)[:n_global]
        return w, s

    return h, finish


class ShardedDigest:
    """Digest this rank's shard and gather the digests to rank 0 in global frame order.

    `digest_fn(frames, offsets, lengths, mtu) -> (words (n,2) int32, status (n,) uint8)`
    defaults to the gfx950 engine (seqs_amd.Engine.digest_device); the CPU tests inject
    the oracle instead so the distribution logic is covered with gloo.
    """

    def __init__(self, world: int, rank: int, digest_fn: Optional[Callable] = None, device: int = 0, group=None):
        self.world, self.rank, self.group = world, rank, group
        if digest_fn is None:
            from .framesum import Engine

            self._engine = Engine(device)
            digest_fn = self._engine.digest_device
        self.digest_fn = digest_fn

    def __call__(self, frames, offsets, lengths, n_global: int, mtu: int = 0):
        import torch.distributed as dist

        words, status = self.digest_fn(frames, offsets, lengths, mtu)
        if words.is_cuda and dist.get_backend(self.group) == "gloo":
            # gloo gathers host tensors: the engine's device results travel as CPU copies
            words, status = words.cpu(), status.cpu()
        _, finish = gather_digests(words, status, self.world, self.rank, n_global, self.group)
        return finish()
