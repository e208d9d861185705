"""Multi-process (world_size 2, gloo, CPU) coverage of the sharded path: round-robin
partition, padded digest gather to rank 0, restoration of global frame order.
The per-shard digest is the CPU oracle here (no GPU in this container); on the GPU
box the same ShardedDigest runs the gfx950 engine over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from seqs_amd import shard


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_digest(buf, off, ln, mtu):
    from oracle import coracle

    dig, st = coracle.digest_batch(buf.numpy(), off.numpy(), ln.numpy(), mtu=mtu)
    words = np.zeros((len(dig), 2), dtype=np.uint32)
    words[:, 0] = dig["crc32"]
    words[:, 1] = dig["ip_csum"].astype(np.uint32) | (dig["l4_csum"].astype(np.uint32) << 16)
    return torch.from_numpy(words.view(np.int32)), torch.from_numpy(st)


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import framegen

        # the same global batch on every rank (seeded); each rank keeps only its shard
        frames = framegen.edge_batch(3, n_random=n)
        from seqs_amd.framesum import pack_frames

        buf, off, ln = pack_frames(frames, align=1)
        b, o, l = shard.shard_batch(buf, off.astype(np.int64), ln.astype(np.int32), world, rank)
        sd = shard.ShardedDigest(world, rank, digest_fn=_oracle_digest)
        res = sd(torch.from_numpy(b), torch.from_numpy(o), torch.from_numpy(l), n_global=len(frames))
        if rank == 0:
            w, s = res
            full_w, full_s = _oracle_digest(torch.from_numpy(buf), torch.from_numpy(off.astype(np.int64)),
                                            torch.from_numpy(ln.astype(np.int32)), 0)
            q.put((bool(torch.equal(w, full_w) and torch.equal(s, full_s)), len(frames)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 120), (3, 61)])
def test_sharded_gather_matches_single(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ok, nf = q.get(timeout=10)
    assert ok and nf > n


def test_partition_is_exact():
    for n in (0, 1, 7, 64, 65537):
        for w in (1, 2, 3, 4, 8):
            idx = np.concatenate([shard.local_indices(n, w, r) for r in range(w)])
            assert np.array_equal(np.sort(idx), np.arange(n))
            assert sum(shard.shard_count(n, w, r) for r in range(w)) == n
