"""One rank of tests/test_multi_gpu.py::test_sharded_gloo_c4, started as a fresh child process.

Every rank builds the same seeded global batch (BASELINE configs[3], C4: 1,048,576 x 1500-B
frames), keeps its round-robin shard (frame i -> rank i mod W), digests it on cuda:0 with the
gfx950 engine (seqs_amd.Engine.digest_device as ShardedDigest's digest_fn) and gathers the
digests to rank 0 over gloo. Rank 0 compares the global-order result with the CPU oracle and
writes {"ok": ..., "n": ...} to the result path.
usage: sharded_worker.py RANK WORLD PORT N RESULT_JSON"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    rank, world, port, n, result = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from seqs_amd import shard, synth

        buf, off, ln = synth.uniform_batch(n, 1500, seed=4)
        b, o, l = shard.shard_batch(buf, off, ln, world, rank)
        dev = torch.device("cuda:0")
        sd = shard.ShardedDigest(world, rank, device=0)  # digest_fn = Engine.digest_device
        res = sd(torch.from_numpy(b).to(dev), torch.from_numpy(o).to(dev), torch.from_numpy(l).to(dev), n_global=n)
        torch.cuda.synchronize()
        if rank == 0:
            from oracle import coracle

            w, s = res
            w = w.numpy().view(np.uint32).reshape(-1, 2)
            dig, est = coracle.digest_batch(buf, off, ln, mtu=0, nthreads=16)
            ok = (np.array_equal(w[:, 0], dig["crc32"]) and np.array_equal(w[:, 1] & 0xFFFF, dig["ip_csum"])
                  and np.array_equal(w[:, 1] >> 16, dig["l4_csum"]) and np.array_equal(s.numpy(), est))
            with open(result, "w") as f:
                json.dump({"ok": bool(ok), "n": int(len(s)), "shard0": int(len(l))}, f)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
