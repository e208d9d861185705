"""One rank of bench.py's N > 1 loop on CPU (tests/test_bench_dist.py starts two of these).

bench.GPU is swapped for CPU stand-ins: tensors on the CPU, streams and events as no-ops and
wall clocks, the process group over gloo, and an engine stand-in whose "digest" writes a
frame's length and its rank into the digest words with verdict 0, and whose de-interleave is
the plan's map in torch. Everything else is bench.py's own code: the rounds, the point-to-point
transfers and their run-time checks, the C4 record and its global-order check.
Test infrastructure only: nothing here is measured."""
import contextlib
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from seqs_amd import shard_slab_bytes  # noqa: E402


class _Stream:
    def wait_stream(self, other):
        pass


class _Event:
    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class FakeEngine:
    def __init__(self, local):
        self.rank = int(os.environ.get("RANK", "0"))

    def set_kernel(self, v):
        pass

    def set_workgroups(self, k):
        pass

    def last_kernel(self):
        return 4

    def close(self):
        pass

    def digest_device(self, frames, offsets, lengths, mtu=0, out=None, status=None, stream=None):
        out[:, 0] = lengths.to(torch.int32)
        out[:, 1] = self.rank + 1
        status.zero_()
        return out, status

    digest_fcs_device = digest_device

    def prepare_digest(self, frames, offsets, lengths, mtu=0, out=None, status=None, stream=None, op="digest",
                       flags=1):
        # the bench's prepared-call path (Engine.prepare_digest): one closure per (batch, slot, stream)
        self.prepared = getattr(self, "prepared", 0) + 1
        return lambda: self.digest_device(frames, offsets, lengths, mtu, out, status, stream)

    def fill_device(self, frames, offsets, lengths, flags=0, mtu=0, out=None, status=None, stream=None):
        return self.digest_device(frames, offsets, lengths, mtu, out, status, stream)

    def deinterleave_device(self, gathered, nshards, n, out=None, status=None, stream=None):
        m = (n + nshards - 1) // nshards
        sb = shard_slab_bytes(n, nshards)
        i = torch.arange(n)
        r, j = i % nshards, i // nshards
        at = (r * sb + 8 * j)[:, None] + torch.arange(8)[None, :]
        out.copy_(gathered[at].contiguous().view(torch.int32).view(n, 2))
        status.copy_(gathered[r * sb + 8 * m + j])
        return out, status


class CpuOps(bench.GpuOps):
    backend = "gloo"

    def device(self, local):
        return torch.device("cpu")

    def init_group(self, dist_, dev, **kw):
        dist_.init_process_group("gloo", **kw)

    def stream(self, dev):
        return _Stream()

    def use(self, s):
        return contextlib.nullcontext()

    def sync(self):
        pass

    def event(self):
        return _Event()

    def empty_cache(self):
        pass

    def settle(self, streams):
        pass

    def mark(self, s):
        return None

    def wait_event(self, s, e):
        pass

    def engine(self, local):
        return FakeEngine(local)


if __name__ == "__main__":
    bench.GPU = CpuOps()
    sys.argv = ["bench.py"] + sys.argv[1:]
    bench.main()
