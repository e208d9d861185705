"""Minimal profiling driver: K launches of the digest kernel on one resident batch set
(used under rocprofv3; no oracle, no CPU baseline)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from seqs_amd import Engine, synth  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--config", default="c2")
p.add_argument("--frames", type=int, default=65536)
p.add_argument("--iters", type=int, default=20)
p.add_argument("--kernel", type=int, default=0, help="fs_ctx_set_kernel variant")
a = p.parse_args()
dev = torch.device("cuda:0")
bs = []
for b in range(4):
    buf, off, ln = (synth.uniform_batch(a.frames, 1500, seed=1 + b) if a.config == "c2"
                    else synth.mixed_batch(a.frames, seed=2 + b))
    bs.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)))
e = Engine(0)
e.set_kernel(a.kernel)
out = torch.empty((a.frames, 2), dtype=torch.int32, device=dev)
st = torch.empty((a.frames,), dtype=torch.uint8, device=dev)
# past the automatic choice's initial window (a context's first 16 launches run the mixed-length
# kernel): the summary keeps the kernel the run chose most often
for i in range((32 if a.kernel == 0 else 0) + a.iters):
    e.digest_device(*bs[i % 4], out=out, status=st)
torch.cuda.synchronize()
print("done", a.config, a.frames, a.iters)
