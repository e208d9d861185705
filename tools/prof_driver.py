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
p.add_argument("--op", choices=["digest", "fill"], default="digest",
               help="fill: fs_fill_batch FS_FILL_CSUM|FS_FCS_APPEND on C2 frames with 4 spare bytes each")
a = p.parse_args()
dev = torch.device("cuda:0")
bs = []
for b in range(4):
    buf, off, ln = (synth.uniform_batch(a.frames, 1500, seed=1 + b) if a.config == "c2"
                    else synth.mixed_batch(a.frames, seed=2 + b))
    if a.op == "fill":  # 4 spare bytes after every frame (the FCS), 4-byte aligned
        import numpy as np

        step = (ln.astype(np.int64) + 4 + 3) // 4 * 4
        noff = np.zeros_like(off)
        noff[1:] = np.cumsum(step[:-1])
        nbuf = np.zeros(int(noff[-1] + step[-1]) + 16, np.uint8)
        nbuf[(noff[:, None] + np.arange(int(ln.max()))[None, :]).ravel()] = \
            buf[(off[:, None] + np.arange(int(ln.max()))[None, :]).ravel()] if (ln == ln[0]).all() else 0
        buf, off = nbuf, noff
    bs.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)))
e = Engine(0)
e.set_kernel(a.kernel)
out = torch.empty((a.frames, 2), dtype=torch.int32, device=dev)
st = torch.empty((a.frames,), dtype=torch.uint8, device=dev)
# past the automatic choice's initial window (a context's first 16 launches run the mixed-length
# kernel): the summary keeps the kernel the run chose most often
for i in range((32 if a.kernel == 0 else 0) + a.iters):
    if a.op == "fill":
        e.fill_device(*bs[i % 4], flags=3, out=out, status=st)
    else:
        e.digest_device(*bs[i % 4], out=out, status=st)
torch.cuda.synchronize()
print("done", a.config, a.frames, a.iters)
