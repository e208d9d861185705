"""Per-wave phase timeline from an FS_STAMPS diagnostic build (measurement tool).
Usage: FRAMESUM_LIB=seqs_amd/lib/diag/libframesum_st4.so python tools/stamps.py [--config c2]"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from seqs_amd import Engine, synth  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--config", default="c2")
p.add_argument("--frames", type=int, default=65536)
a = p.parse_args()
dev = torch.device("cuda:0")
bs = []
for b in range(4):
    buf, off, ln = (synth.uniform_batch(a.frames, 1500, seed=1 + b) if a.config == "c2"
                    else synth.mixed_batch(a.frames, seed=2 + b))
    bs.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)))
e = Engine(0)
out = torch.empty((a.frames, 2), dtype=torch.int32, device=dev)
st = torch.empty((a.frames,), dtype=torch.uint8, device=dev)
for i in range(8):
    e.digest_device(*bs[i % 4], out=out, status=st)
torch.cuda.synchronize()
arr = np.zeros(8192 * 8, dtype=np.uint64)
rc = e.lib.fs_debug_read_stamps(arr.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(arr.nbytes))
assert rc == 0, rc
nw = min(8192, (a.frames + 15) // 16)
s = arr.reshape(8192, 8)[:nw].astype(np.int64)
names = ["fill+desc->sync", "main loop", "combine", "finalize"]
print(f"waves={nw}  (cycles, s_memtime ticks)")
for k, nm in enumerate(names):
    d = s[:, k + 1] - s[:, k]
    print(f"  {nm:18s} median {int(np.median(d)):8d}  p10 {int(np.percentile(d, 10)):8d}  p90 {int(np.percentile(d, 90)):8d}")
tot = s[:, 4] - s[:, 0]
blk = np.arange(nw) // 16
ml = s[:, 2] - s[:, 1]
print("  main loop median by blockIdx % 8 (XCD group):",
      [int(np.median(ml[(blk % 8) == x])) for x in range(8)])
print("  main loop median by wave-in-block:", [int(np.median(ml[(np.arange(nw) % 16) == w])) for w in range(16)])
st = s[:, 0] - s[:, 0].min()
print("  start skew (ticks) p50/p90/max:", int(np.median(st)), int(np.percentile(st, 90)), int(st.max()))
print(f"  {'wave total':18s} median {int(np.median(tot)):8d}  p10 {int(np.percentile(tot, 10)):8d}  p90 {int(np.percentile(tot, 90)):8d}")
