"""Where the segment kernel (variant 3) wins: tiles that mix a frame far longer than the piece kernel's
mode B covers (at most 6 passes of 16 768-B pieces, ~74 KB) with short frames. Each tile: one frame of
GIANT bytes (default 128 KB) and 15 frames of 64 B, packed back to back, 1,024 tiles; every variant
timed over 20 launches (HIP events, one stream) and checked bit-exact against the C oracle."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from oracle import coracle  # noqa: E402
from seqs_amd import Engine, split_digests  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--giant", type=int, default=131072)
p.add_argument("--tiles", type=int, default=1024)
a = p.parse_args()
rng = np.random.default_rng(5)
ln = np.tile(np.array([a.giant] + [64] * 15, dtype=np.int32), a.tiles)
off = np.zeros(len(ln), np.int64)
off[1:] = np.cumsum(ln[:-1].astype(np.int64))
buf = rng.integers(0, 256, int(off[-1] + ln[-1] + 64), dtype=np.uint8)
dig, est = coracle.digest_batch(buf, off, ln, nthreads=16)
dev = torch.device("cuda:0")
tb, to, tl = torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)
for v in (2, 3, 4):
    e = Engine(0)
    e.set_kernel(v)
    out, st = e.digest_device(tb, to, tl)
    torch.cuda.synchronize()
    crc, ipc, l4c = split_digests(out.cpu().numpy())
    ok = bool((crc == dig["crc32"]).all() and (ipc == dig["ip_csum"]).all() and (l4c == dig["l4_csum"]).all()
              and (st.cpu().numpy() == est).all())
    for _ in range(5):
        e.digest_device(tb, to, tl, out=out, status=st)
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    for _ in range(20):
        e.digest_device(tb, to, tl, out=out, status=st)
    s1.record()
    torch.cuda.synchronize()
    us = s0.elapsed_time(s1) * 1e3 / 20
    print(json.dumps({"variant": v, "kernel": e.last_kernel(), "bit_exact": ok, "us_per_launch": round(us, 1),
                      "GiB_s": round(float(ln.astype(np.int64).sum()) / (us * 1e-6) / 2**30, 1),
                      "frames": int(len(ln)), "giant": a.giant}))
    e.close()
