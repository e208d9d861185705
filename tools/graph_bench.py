"""Launch-overhead experiment (measurement tool): the bench's C2 step sequence issued eagerly
(Python loop, 1 or 2 streams) vs replayed from a captured HIP graph (chain on one stream, or
two independent branches)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from seqs_amd import Engine, synth  # noqa: E402

dev = torch.device("cuda:0")
n = 65536
e = Engine(0)
bs = []
for b in range(4):
    buf, off, ln = synth.uniform_batch(n, 1500, seed=1 + b)
    bs.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)))
nbytes = int(ln.astype(np.int64).sum())
outs = [torch.empty((n, 2), dtype=torch.int32, device=dev) for _ in range(2)]
sts = [torch.empty((n,), dtype=torch.uint8, device=dev) for _ in range(2)]
s0 = torch.cuda.current_stream(dev)
s1 = torch.cuda.Stream(dev)
K = 400


def report(name, t):
    print(f"{name:40s} {t / K * 1e6:7.2f} us/step  {nbytes * K / t / 2**30:8.1f} GiB/s", flush=True)


def eager(nstreams):
    ss = [s0, s1][:nstreams]
    for i in range(K):
        s = ss[i % nstreams]
        fb, fo, fl = bs[i % 4]
        e.digest_device(fb, fo, fl, out=outs[i % 2], status=sts[i % 2], stream=s)


for ns in (1, 2):
    eager(ns)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eager(ns)
    torch.cuda.synchronize()
    report(f"eager, {ns} stream(s), no events", time.perf_counter() - t0)

G = 8  # launches per graph
for mode in ("chain", "two-branch"):
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(dev)
    with torch.cuda.graph(g, stream=cap):
        if mode == "chain":
            for i in range(G):
                fb, fo, fl = bs[i % 4]
                e.digest_device(fb, fo, fl, out=outs[i % 2], status=sts[i % 2], stream=cap)
        else:
            side = torch.cuda.Stream(dev)
            side.wait_stream(cap)
            for i in range(G):
                s = cap if i % 2 == 0 else side
                fb, fo, fl = bs[i % 4]
                e.digest_device(fb, fo, fl, out=outs[i % 2], status=sts[i % 2], stream=s)
            cap.wait_stream(side)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K // G):
        g.replay()
    torch.cuda.synchronize()
    report(f"graph of {G}, {mode}", time.perf_counter() - t0)
e.close()
