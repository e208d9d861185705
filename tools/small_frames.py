"""Throughput for uniform batches of small and medium frames (measurement tool): the per-tile
work (descriptors, geometry, header DMA, parse, combine, finish) against the frame bytes."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from seqs_amd import Engine, synth  # noqa: E402

dev = torch.device("cuda:0")
e = Engine(0)
for L, n in ((64, 1 << 20), (128, 1 << 19), (256, 1 << 18), (576, 1 << 17), (1500, 65536), (9000, 16384)):
    bs = []
    for b in range(4):
        buf, off, ln = synth.uniform_batch(n, L, seed=1 + b)
        bs.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)))
    out = torch.empty((n, 2), dtype=torch.int32, device=dev)
    st = torch.empty((n,), dtype=torch.uint8, device=dev)
    for i in range(300):
        e.digest_device(*bs[i % 4], out=out, status=st)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    K = 300
    for i in range(K):
        e.digest_device(*bs[i % 4], out=out, status=st)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / K
    nbytes = n * L
    print(f"{L:5d}-B frames x {n:8d}: {us:8.2f} us/batch  {nbytes / us / 1e3:7.1f} GB/s  {n / us:8.1f} Mframes/s", flush=True)
e.close()
