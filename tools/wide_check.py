"""Wide one-pass kernel (variant 6) against the one-pass kernel (variant 4): bit-exact outputs on
C2 / C3 / C4-style batches, and the kernel time of each (HIP events around K launches on one
stream), alternated (measurement + check tool)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from seqs_amd import Engine, synth  # noqa: E402

dev = torch.device("cuda:0")
e = Engine(0)


def batch(kind, seed):
    if kind == "c2":
        return synth.uniform_batch(65536, 1500, seed=seed)
    if kind == "c3":
        return synth.mixed_batch(65536, seed=seed)
    raise ValueError(kind)


def run(v, tb, to, tl, out, st):
    e.set_kernel(v)
    e.digest_device(tb, to, tl, out=out, status=st)


for kind in sys.argv[1:] or ["c2", "c3"]:
    bs = []
    for b in range(4):
        buf, off, ln = batch(kind, 1 + b)
        bs.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)))
    n = int(bs[0][2].numel())
    nbytes = int(bs[0][2].cpu().numpy().astype(np.int64).sum())
    outs = {v: (torch.empty((n, 2), dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.uint8, device=dev))
            for v in (4, 6, 2)}
    for v in (4, 6, 2):
        run(v, *bs[0], *outs[v])
    torch.cuda.synchronize()
    same = all(torch.equal(outs[4][i], outs[6][i]) for i in range(2))
    bad = int((outs[4][0] != outs[6][0]).any(dim=1).sum()) + int((outs[4][1] != outs[6][1]).sum())
    print(f"{kind}: wide == one-pass: {same} (mismatching frames {bad})", flush=True)
    if not same:
        idx = torch.nonzero((outs[4][0] != outs[6][0]).any(dim=1) | (outs[4][1] != outs[6][1])).flatten()[:5]
        for i in idx.tolist():
            print("  frame", i, "len", int(bs[0][2][i]), "a", outs[4][0][i].tolist(), int(outs[4][1][i]), "w",
                  outs[6][0][i].tolist(), int(outs[6][1][i]), flush=True)
    s = torch.cuda.Stream(dev)
    K = 400
    res = {4: [], 6: [], 2: []}
    for rep in range(3):
        for v in (4, 6, 2):
            e.set_kernel(v)
            o, st = outs[v]
            with torch.cuda.stream(s):
                for i in range(50):
                    e.digest_device(*bs[i % 4], out=o, status=st, stream=s)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                for i in range(K):
                    e.digest_device(*bs[i % 4], out=o, status=st, stream=s)
                b.record(s)
            torch.cuda.synchronize()
            res[v].append(a.elapsed_time(b) / K * 1e3)
    for v in (4, 6, 2):
        us = min(res[v])
        print(f"{kind} variant {v}: {us:.2f} us per launch ({nbytes / us / 1e3:.0f} GB/s; runs {[round(x, 2) for x in res[v]]})",
              flush=True)
