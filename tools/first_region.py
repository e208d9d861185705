"""Consecutive 20-step timed regions (the driver's K) after the bench's warmup, on created
streams (POOL=1) or with the legacy default stream as stream 0 (POOL=0): measurement tool."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from seqs_amd import Engine, synth
dev = torch.device("cuda:0")
bs = []
for b in range(4):
    buf, off, ln = synth.uniform_batch(65536, 1500, seed=1 + b)
    bs.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)))
e = Engine(0)
pool = os.environ.get("POOL", "1") == "1"
streams = [torch.cuda.Stream(dev) for _ in range(4)] if pool else [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(3)]
outs = [torch.empty((65536, 2), dtype=torch.int32, device=dev) for _ in range(4)]
sts = [torch.empty((65536,), dtype=torch.uint8, device=dev) for _ in range(4)]
def run(k, s0=0):
    for i in range(k):
        e.digest_device(*bs[i % 4], out=outs[i % 4], status=sts[i % 4], stream=streams[(s0 + i) % 4])
for i in range(495):
    e.digest_device(*bs[i % 4], out=outs[i % 4], status=sts[i % 4], stream=streams[0])
torch.cuda.synchronize()
run(5)
torch.cuda.synchronize()
ts = []
for rep in range(12):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(20)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e6 / 20)
print("pool" if pool else "default", " ".join(f"{t:.2f}" for t in ts))
