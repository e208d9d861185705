import os, sys, time
import numpy as np, torch
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
from seqs_amd import Engine, synth
dev = torch.device("cuda:0"); n = 65536
e = Engine(0)
bs = []
for b in range(4):
    buf, off, ln = synth.mixed_batch(n, seed=2 + b)
    bs.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)))
outs = [torch.empty((n, 2), dtype=torch.int32, device=dev) for _ in range(2)]
sts = [torch.empty((n,), dtype=torch.uint8, device=dev) for _ in range(2)]
s = torch.cuda.current_stream(dev)
K = 200
def run(tag):
    for i in range(20):
        fb, fo, fl = bs[i % 4]; e.digest_device(fb, fo, fl, out=outs[i % 2], status=sts[i % 2], stream=s)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter(); a.record(s)
    for i in range(K):
        fb, fo, fl = bs[i % 4]; e.digest_device(fb, fo, fl, out=outs[i % 2], status=sts[i % 2], stream=s)
    t1 = time.perf_counter(); b.record(s)
    torch.cuda.synchronize(); t2 = time.perf_counter()
    print(f"{tag}: enqueue {1e6*(t1-t0)/K:.2f} us/step, wall {1e6*(t2-t0)/K:.2f} us/step, events {1e3*a.elapsed_time(b)/K:.2f} us/step", flush=True)
for r in range(3): run(f"run{r}")
e.close()
