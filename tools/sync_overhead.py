"""Fixed overhead of a short timed region (measurement tool): wall time of
synchronize; K launches over 4 streams; synchronize, against HIP-event GPU time, for small K;
optionally with hipDeviceScheduleSpin set before the context exists (--spin)."""
import argparse
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
p = argparse.ArgumentParser()
p.add_argument("--spin", action="store_true")
p.add_argument("--yield_", action="store_true")
p.add_argument("--streams", type=int, default=4)
p.add_argument("--pool", action="store_true", help="no launch on the default stream")
a = p.parse_args()
if a.spin or a.yield_:
    hip = ctypes.CDLL("libamdhip64.so")
    flag = 1 if a.spin else 2  # hipDeviceScheduleSpin = 1, hipDeviceScheduleYield = 2
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(flag))
    print("hipSetDeviceFlags", flag, "rc", rc)
import torch  # noqa: E402

from seqs_amd import Engine, synth  # noqa: E402

dev = torch.device("cuda:0")
bs = []
for b in range(4):
    buf, off, ln = synth.uniform_batch(65536, 1500, seed=1 + b)
    bs.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)))
e = Engine(0)
streams = ([torch.cuda.Stream(dev) for _ in range(a.streams)] if a.pool else
           [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(a.streams - 1)])
outs = [torch.empty((65536, 2), dtype=torch.int32, device=dev) for _ in range(4)]
sts = [torch.empty((65536,), dtype=torch.uint8, device=dev) for _ in range(4)]


def run(k):
    for i in range(k):
        e.digest_device(*bs[i % 4], out=outs[i % 4], status=sts[i % 4], stream=streams[i % len(streams)])


run(600)
torch.cuda.synchronize()
for k in (0, 1, 2, 3, 4, 5, 6, 8, 12, 20, 20, 200):
    ts = []
    for rep in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(k)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    ts.sort()
    print(f"K={k:4d} wall us: min {ts[0]:8.1f} med {ts[2]:8.1f}  per step (med) {ts[2] / max(k, 1):6.2f}")
