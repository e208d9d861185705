"""Start-of-region ramp (measurement tool): after a warm-up, bursts of K digest launches over
`--streams` streams, each burst between two synchronizes -- the shape of a short timed region.
Run it under `rocprofv3 --kernel-trace --output-format csv`, then `--analyze <kernel_trace.csv>`
prints, per burst, every kernel's start and end relative to the burst's first start."""
import argparse
import csv
import os
import sys
import time

p = argparse.ArgumentParser()
p.add_argument("--streams", type=int, default=5)
p.add_argument("--k", type=int, default=8)
p.add_argument("--bursts", type=int, default=6)
p.add_argument("--gap-us", type=float, default=0.0, help="host sleep between a burst's launches")
p.add_argument("--wake", action="store_true", help="an empty kernel on every stream right before each burst")
p.add_argument("--analyze", default=None)
a = p.parse_args()

if a.analyze:
    rows = list(csv.DictReader(open(a.analyze)))
    rows = [r for r in rows if "digest_kernel" in r["Kernel_Name"] or "wake" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # bursts: separated by > 50 us of idle
    bursts, cur, last_end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last_end is not None and s - last_end > 50000:
            bursts.append(cur)
            cur = []
        cur.append((s, e, r["Kernel_Name"][:30], r.get("Queue_Id", "?")))
        last_end = max(last_end or 0, e)
    bursts.append(cur)
    for b in bursts[-a.bursts:]:
        t0 = b[0][0]
        span = max(e for _, e, _, _ in b) - t0
        print(f"burst: {len(b)} kernels, span {span / 1000:.1f} us")
        for s, e, n, q in b:
            print(f"   q{q:>3} start {(s - t0) / 1000:7.2f}  end {(e - t0) / 1000:7.2f}  dur {(e - s) / 1000:6.2f}  {n}")
    sys.exit(0)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from seqs_amd import Engine, synth  # noqa: E402

dev = torch.device("cuda:0")
bs = []
for b in range(4):
    buf, off, ln = synth.uniform_batch(65536, 1500, seed=1 + b)
    bs.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)))
e = Engine(0)
streams = [torch.cuda.Stream(dev) for _ in range(a.streams)]
nslot = max(2, a.streams)
outs = [torch.empty((65536, 2), dtype=torch.int32, device=dev) for _ in range(nslot)]
sts = [torch.empty((65536,), dtype=torch.uint8, device=dev) for _ in range(nslot)]
tiny = torch.zeros(1, device=dev)


def run(k, gap=0.0):
    for i in range(k):
        e.digest_device(*bs[i % 4], out=outs[i % nslot], status=sts[i % nslot], stream=streams[i % len(streams)])
        if gap:
            t = time.perf_counter() + gap * 1e-6
            while time.perf_counter() < t:
                pass


run(600)
torch.cuda.synchronize()
for rep in range(a.bursts):
    torch.cuda.synchronize()
    time.sleep(0.001)
    if a.wake:
        for s in streams:
            with torch.cuda.stream(s):
                tiny.add_(1.0)
    t0 = time.perf_counter()
    run(a.k, a.gap_us)
    torch.cuda.synchronize()
    print(f"burst {rep}: wall {(time.perf_counter() - t0) * 1e6:.1f} us")
