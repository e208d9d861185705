"""Where a short timed region's time goes (measurement tool): the bench's C2 loop (device
pre-warm over every stream, then 12 consecutive K-step regions, each synchronize; K launches;
synchronize), printing every region's host clocks so a rocprofv3 kernel trace of the same run
can be lined up with them: `rocprofv3 --kernel-trace --output-format csv -d <dir> -- python3
tools/region_trace.py` then `python3 tools/region_trace.py --analyse <dir> <this run's stdout>`."""
import argparse
import csv
import glob
import json
import os
import sys
import time

p = argparse.ArgumentParser()
p.add_argument("--streams", type=int, default=5)
p.add_argument("--steps", type=int, default=20)
p.add_argument("--regions", type=int, default=12)
p.add_argument("--spin", action="store_true", help="hipSetDeviceFlags(hipDeviceScheduleSpin) before the context")
p.add_argument("--analyse", nargs=2, metavar=("TRACE_DIR", "STDOUT"))
a = p.parse_args()

CLOCKS = {"mono": time.CLOCK_MONOTONIC, "boot": getattr(time, "CLOCK_BOOTTIME", time.CLOCK_MONOTONIC)}


def clocks():
    return {k: time.clock_gettime_ns(c) for k, c in CLOCKS.items()}


if a.analyse:
    tdir, out = a.analyse
    rows = []
    for f in glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "digest_kernel" in r.get("Kernel_Name", ""):
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    regs = [json.loads(line) for line in open(out) if line.startswith("{")]
    for ck in CLOCKS:
        inside = sum(1 for s, e in rows for r in regs if r["t0"][ck] <= s <= r["t1"][ck])
        print(f"clock {ck}: {inside} dispatches inside regions (expect {len(regs) * regs[0]['k']})")
    ck = max(CLOCKS, key=lambda c: sum(1 for s, e in rows for r in regs if r["t0"][c] <= s <= r["t1"][c]))
    for r in regs:
        t0, t1 = r["t0"][ck], r["t1"][ck]
        ks = [(s, e) for s, e in rows if t0 <= s <= t1]
        if not ks:
            continue
        first_s, last_e = ks[0][0], max(e for _, e in ks)
        dur = [(e - s) / 1e3 for s, e in ks]
        print(f"region wall {(t1 - t0) / 1e3:7.1f} us | to 1st start {(first_s - t0) / 1e3:5.1f} | kernel span "
              f"{(last_e - first_s) / 1e3:6.1f} | last end to host {(t1 - last_e) / 1e3:5.1f} | n {len(ks)} | "
              f"dur first {dur[0]:.1f} med {sorted(dur)[len(dur) // 2]:.1f} max {max(dur):.1f} | starts "
              + " ".join(f"{(s - first_s) / 1e3:.0f}" for s, _ in ks))
    sys.exit(0)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

if a.spin:  # the HIP runtime torch loaded (same soname), before torch creates the context
    import ctypes
    rc = ctypes.CDLL("libamdhip64.so.7").hipSetDeviceFlags(ctypes.c_uint(1))
    assert rc == 0, rc

from seqs_amd import Engine, synth  # noqa: E402

dev = torch.device("cuda:0")
bs = []
for b in range(4):
    buf, off, ln = synth.uniform_batch(65536, 1500, seed=1 + b)
    bs.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)))
e = Engine(0)
streams = [torch.cuda.Stream(dev) for _ in range(a.streams)]
ns = a.streams
outs = [torch.empty((65536, 2), dtype=torch.int32, device=dev) for _ in range(ns)]
sts = [torch.empty((65536,), dtype=torch.uint8, device=dev) for _ in range(ns)]


def run(k, base=0):
    for i in range(k):
        j = base + i
        e.digest_device(*bs[j % 4], out=outs[j % ns], status=sts[j % ns], stream=streams[j % ns])


run(500)
torch.cuda.synchronize()
run(5)
torch.cuda.synchronize()
for rep in range(a.regions):
    torch.cuda.synchronize()
    c0 = clocks()
    t0 = time.perf_counter()
    run(a.steps, 5 + rep * a.steps)
    th = time.perf_counter()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    c1 = clocks()
    print(json.dumps({"spin": a.spin, "hsa_interrupt": os.environ.get("HSA_ENABLE_INTERRUPT"), "k": a.steps, "t0": c0, "t1": c1, "us_per_step": (t1 - t0) * 1e6 / a.steps,
                      "host_enqueue_us": (th - t0) * 1e6}), flush=True)
