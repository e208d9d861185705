"""Short-region A/B (measurement tool): the driver's 20-step C2 region (5 warmup steps, then
K timed steps over created streams, synchronize on both sides), with different launch paths
and end-of-region waits, alternated within one process so box drift hits every variant alike.

  base       bench.py's step: Engine.digest_device, torch.cuda.synchronize()
  fast       ctypes arguments built before the region, lib.fs_digest_batch called directly
  fast_spin  fast, then an event per stream, polled until all have completed, then synchronize
  fast_ssync fast, then every stream synchronized, then synchronize
  <v>@S      the same over S streams (default 5)

--spin sets hipDeviceScheduleSpin before the HIP context exists (a separate process)."""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
p = argparse.ArgumentParser()
p.add_argument("--spin", action="store_true")
p.add_argument("--reps", type=int, default=15)
p.add_argument("--steps", type=int, default=20)
p.add_argument("--warmup", type=int, default=5)
p.add_argument("--variants", default="base,fast,fast_spin,fast_ssync")
p.add_argument("--tag", default="")
p.add_argument("--fresh", type=int, default=0,
               help="start every region with a burst of this many launches and a synchronize, as bench.py's "
                    "pre-warm (its timed region is the first after the burst)")
a = p.parse_args()
if a.spin:
    hip = ctypes.CDLL("libamdhip64.so")
    print("hipSetDeviceFlags(spin) rc", hip.hipSetDeviceFlags(ctypes.c_uint(1)), flush=True)
import torch  # noqa: E402

from seqs_amd import Engine, synth  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(0)
n = 65536
bs = []
for b in range(4):
    buf, off, ln = synth.uniform_batch(n, 1500, seed=1 + b)
    bs.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)))
nbytes = int(ln.astype("int64").sum())
e = Engine(0)
lib, ctx = e.lib, e._ctx
NS = 8
streams = [torch.cuda.Stream(dev) for _ in range(NS)]
slab = (9 * n + 255) // 256 * 256
flat = torch.empty(NS * slab, dtype=torch.uint8, device=dev)
outs = [flat[k * slab: k * slab + 8 * n].view(torch.int32).view(n, 2) for k in range(NS)]
sts = [flat[k * slab + 8 * n: k * slab + 9 * n] for k in range(NS)]
vp = ctypes.c_void_p


def fast_args(i, ns):
    fb, fo, fl = bs[i % 4]
    k = i % ns
    return (ctx, vp(fb.data_ptr()), vp(fo.data_ptr()), vp(fl.data_ptr()), n, 0, vp(outs[k].data_ptr()),
            vp(sts[k].data_ptr()), vp(streams[k].cuda_stream))


def run_base(i0, k, ns):
    for i in range(i0, i0 + k):
        fb, fo, fl = bs[i % 4]
        e.digest_device(fb, fo, fl, mtu=0, out=outs[i % ns], status=sts[i % ns], stream=streams[i % ns])


def region(v, i0):
    name, _, s = v.partition("@")
    ns = int(s) if s else 5
    K = a.steps
    name, *mods = name.split("+")
    if a.fresh:
        for i in range(a.fresh):
            fb, fo, fl = bs[i % 4]
            e.digest_device(fb, fo, fl, out=outs[i % NS], status=sts[i % NS], stream=streams[i % NS])
        torch.cuda.synchronize()
    if "rehearse" in mods:  # an untimed region first, the same steps, settle and synchronize
        run_base(i0, K, ns)
        evs0 = [torch.cuda.Event() for _ in range(ns)]
        for q in range(ns):
            evs0[q].record(streams[q])
        while not all(ev.query() for ev in evs0):
            pass
        torch.cuda.synchronize()
    if "prespin" in mods:  # the host spin before the warmup steps (the GPU busy until the region)
        t = time.perf_counter()
        while time.perf_counter() - t < 3e-3:
            pass
    # warmup steps (untimed), as the bench
    run_base(i0, a.warmup, ns)
    if "settlewarm" in mods:  # wait for the warmup by polling events (the host thread never sleeps)
        evw = [torch.cuda.Event() for _ in range(ns)]
        for q in range(ns):
            evw[q].record(streams[q])
        while not all(ev.query() for ev in evw):
            pass
    torch.cuda.synchronize()
    pre = [fast_args(i, ns) for i in range(i0 + a.warmup, i0 + a.warmup + K)] if name != "base" else None
    spin = name == "fast_spin" or "settle" in mods
    evs = [torch.cuda.Event() for _ in range(ns)] if spin else None
    f = lib.fs_digest_batch
    torch.cuda.synchronize()
    if "hostspin" in mods:  # keep the host core busy for 3 ms (no GPU work)
        t = time.perf_counter()
        while time.perf_counter() - t < 3e-3:
            pass
    t0 = time.perf_counter()
    if name == "base":
        run_base(i0 + a.warmup, K, ns)
    else:
        for args in pre:
            f(*args)
    if spin:
        for q in range(ns):
            evs[q].record(streams[q])
        while not all(ev.query() for ev in evs):
            pass
    elif name == "fast_ssync":
        for q in range(ns):
            streams[q].synchronize()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6


# pre-warm over every stream
for i in range(600):
    fb, fo, fl = bs[i % 4]
    e.digest_device(fb, fo, fl, out=outs[i % NS], status=sts[i % NS], stream=streams[i % NS])
torch.cuda.synchronize()
variants = a.variants.split(",")
res = {v: [] for v in variants}
i0 = 0
for r in range(a.reps):
    for v in (variants if r % 2 == 0 else variants[::-1]):
        res[v].append(region(v, i0))
        i0 += a.warmup + a.steps
    if r % 5 == 4:
        print(f"rep {r + 1}/{a.reps}", flush=True)
for v in variants:
    ts = sorted(res[v])
    med = statistics.median(ts)
    print(json.dumps({"tag": a.tag, "spin": a.spin, "variant": v, "steps": a.steps, "med_us": round(med, 1),
                      "min_us": round(ts[0], 1), "p75_us": round(ts[(3 * len(ts)) // 4], 1),
                      "med_gibs": round(nbytes * a.steps / (med * 1e-6) / 2**30, 1),
                      "us_per_step_med": round(med / a.steps, 2),
                      "reps_us": [round(x, 1) for x in res[v]]}), flush=True)
