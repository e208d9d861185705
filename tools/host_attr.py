#!/usr/bin/env python3
"""Attribution of one host-staged call (fs_digest_batch_host) of the reference's benchmark shape
(65,536 x 47-B frames). Measurement tool.

  run:  python3 tools/host_attr.py run <clk.json> [--pageable-desc] [--calls K]
        K calls in the Go binding's arrangement (frames + descriptors pinned, results pageable),
        each call's host clocks (CLOCK_MONOTONIC / BOOTTIME) around it written to clk.json
  attr: python3 tools/host_attr.py attr <trace dir> <clk.json>
        lines a rocprofv3 --kernel-trace --memory-copy-trace --hip-trace of `run` up with those
        clocks and prints, per phase, the median over the calls: when each copy and the kernel
        start and end after the call's start, and the host time spent in the HIP calls.

  rocprofv3 --kernel-trace --memory-copy-trace --hip-trace --output-format csv -d <dir> -- \\
      python3 tools/host_attr.py run <clk.json>
"""
import csv
import glob
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def clocks():
    return {"mono": time.clock_gettime_ns(time.CLOCK_MONOTONIC),
            "boot": time.clock_gettime_ns(getattr(time, "CLOCK_BOOTTIME", time.CLOCK_MONOTONIC))}


def run(clk, calls=50, pageable_desc=False):
    import numpy as np

    from seqs_amd import Engine, synth
    from seqs_amd.framesum import DIGEST_DTYPE

    eng = Engine(0)
    buf, off, ln = synth.hello_batch(65536, seed=77)
    n = len(ln)
    pin = eng.host_empty(buf.shape, np.uint8)
    pin[:] = buf
    if pageable_desc:
        poff, plen = off.astype(np.uint64), ln.astype(np.uint32)
    else:
        poff = eng.host_empty(off.shape, np.uint64)
        poff[:] = off
        plen = eng.host_empty(ln.shape, np.uint32)
        plen[:] = ln
    out = np.zeros(n, dtype=DIGEST_DTYPE)
    st = np.zeros(n, dtype=np.uint8)
    lib, ctx = eng.lib, eng._ctx
    import ctypes

    args = (ctx, pin.ctypes.data_as(ctypes.c_void_p), pin.nbytes, poff.ctypes.data_as(ctypes.c_void_p),
            plen.ctypes.data_as(ctypes.c_void_p), n, 0, out.ctypes.data_as(ctypes.c_void_p),
            st.ctypes.data_as(ctypes.c_void_p))
    for _ in range(20):
        assert lib.fs_digest_batch_host(*args) == 0
    recs = []
    for _ in range(calls):
        t0 = clocks()
        rc = lib.fs_digest_batch_host(*args)
        t1 = clocks()
        assert rc == 0
        recs.append({"t0": t0, "t1": t1})
        time.sleep(0.002)  # calls apart in the trace
    with open(clk, "w") as f:
        json.dump(recs, f)
    eng.close()
    print("calls", calls, "median us", statistics.median((r["t1"]["mono"] - r["t0"]["mono"]) / 1e3 for r in recs))


def rows(tdir, pattern):
    out = []
    for f in glob.glob(os.path.join(tdir, "**", pattern), recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def attr(tdir, clk):
    recs = json.load(open(clk))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "kernel " + r.get("Kernel_Name", "")[:24])
          for r in rows(tdir, "*kernel_trace.csv")]
    cps = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
            "copy " + r.get("Direction", r.get("Operation", "")) + " " + r.get("Size", r.get("Bytes", "")))
           for r in rows(tdir, "*memory_copy_trace.csv")]
    api = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Function", ""))
           for r in rows(tdir, "*hip_api_trace.csv")]
    best = None
    for ck in ("mono", "boot"):
        inside = sum(1 for s, e, _ in ks for r in recs if r["t0"][ck] <= s <= r["t1"][ck])
        if best is None or inside > best[1]:
            best = (ck, inside)
    ck = best[0]
    print(f"trace clock {ck}: {best[1]} kernels inside {len(recs)} calls")
    phases = {}
    apis = {}
    walls = []
    for r in recs:
        t0, t1 = r["t0"][ck], r["t1"][ck]
        walls.append((t1 - t0) / 1e3)
        seen = {}
        for s, e, name in sorted(ks + cps):
            if t0 <= s <= t1:
                k = name
                seen[k] = seen.get(k, 0) + 1
                k = f"{k} #{seen[k]}"
                phases.setdefault(k, []).append(((s - t0) / 1e3, (e - t0) / 1e3))
        for s, e, name in api:
            if t0 <= s <= t1:
                a = apis.setdefault(name, [0, 0.0, []])
                a[0] += 1
                a[1] += (e - s) / 1e3
                a[2].append((s - t0) / 1e3)
    med = statistics.median
    print(f"call wall: median {med(walls):.1f} us (min {min(walls):.1f})")
    for k, v in sorted(phases.items(), key=lambda kv: med(x[0] for x in kv[1])):
        print(f"  {k:<44s} start {med(x[0] for x in v):7.1f}  end {med(x[1] for x in v):7.1f}  "
              f"dur {med(x[1] - x[0] for x in v):6.1f} us  ({len(v)} calls)")
    print("HIP API per call (count, host us, first start):")
    for name, (c, tot, starts) in sorted(apis.items(), key=lambda kv: -kv[1][1]):
        print(f"  {name:<32s} {c / len(recs):6.1f}  {tot / len(recs):7.1f} us  first at {min(starts):6.1f}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], calls=int(sys.argv[sys.argv.index("--calls") + 1]) if "--calls" in sys.argv else 50,
            pageable_desc="--pageable-desc" in sys.argv)
    else:
        attr(sys.argv[2], sys.argv[3])
