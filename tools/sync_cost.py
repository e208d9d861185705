"""Measurement aid: where the fixed time of a short timed region goes.

For each runtime setting (a child process per setting; this parent never touches the GPU) it
times, on the C2 batch over 5 streams as bench.py runs it:
  - an idle torch.cuda.synchronize() (nothing queued),
  - the host cost of one step's call (Engine.digest_device, and a prepared call with its ctypes
    arguments built once: Engine.prepare_digest),
  - a 20-step region: t0 -> enqueued -> settled (events polled) -> synchronized.
Settings: the defaults, ROC_ACTIVE_WAIT_TIMEOUT values, hipSetDeviceFlags(hipDeviceScheduleSpin /
Yield) before torch creates the device context.

  python tools/sync_cost.py            # every setting
  python tools/sync_cost.py --child k  # one setting (internal)
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SETTINGS = [
    ("default", {}, None),
    ("ROC_ACTIVE_WAIT_TIMEOUT=0", {"ROC_ACTIVE_WAIT_TIMEOUT": "0"}, None),
    ("ROC_ACTIVE_WAIT_TIMEOUT=200", {"ROC_ACTIVE_WAIT_TIMEOUT": "200"}, None),
    ("ROC_ACTIVE_WAIT_TIMEOUT=2000", {"ROC_ACTIVE_WAIT_TIMEOUT": "2000"}, None),
    ("hipDeviceScheduleSpin", {}, 1),
    ("hipDeviceScheduleYield", {}, 2),
]


def med(x):
    x = sorted(x)
    return x[len(x) // 2]


def child(k: int) -> None:
    name, _, flags = SETTINGS[k]
    import ctypes

    import torch

    if flags is not None:
        hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch loaded (same soname)
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(flags))
        print(f"hipSetDeviceFlags({flags}) -> {rc}", file=sys.stderr)
    sys.path.insert(0, ROOT)
    from seqs_amd import Engine, synth

    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    eng = Engine(0)
    bs = []
    for b in range(4):
        buf, off, ln = synth.uniform_batch(65536, 1500, seed=1 + b)
        bs.append(tuple(torch.from_numpy(x).to(dev) for x in (buf, off, ln)))
    ns = 5
    streams = [torch.cuda.Stream(dev) for _ in range(ns)]
    outs = [torch.empty((65536, 2), dtype=torch.int32, device=dev) for _ in range(ns)]
    sts = [torch.empty((65536,), dtype=torch.uint8, device=dev) for _ in range(ns)]
    prep = None
    if hasattr(eng, "prepare_digest"):
        prep = [[eng.prepare_digest(*bs[b], out=outs[s], status=sts[s], stream=streams[s]) for s in range(ns)]
                for b in range(4)]
    for i in range(600):
        eng.digest_device(*bs[i % 4], out=outs[i % ns], status=sts[i % ns], stream=streams[i % ns])
    torch.cuda.synchronize()

    def settle():
        evs = []
        for s in streams:
            e = torch.cuda.Event()
            e.record(s)
            evs.append(e)
        for e in evs:
            while not e.query():
                pass

    res = {"setting": name}
    t = []
    for _ in range(300):
        a = time.perf_counter_ns()
        torch.cuda.synchronize()
        t.append(time.perf_counter_ns() - a)
    res["idle_sync_us"] = med(t) / 1e3

    def region(K, use_prep, do_settle):
        torch.cuda.synchronize()
        t0 = time.perf_counter_ns()
        for i in range(K):
            if use_prep:
                prep[i % 4][i % ns]()
            else:
                eng.digest_device(*bs[i % 4], out=outs[i % ns], status=sts[i % ns], stream=streams[i % ns])
        t1 = time.perf_counter_ns()
        if do_settle:
            settle()
        t2 = time.perf_counter_ns()
        torch.cuda.synchronize()
        t3 = time.perf_counter_ns()
        return (t1 - t0) / 1e3, (t2 - t1) / 1e3, (t3 - t2) / 1e3, (t3 - t0) / 1e3

    import gc

    gc.collect()
    gc.disable()
    for label, up, ds in (("call", False, True), ("prep", True, True), ("call_nosettle", False, False),
                          ("prep_nosettle", True, False)):
        if up and prep is None:
            continue
        rows = [region(20, up, ds) for _ in range(40)]
        res[label] = {"enqueue_us": round(med([r[0] for r in rows]), 2), "settle_us": round(med([r[1] for r in rows]), 2),
                      "sync_us": round(med([r[2] for r in rows]), 2), "region_us": round(med([r[3] for r in rows]), 2),
                      "region_min_us": round(min(r[3] for r in rows), 2)}
    gc.enable()
    print(json.dumps(res), flush=True)


def main() -> None:
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        return child(int(sys.argv[2]))
    ok = True
    for k, (name, env, _) in enumerate(SETTINGS):
        e = dict(os.environ)
        e.update(env)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", str(k)], env=e, timeout=240)
        ok &= r.returncode == 0
        if r.returncode != 0:
            print(f"{name}: rc {r.returncode}", flush=True)
            break
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
