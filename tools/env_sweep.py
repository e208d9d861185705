"""Measurement aid: the driver's bench command (`bench.py --steps 20 --warmup 5`) under runtime
settings (environment of the bench process) and stream counts, interleaved round by round so box
drift spreads over every setting. This parent never touches the GPU; each run is a child process.

  python tools/env_sweep.py [--rounds 3] [--steps 20] [--out gpurun_out/env_sweep.jsonl]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SETTINGS = [
    ("base", {}, []),
    ("HIP_FORCE_DEV_KERNARG=0", {"HIP_FORCE_DEV_KERNARG": "0"}, []),
    ("HIP_FORCE_DEV_KERNARG=1", {"HIP_FORCE_DEV_KERNARG": "1"}, []),
    ("ROC_USE_FGS_KERNARG=0", {"ROC_USE_FGS_KERNARG": "0"}, []),
    ("ROC_USE_FGS_KERNARG=1", {"ROC_USE_FGS_KERNARG": "1"}, []),
    ("DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0", {"DEBUG_CLR_KERNARG_HDP_FLUSH_WA": "0"}, []),
    ("streams=3", {}, ["--streams", "3"]),
    ("streams=4", {}, ["--streams", "4"]),
    ("streams=6", {}, ["--streams", "6"]),
    ("streams=7", {}, ["--streams", "7"]),
    ("streams=8", {}, ["--streams", "8"]),
    ("wg=192", {}, ["--workgroups", "192"]),
    ("wg=128", {}, ["--workgroups", "128"]),
    ("wg=64", {}, ["--workgroups", "64"]),
    ("wg=128,streams=8", {}, ["--workgroups", "128", "--streams", "8"]),
    # a previous build of the library (seqs_amd/lib/ab/, built from an earlier commit's sources) for
    # same-box A/B
    ("lib=old", {"FRAMESUM_LIB": os.path.join(ROOT, "seqs_amd", "lib", "ab", "libframesum_old.so")}, []),
    ("wg=32", {}, ["--workgroups", "32"]),
    ("wg=16", {}, ["--workgroups", "16"]),
]


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--only", default=None, help="setting names separated by '+'")
    p.add_argument("--extra", default="", help="more bench arguments for every run (space-separated)")
    p.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "env_sweep.jsonl"))
    a = p.parse_args()
    sets = [s for s in SETTINGS if a.only is None or s[0] in a.only.split("+")]
    # lib=<name> not listed above: seqs_amd/lib/ab/libframesum_<name>.so (an A/B build)
    for nm in (a.only or "").split("+"):
        if nm.startswith("lib=") and nm not in [x[0] for x in sets]:
            sets.append((nm, {"FRAMESUM_LIB": os.path.join(ROOT, "seqs_amd", "lib", "ab", f"libframesum_{nm[4:]}.so")}, []))
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    res = {s[0]: [] for s in sets}
    with open(a.out, "a") as f:
        for r in range(a.rounds):
            for name, env, extra in sets:
                e = dict(os.environ)
                e.update(env)
                cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(a.steps), "--warmup", str(a.warmup),
                       "--cpu-seconds", "0", "--no-sub"] + extra + a.extra.split()
                cp = subprocess.run(cmd, env=e, capture_output=True, text=True, timeout=180)
                if cp.returncode != 0:
                    print(f"{name}: rc {cp.returncode}\n{cp.stderr[-2000:]}", flush=True)
                    sys.exit(1)
                d = json.loads(cp.stdout.strip().splitlines()[-1])
                res[name].append(d["value"])
                f.write(json.dumps({"setting": name, "round": r, "value": d["value"], "ms_per_step": d["ms_per_step"],
                                    "kernel_avg_us": d["roofline"]["kernel_avg_us"]}) + "\n")
                f.flush()
                print(f"round {r} {name:34s} {d['value']:8.1f} GiB/s  {d['ms_per_step'] * 1e3:6.2f} us/step", flush=True)
    for name, v in res.items():
        v = sorted(v)
        print(f"{name:34s} median {v[len(v) // 2]:8.1f}  min {v[0]:8.1f}  max {v[-1]:8.1f}", flush=True)


if __name__ == "__main__":
    main()
