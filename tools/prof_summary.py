#!/usr/bin/env python3
"""Summarise a tools/gpu_prof.sh collection into the files committed under profiles/.

usage: prof_summary.py <collection dir (gpurun_out/prof)> <output dir>

Writes, per config (c2, c3):
  kernel_stats_<cfg>.csv   rocprofv3 --kernel-trace --stats summary of the bench.py command
  bench_<cfg>.json         the bench line printed by that same command
  trace_<cfg>.json         kernel durations from that command's kernel trace: all dispatches, and the
                           last `steps` ones = bench.py's single-stream event-timed pass (the one its
                           roofline.kernel_avg_us comes from; the timed loop's 2-stream overlap makes
                           individual durations longer there), next to the bench's own figure
  pmc_<cfg>.json           per-dispatch medians of every PMC counter for digest_kernel, plus
                           hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
                           (FETCH_SIZE/WRITE_SIZE are KiB; gfx950 FETCH_SIZE reads 1/2 of a wide
                           coalesced stream's bytes, MI355X_MICROARCH.md "HBM [CDNA4]")
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

KERNEL = "digest_kernel"


def counters(pass_dir):
    # only the kernel the run chose most often (a context's first launches run the mixed-length
    # kernel whatever the batch: the automatic choice's initial window)
    rows = []
    for path in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            rows += [r for r in csv.DictReader(f) if KERNEL in r["Kernel_Name"]]
    names = {}
    for r in rows:
        names.setdefault(r["Kernel_Name"], set()).add(r["Dispatch_Id"])
    main = max(names, key=lambda k: len(names[k])) if names else None
    per = {}
    for row in rows:
        if row["Kernel_Name"] == main:
            key = (row["Counter_Name"], row["Dispatch_Id"])
            per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
    by_name = {}
    for (name, _), v in per.items():
        by_name.setdefault(name, []).append(v)
    return {k: statistics.median(v) for k, v in by_name.items()}, {k: len(v) for k, v in by_name.items()}


def trace_timing(trace_csv, bench):
    durs = []
    with open(trace_csv) as f:
        for row in csv.DictReader(f):
            if KERNEL in row["Kernel_Name"]:
                durs.append((int(row["Dispatch_Id"]), int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    durs.sort()
    spans = [(a, b) for _, a, b in durs]
    durs = [b - a for _, a, b in durs]
    steps = int(bench.get("steps", 0)) if bench else 0
    last = durs[-steps:] if steps else []
    us = lambda v: round(v / 1e3, 3)
    out = {"kernel": KERNEL, "dispatches": len(durs), "all_avg_us": us(statistics.mean(durs)) if durs else None}
    if last:
        out.update({"single_stream_pass_dispatches": len(last), "single_stream_pass_avg_us": us(statistics.mean(last)),
                    "single_stream_pass_median_us": us(statistics.median(last))})
        # first start to last end of the pass, per launch: what the bench's one event pair measures
        out["single_stream_pass_span_per_launch_us"] = us((spans[-1][1] - spans[-len(last)][0]) / len(last))
    if bench:
        out["bench_kernel_avg_us"] = bench["roofline"]["kernel_avg_us"]
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    for cfg in ("c2", "c3", "c2fill"):
        stats = glob.glob(os.path.join(src, cfg, "**", "*kernel_stats.csv"), recursive=True)
        if stats:
            shutil.copy(stats[0], os.path.join(dst, f"kernel_stats_{cfg}.csv"))
        bj = os.path.join(src, f"bench_{cfg}.json")
        if os.path.exists(bj):
            lines = [l for l in open(bj).read().splitlines() if l.startswith("{")]
            if lines:
                with open(os.path.join(dst, f"bench_{cfg}.json"), "w") as f:
                    f.write(lines[-1] + "\n")
                traces = glob.glob(os.path.join(src, cfg, "**", "*kernel_trace.csv"), recursive=True)
                if traces:
                    tt = trace_timing(traces[0], json.loads(lines[-1]))
                    with open(os.path.join(dst, f"trace_{cfg}.json"), "w") as f:
                        json.dump(tt, f, indent=1)
                        f.write("\n")
                    print(cfg, json.dumps(tt))
        med, n = {}, {}
        for d in sorted(glob.glob(os.path.join(src, f"pmc_{cfg}_*"))):
            if os.path.isdir(d):
                m, c = counters(d)
                med.update(m)
                n.update(c)
        if not med:
            continue
        out = {"kernel": KERNEL, "config": cfg, "dispatches_per_counter": n, "median_per_dispatch": med}
        if "FETCH_SIZE" in med:
            out["hbm_bytes_per_launch"] = int(round((2 * med["FETCH_SIZE"] + med.get("WRITE_SIZE", 0.0)) * 1024))
            out["hbm_bytes_note"] = ("(2*FETCH_SIZE + WRITE_SIZE) * 1024: counters in KiB, FETCH_SIZE doubled per the "
                                     "gfx950 correction for wide coalesced reads; separate --pmc passes")
        cal = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "fetch_size_calibration.json")
        if "hbm_bytes_per_launch" in out and os.path.exists(cal):
            c = json.load(open(cal))
            f = c["pattern_factor"][c["config_pattern"].get(cfg, c["config_pattern"]["c2"])]
            out["hbm_bytes_per_launch_calibrated"] = int(round(out["hbm_bytes_per_launch"] / f))
            out["calibration_note"] = (f"divided by {f}: the doubled FETCH_SIZE of this access pattern without "
                                       "compute over its true bytes (profiles/fetch_size_calibration.json). That "
                                       "factor is real traffic of the pattern, not a counter artefact: the 128-B line "
                                       "two neighbouring frames share is fetched twice (reading alternate frames "
                                       "backwards fetches it once: profiles/round2/tile_pattern_dir_fetch.txt), so "
                                       "this figure is the kernel's traffic beyond its read pattern's own")
        if "TCC_HIT_sum" in med and "TCC_MISS_sum" in med:
            out["l2_hit_rate"] = med["TCC_HIT_sum"] / max(1.0, med["TCC_HIT_sum"] + med["TCC_MISS_sum"])
        with open(os.path.join(dst, f"pmc_{cfg}.json"), "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
            f.write("\n")
        print(cfg, json.dumps({k: out[k] for k in out if k in ("hbm_bytes_per_launch", "l2_hit_rate")}))


if __name__ == "__main__":
    main()
