"""Attribution of a bench timed region (measurement tool).

Run the bench under a rocprofv3 HIP-API + kernel trace with --region-clocks, then line the
trace up with the region's host clocks:

  rocprofv3 --hip-trace --kernel-trace --output-format csv -d <dir> -- \
      python3 bench.py --steps 20 --warmup 5 --no-sub --cpu-seconds 0 --region-clocks <clk.json>
  python3 tools/region_attr.py <dir> <clk.json>

Per region: t0 -> the first launch call's start (Python + ctypes), that call's duration (the HIP
enqueue), its end -> the first kernel's start (dispatch), the kernel span, the last kernel's
end -> the polled settle seeing it, settle -> t1 (the synchronize), and the launch calls'
spacing."""
import csv
import glob
import json
import os
import sys


def rows(tdir, pattern):
    out = []
    for f in glob.glob(os.path.join(tdir, "**", pattern), recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def main():
    tdir, clk = sys.argv[1], sys.argv[2]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", ""))
                for r in rows(tdir, "*kernel_trace.csv"))
    api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Function", ""))
                 for r in rows(tdir, "*hip_api_trace.csv"))
    regs = [json.loads(line) for line in open(clk) if line.strip()]
    # which host clock the trace uses: the one that puts digest dispatches inside the regions
    best = None
    for ck in ("mono", "boot"):
        inside = sum(1 for s, e, n in ks for r in regs if "digest" in n and r["t0"][ck] <= s <= r["t1"][ck])
        if best is None or inside > best[1]:
            best = (ck, inside)
    ck = best[0]
    off = {r_i: r["t0"][ck] - r["t0"]["mono"] for r_i, r in enumerate(regs)}  # steps/settle are mono stamps
    print(f"trace clock: {ck} ({best[1]} digest dispatches inside {len(regs)} regions)")
    for i, r in enumerate(regs):
        t0, t1 = r["t0"][ck], r["t1"][ck]
        kin = [(s, e) for s, e, n in ks if "digest" in n and t0 <= s <= t1]
        lin = [(s, e, f) for s, e, f in api if t0 <= s <= t1 and "aunch" in f]
        us = lambda x: x / 1e3  # noqa: E731
        if kin and not lin and r.get("steps"):
            # kernel trace only (no HIP-API trace, whose own overhead inflates the host side): the
            # first step's return stands for the first launch call's end
            settled = r.get("settled", 0) + off[i]
            s0 = r["steps"][0] + off[i]
            steps = [x + off[i] for x in r["steps"]]
            gaps = [us(b - a) for a, b in zip(steps, steps[1:])]
            print(f"region {i}: wall {r['elapsed_us']:.1f} us | t0->1st step returned {us(s0 - t0):.1f} | "
                  f"returned->1st kernel {us(kin[0][0] - s0):.1f} | t0->1st kernel {us(kin[0][0] - t0):.1f} | "
                  f"kernel span {us(max(e for _, e in kin) - kin[0][0]):.1f} ({len(kin)} kernels, first "
                  f"{us(kin[0][1] - kin[0][0]):.1f}) | last end->settled {us(settled - max(e for _, e in kin)):.1f} | "
                  f"settled->t1 {us(t1 - settled):.1f} | step returns every {sum(gaps) / max(1, len(gaps)):.1f} us")
            continue
        if not kin or not lin:
            print(f"region {i}: no kernels/launches inside")
            continue
        first_call = lin[0]
        settled = r.get("settled", 0) + off[i]
        steps = [x + off[i] for x in r.get("steps", [])]
        gaps = [us(b - a) for a, b in zip(steps, steps[1:])]
        print(f"region {i}: wall {r['elapsed_us']:.1f} us | t0->1st launch call {us(first_call[0] - t0):.1f} | "
              f"call {us(first_call[1] - first_call[0]):.1f} ({first_call[2]}) | call end->1st kernel "
              f"{us(kin[0][0] - first_call[1]):.1f} | t0->1st kernel {us(kin[0][0] - t0):.1f} | kernel span "
              f"{us(max(e for _, e in kin) - kin[0][0]):.1f} ({len(kin)} kernels, first {us(kin[0][1] - kin[0][0]):.1f}) | "
              f"last end->settled {us(settled - max(e for _, e in kin)):.1f} | settled->t1 {us(t1 - settled):.1f} | "
              f"step returns every {sum(gaps) / max(1, len(gaps)):.1f} us | launch calls "
              f"{sum(us(e - s) for s, e, _ in lin) / len(lin):.1f} us avg")


if __name__ == "__main__":
    main()
