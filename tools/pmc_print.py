#!/usr/bin/env python3
"""Print per-dispatch medians of every PMC counter of digest_kernel under a directory of
rocprofv3 --pmc passes (measurement tool). usage: pmc_print.py <dir>"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict

root = sys.argv[1]
for cfgdir in sorted({os.path.basename(p).split("_")[0] for p in glob.glob(os.path.join(root, "*_*")) if os.path.isdir(p)}):
    per = defaultdict(float)
    for path in glob.glob(os.path.join(root, cfgdir + "_*", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if "digest_kernel" in row["Kernel_Name"] or "rx_kernel" in row["Kernel_Name"]:
                    per[(row["Counter_Name"], path, row["Dispatch_Id"])] += float(row["Counter_Value"])
    by = defaultdict(list)
    for (name, _, _), v in per.items():
        by[name].append(v)
    med = {k: statistics.median(v) for k, v in by.items()}
    waves = med.get("SQ_WAVES", 1) or 1
    print(f"== {cfgdir}")
    for k in sorted(med):
        print(f"  {k:24s} {med[k]:14.1f}   per wave {med[k] / waves:10.1f}")
