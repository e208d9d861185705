#!/usr/bin/env python3
"""Average / median kernel durations from rocprofv3 --kernel-trace CSVs under a directory
(measurement tool). usage: trace_stats.py <dir> [name-substring]"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict

root = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "kernel"
for d in sorted(glob.glob(os.path.join(root, "*"))):
    dur = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if sub in row["Kernel_Name"]:
                    dur[row["Kernel_Name"][:60]].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1000.0)
    for k, v in dur.items():
        v = v[5:] if len(v) > 10 else v  # skip the first launches
        print(f"{os.path.basename(d):24s} {k:60s} n={len(v):4d} avg={statistics.mean(v):8.2f} us  med={statistics.median(v):8.2f} us")
