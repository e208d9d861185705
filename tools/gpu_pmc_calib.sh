#!/bin/bash
# FETCH_SIZE calibration on known byte counts: the HBM microbenchmark's kernels (98.3 MB per launch).
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/calib"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/calib/fetch" -o run -- "$R/tools/hbm_read_bw" > "$R/gpurun_out/calib/fetch.log" 2>&1 || { echo "calib failed"; tail -5 "$R/gpurun_out/calib/fetch.log"; exit 1; }
cd "$R" && python3 - <<'PY'
import csv, glob, statistics, collections
per = collections.defaultdict(list)
for p in glob.glob("gpurun_out/calib/fetch/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(p)):
        per[row["Kernel_Name"][:60]].append(float(row["Counter_Value"]))
for k, v in per.items():
    print(f"{k:60s} n={len(v):3d} median FETCH_SIZE KiB={statistics.median(v):10.0f}  x1024/98304000={statistics.median(v)*1024/98304000:.3f}")
PY
