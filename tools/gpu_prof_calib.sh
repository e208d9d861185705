#!/bin/bash
# Round-2 profile set: rocprofv3 kernel-trace + stats and PMC passes of the bench (tools/gpu_prof.sh),
# then the FETCH_SIZE calibration of the access patterns (tools/tile_pattern calib).
set -o pipefail
R="$GRAFT_REPO_ROOT"
bash "$R/tools/gpu_prof.sh" || exit 1
mkdir -p "$R/gpurun_out/calib2"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/calib2/fetch" -o run -- "$R/tools/tile_pattern" calib > "$R/gpurun_out/calib2/fetch.log" 2>&1 || { echo "calib failed"; tail -5 "$R/gpurun_out/calib2/fetch.log"; exit 1; }
cd "$R" && python3 - <<'PY'
import csv, glob, statistics, collections
per = collections.defaultdict(list)
for p in glob.glob("gpurun_out/calib2/fetch/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(p)):
        per[row["Kernel_Name"][:70]].append(float(row["Counter_Value"]))
for k, v in per.items():
    print(f"{k:70s} n={len(v):3d} median FETCH_SIZE KiB={statistics.median(v):10.0f}  2x1024/98304000={2*statistics.median(v)*1024/98304000:.3f}")
PY
