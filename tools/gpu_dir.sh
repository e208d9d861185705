#!/bin/bash
# Forward-only vs alternating-direction whole-block reads (tile_pattern dir), 1500-B and 1536-B
# frames, then FETCH_SIZE per pattern (one --pmc pass).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/tile_pattern dir 1500 > gpurun_out/dir_1500.log 2>&1 && cat gpurun_out/dir_1500.log || exit 1
timeout -k 10 120 ./tools/tile_pattern dir 1536 > gpurun_out/dir_1536.log 2>&1 && cat gpurun_out/dir_1536.log || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/dir_pmc
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/dir_pmc -- ./tools/tile_pattern dircal 1500 > gpurun_out/dir_pmc.log 2>&1 || { tail gpurun_out/dir_pmc.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/dir_pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Kernel_Name"][:40]].append(float(r["Counter_Value"]))
for k, v in d.items():
    v.sort()
    print(f"{k:42s} n {len(v):3d} FETCH_SIZE med {v[len(v)//2]:.0f} KB -> 2x = {2*v[len(v)//2]*1024/98304000:.4f} of bytes")
PY
