#!/bin/bash
# Kernel timing cross-check: bench.py plain, then under rocprofv3 --kernel-trace --stats (c2, c3).
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/tprof"
export TMPDIR=/tmp
cd "$R"
for cfg in c2 c3; do
  timeout -k 10 120 python bench.py --config $cfg --cpu-seconds 0 > gpurun_out/tprof/plain_$cfg.json || { echo "bench $cfg failed"; exit 1; }
  tail -1 gpurun_out/tprof/plain_$cfg.json
done
cd /tmp
for cfg in c2 c3; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/tprof/$cfg" -o run -- \
    python3 "$R/bench.py" --config $cfg --cpu-seconds 0 > "$R/gpurun_out/tprof/bench_$cfg.json" 2> "$R/gpurun_out/tprof/bench_$cfg.err" \
    || { echo "rocprof bench $cfg failed"; tail -5 "$R/gpurun_out/tprof/bench_$cfg.err"; exit 1; }
done
cd "$R" && python3 tools/prof_summary.py gpurun_out/tprof gpurun_out/tprof/summary
