#!/bin/bash
# Start-of-region ramp: kernel traces of short launch bursts (tools/ramp_trace.py) under rocprofv3.
# usage: gpu_ramp.sh <tag> [ramp_trace.py args...]
set -o pipefail
R="$GRAFT_REPO_ROOT"
tag="$1"
shift
out="$R/gpurun_out/ramp_$tag"
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$out/tr" -o run -- python3 "$R/tools/ramp_trace.py" "$@" > "$out/run.log" 2>&1 || { echo "ramp run failed"; tail -5 "$out/run.log"; exit 1; }
f=$(ls "$out"/tr/*/*kernel_trace.csv "$out"/tr/*kernel_trace.csv 2>/dev/null | head -1)
cd "$R" && python3 tools/ramp_trace.py --analyze "$f" --bursts 3 > "$out/analysis.txt" && grep burst "$out/run.log" | tail -3 && cat "$out/analysis.txt"
