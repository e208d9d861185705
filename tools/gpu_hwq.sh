#!/bin/bash
# Whole-job C2 rate against the HIP hardware-queue count and the stream count (driver-style
# 20-step regions and 2,000-step regions).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
for q in 4 8 16; do
  for ns in 5 8; do
    for k in 20 2000; do
      w=$([ $k = 20 ] && echo 5 || echo 1000)
      GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --cpu-seconds 0 --streams $ns --steps $k --warmup $w > gpurun_out/hwq.log 2>&1 || { echo "FAIL q=$q ns=$ns"; tail -5 gpurun_out/hwq.log; exit 1; }
      echo "hwq $q streams $ns K $k $(python -c "import json; d=json.loads(open('gpurun_out/hwq.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
    done
  done
done
done
