#!/bin/bash
# TX fill / FCS-verify bench lines (c2, c3) next to the digest line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for op in digest fill fcs; do
  for cfg in c2 c3; do
    timeout -k 10 120 python bench.py --cpu-seconds 0 --op $op --config $cfg > gpurun_out/op_${op}_$cfg.log 2>&1 || { echo "BENCH $op $cfg FAILED"; tail -5 gpurun_out/op_${op}_$cfg.log; exit 1; }
    echo "$op $cfg $(python -c "import json; d=json.loads(open('gpurun_out/op_${op}_$cfg.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])")"
  done
done
