#!/bin/bash
# Quick GPU check: parity suite then c2/c3 benches (no CPU baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_tx_fcs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for cfg in c2 c3; do
  timeout -k 10 120 python bench.py --cpu-seconds 0 --config $cfg > gpurun_out/q_$cfg.log 2>&1 || { echo "BENCH $cfg FAILED"; tail -5 gpurun_out/q_$cfg.log; exit 1; }
  echo "$cfg $(python -c "import json; d=json.loads(open('gpurun_out/q_$cfg.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])")"
done
