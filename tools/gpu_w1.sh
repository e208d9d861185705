#!/bin/bash
# 16-lane kernel bring-up: the parity suites, then C2/C3 bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_tx_fcs.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_w1.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_w1.log
[ $rc -eq 0 ] || exit 1
for cfg in c2 c3; do
  timeout -k 10 120 python bench.py --cpu-seconds 0 --config $cfg > gpurun_out/w_$cfg.log 2>&1 || { echo "BENCH $cfg FAILED"; tail -5 gpurun_out/w_$cfg.log; exit 1; }
  echo "$cfg $(python -c "import json; d=json.loads(open('gpurun_out/w_$cfg.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])")"
done
