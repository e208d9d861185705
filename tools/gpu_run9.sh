#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for cfg in "c2 65536" "c3 65536" "c2 16384"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 200 --config $1 --frames $2 > gpurun_out/b_$1_$2.log 2>&1 || { echo "BENCH $cfg FAILED"; tail -5 gpurun_out/b_$1_$2.log; exit 1; }
  echo "$cfg $(python -c "import json; d=json.loads(open('gpurun_out/b_$1_$2.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])")"
done
bash tools/gpu_stamps.sh
