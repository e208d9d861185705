#!/bin/bash
# Parity suite (every kernel variant), then A/B of kernel variants: tools/gpu_al.sh base:1 base:4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_tx_fcs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_al.log 2>&1 || { echo "PARITY FAILED"; tail -40 gpurun_out/pytest_al.log; exit 1; }
tail -1 gpurun_out/pytest_al.log
STEPS=${STEPS:-1000} WARM=${WARM:-500} bash tools/gpu_abk.sh "$@"
