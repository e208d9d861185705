#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python tools/host_bench.py > gpurun_out/host_bench.log 2>&1 || { echo "HOST BENCH FAILED"; tail -10 gpurun_out/host_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/host_bench.log
