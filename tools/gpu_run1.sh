#!/bin/bash
# GPU session 1: parity tests, smoke, bench, rocprof kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 240 python bench.py --cpu-seconds 5 > gpurun_out/bench.log 2>&1 || { echo BENCH FAILED; tail -30 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof1" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 5 --cpu-seconds 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof1.log" 2>&1 || { echo PROF FAILED; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof1.log"; exit 1; }
find "$GRAFT_REPO_ROOT/gpurun_out/prof1" -name "*stats*" | head
