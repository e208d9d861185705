#!/bin/bash
# Round check on the GPU box: parity suite, smoke, bench c2/c3, HBM ceiling microbenchmark.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 200 ./tools/hbm_read_bw > gpurun_out/hbm_98.log 2>&1 || { echo "HBM BW FAILED"; tail -5 gpurun_out/hbm_98.log; exit 1; }
cat gpurun_out/hbm_98.log
for cfg in c2 c3; do
  timeout -k 10 180 python bench.py --config $cfg > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { echo "BENCH $cfg FAILED"; tail -10 gpurun_out/bench_$cfg.err; exit 1; }
  tail -1 gpurun_out/bench_$cfg.json
done
