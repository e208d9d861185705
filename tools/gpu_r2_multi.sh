#!/bin/bash
# Round-2 check of the multi-GPU paths: the new GPU tests, then C4 / C5 bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_multi_gpu.py tests/test_go_binding.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_multi.log 2>&1 || { echo "MULTI TESTS FAILED"; tail -60 gpurun_out/pytest_multi.log; exit 1; }
tail -3 gpurun_out/pytest_multi.log
timeout -k 10 200 python bench.py --config c4 --steps 50 --warmup 5 --cpu-seconds 0 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo "C4 FAILED"; tail -30 gpurun_out/bench_c4.err; exit 1; }
tail -1 gpurun_out/bench_c4.json
timeout -k 10 200 python bench.py --config c4 --steps 50 --warmup 5 --cpu-seconds 0 --force-gather > gpurun_out/bench_c4_gather.json 2> gpurun_out/bench_c4_gather.err || { echo "C4 gather FAILED"; tail -30 gpurun_out/bench_c4_gather.err; exit 1; }
tail -1 gpurun_out/bench_c4_gather.json
timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo "C5 FAILED"; tail -30 gpurun_out/bench_c5.err; exit 1; }
tail -1 gpurun_out/bench_c5.json
