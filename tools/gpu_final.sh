#!/bin/bash
# Round-end check of the committed tree: the whole GPU suite, smoke(), then the profile set
# (tools/gpu_prof.sh: rocprofv3 kernel trace + stats of the bench, PMC passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
rm -rf gpurun_out/prof
bash tools/gpu_prof.sh
