#!/bin/bash
# Round 4: PMC + trace of the one-pass (4) and 16-lane (6) kernels on C2, then the driver's
# command under runtime settings and stream counts (tools/env_sweep.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r3_pmc.sh k4 4 k6 6 > gpurun_out/r4b_pmc.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r4b_pmc.log | tail -60
[ $rc -eq 0 ] || exit 1
cd $GRAFT_REPO_ROOT && timeout -k 10 900 python tools/env_sweep.py --rounds 3 --out gpurun_out/r4b_env.jsonl
