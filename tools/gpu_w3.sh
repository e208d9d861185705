#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python tools/wdebug.py > gpurun_out/wdebug4.log 2>&1; grep -E "^[a-z]" gpurun_out/wdebug4.log | grep -v "bad=0" ; echo "wdebug done"
STEPS=1000 WARM=500 bash tools/gpu_abk.sh base:1 base:3
