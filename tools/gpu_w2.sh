#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
FRAMESUM_LIB=$PWD/seqs_amd/lib/diag/libframesum_wdump.so timeout -k 10 100 python tools/wdump.py > gpurun_out/wdump.log 2>&1; grep -v amdgpu.ids gpurun_out/wdump.log | tail -5
timeout -k 10 200 python tools/wdebug.py > gpurun_out/wdebug3.log 2>&1; grep -E "^[a-z]" gpurun_out/wdebug3.log
