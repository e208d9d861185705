#!/bin/bash
# parity + c2/c3 bench + c2 stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_quick.sh || exit 1
FRAMESUM_LIB="$GRAFT_REPO_ROOT/seqs_amd/lib/diag/libframesum_st.so" timeout -k 10 120 python tools/stamps.py --config c2 > gpurun_out/stamps_c2.log 2>&1 || { echo "STAMPS FAILED"; tail -5 gpurun_out/stamps_c2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_c2.log
