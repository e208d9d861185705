#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in st4 st_d4; do
  FRAMESUM_LIB="$GRAFT_REPO_ROOT/seqs_amd/lib/diag/libframesum_$v.so" timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps_$v.log 2>&1 || { echo "STAMPS FAILED"; tail -5 gpurun_out/stamps_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/stamps_$v.log
done
