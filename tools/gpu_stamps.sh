#!/bin/bash
# stamps for given stamp-build variants [: kernel variant]: tools/gpu_stamps.sh st st:5
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for pair in "$@"; do
  v=${pair%%:*}; k=0; [ "$pair" != "$v" ] && k=${pair##*:}
  for cfg in c2; do
    echo "== $v kernel $k $cfg"
    FRAMESUM_LIB="$GRAFT_REPO_ROOT/seqs_amd/lib/diag/libframesum_$v.so" timeout -k 10 120 python tools/stamps.py --config $cfg --kernel $k > gpurun_out/stamps_${v}_$cfg.log 2>&1 || { echo "STAMPS FAILED"; tail -5 gpurun_out/stamps_${v}_$cfg.log; exit 1; }
    grep -v amdgpu.ids gpurun_out/stamps_${v}_$cfg.log
  done
done
