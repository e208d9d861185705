#!/bin/bash
# A/B bench of library variants (c2, c3): tools/gpu_ab.sh base pp base pp  (base = the product library)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  lib=seqs_amd/lib/diag/libframesum_$v.so; [ "$v" = base ] && lib=seqs_amd/lib/libframesum.so
  for cfg in c2 c3; do
    timeout -k 10 120 env FRAMESUM_LIB="$GRAFT_REPO_ROOT/$lib" python bench.py --cpu-seconds 0 --config $cfg > gpurun_out/ab.log 2>&1 || { echo "BENCH $v $cfg FAILED"; tail -5 gpurun_out/ab.log; exit 1; }
    echo "$v $cfg $(python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_us'])")"
  done
done
