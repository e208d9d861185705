#!/bin/bash
# timing-only A/B of diagnostic builds (wrong results by design: no parity check)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for v in "$@"; do
  for cfg in c2 c3; do
    FRAMESUM_LIB="$GRAFT_REPO_ROOT/seqs_amd/lib/diag/libframesum_$v.so" timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 300 --streams 1 --config $cfg > gpurun_out/ab/d_${v}_$cfg.log 2>&1 || { echo "BENCH $v $cfg FAILED"; tail -5 gpurun_out/ab/d_${v}_$cfg.log; exit 1; }
    echo "$v $cfg $(python -c "import json; d=json.loads(open('gpurun_out/ab/d_${v}_$cfg.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_us'])")"
  done
done
