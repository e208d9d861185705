#!/bin/bash
# A/B of (library, kernel variant) pairs on c2 / c3: tools/gpu_abk.sh base:1 base:3 pf6:3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CFGS=${CFGS:-"c2 c3"}
for pair in "$@"; do
  v=${pair%%:*}; k=${pair##*:}
  lib=seqs_amd/lib/diag/libframesum_$v.so; [ "$v" = base ] && lib=seqs_amd/lib/libframesum.so
  for cfg in $CFGS; do
    timeout -k 10 120 env FRAMESUM_LIB="$GRAFT_REPO_ROOT/$lib" python bench.py --cpu-seconds 0 --config $cfg --kernel $k --steps ${STEPS:-2000} --warmup ${WARM:-1000} > gpurun_out/ab.log 2>&1 || { echo "BENCH $pair $cfg FAILED"; tail -5 gpurun_out/ab.log; exit 1; }
    echo "$pair $cfg $(python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])")"
  done
done
