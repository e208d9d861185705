#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in base d2 d3; do
  if [ "$v" = base ]; then unset FRAMESUM_LIB; else export FRAMESUM_LIB="$GRAFT_REPO_ROOT/seqs_amd/lib/diag/libframesum_$v.so"; fi
  for fr in 16384 65536; do
    timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 200 --frames $fr > gpurun_out/dg_${v}_$fr.log 2>&1 || { echo "BENCH $v FAILED"; tail -5 gpurun_out/dg_${v}_$fr.log; exit 1; }
    echo "$v n=$fr $(python -c "import json; d=json.loads(open('gpurun_out/dg_${v}_$fr.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])")"
  done
done
