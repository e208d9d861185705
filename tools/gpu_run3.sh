#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in st4 st8; do
  FRAMESUM_LIB="$GRAFT_REPO_ROOT/seqs_amd/lib/diag/libframesum_$v.so" timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps_$v.log 2>&1 || { echo "STAMPS $v FAILED"; tail -5 gpurun_out/stamps_$v.log; exit 1; }
  echo "== $v"; cat gpurun_out/stamps_$v.log
done
for v in base p6 p8 p12; do
  if [ "$v" = base ]; then unset FRAMESUM_LIB; else export FRAMESUM_LIB="$GRAFT_REPO_ROOT/seqs_amd/lib/diag/libframesum_$v.so"; fi
  timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 200 > gpurun_out/pf_$v.log 2>&1 || { echo "BENCH $v FAILED"; tail -5 gpurun_out/pf_$v.log; exit 1; }
  echo "$v $(python -c "import json; d=json.loads(open('gpurun_out/pf_$v.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])")"
done
