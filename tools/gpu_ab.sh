#!/bin/bash
# A/B of kernel build variants (seqs_amd/lib/diag/libframesum_<v>.so): parity + bench c2/c3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
VARIANTS="$*"
for v in $VARIANTS; do
  FRAMESUM_LIB="$GRAFT_REPO_ROOT/seqs_amd/lib/diag/libframesum_$v.so" timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/ab/t_$v.log 2>&1 || { echo "PARITY $v FAILED"; tail -20 gpurun_out/ab/t_$v.log; exit 1; }
done
echo "parity ok: $VARIANTS"
for rep in 1 2; do
  for v in $VARIANTS; do
    for cfg in c2 c3; do
      FRAMESUM_LIB="$GRAFT_REPO_ROOT/seqs_amd/lib/diag/libframesum_$v.so" timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 300 --config $cfg > gpurun_out/ab/b_${v}_$cfg.log 2>&1 || { echo "BENCH $v $cfg FAILED"; tail -5 gpurun_out/ab/b_${v}_$cfg.log; exit 1; }
      echo "$rep $v $cfg $(python -c "import json; d=json.loads(open('gpurun_out/ab/b_${v}_$cfg.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_us'], d['roofline']['kernel_median_us'])")"
    done
  done
done
