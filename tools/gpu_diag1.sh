#!/bin/bash
# GPU session: HBM microbench + diagnostic variants of the digest kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/hbm_read_bw > gpurun_out/hbm_bw.log 2>&1 || { echo HBM FAILED; cat gpurun_out/hbm_bw.log; exit 1; }
cat gpurun_out/hbm_bw.log
for v in base d1 d2 p8 p2; do
  if [ "$v" = base ]; then unset FRAMESUM_LIB; else export FRAMESUM_LIB="$GRAFT_REPO_ROOT/seqs_amd/lib/diag/libframesum_$v.so"; fi
  timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 200 > gpurun_out/diag_$v.log 2>&1 || { echo "BENCH $v FAILED"; tail -5 gpurun_out/diag_$v.log; exit 1; }
  echo "$v $(python -c "import json,sys; d=json.loads(open('gpurun_out/diag_$v.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])")"
done
unset FRAMESUM_LIB
for fr in 16384 262144; do
  timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 100 --frames $fr > gpurun_out/diag_n$fr.log 2>&1 || exit 1
  echo "n=$fr $(python -c "import json; d=json.loads(open('gpurun_out/diag_n$fr.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])")"
done
timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 100 --config c3 > gpurun_out/diag_c3.log 2>&1 || exit 1
echo "c3 $(python -c "import json; d=json.loads(open('gpurun_out/diag_c3.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])")"
