#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
FRAMESUM_LIB="$GRAFT_REPO_ROOT/seqs_amd/lib/diag/libframesum_st4.so" timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps.log 2>&1 || { echo "STAMPS FAILED"; tail -5 gpurun_out/stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps.log
for v in base noprio; do
  if [ "$v" = base ]; then unset FRAMESUM_LIB; else export FRAMESUM_LIB="$GRAFT_REPO_ROOT/seqs_amd/lib/diag/libframesum_$v.so"; fi
  for cfg in "c2 65536" "c3 65536"; do
    set -- $cfg
    timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 200 --config $1 --frames $2 > gpurun_out/p_${v}_$1.log 2>&1 || { echo "BENCH FAILED"; tail -5 gpurun_out/p_${v}_$1.log; exit 1; }
    echo "$v $cfg $(python -c "import json; d=json.loads(open('gpurun_out/p_${v}_$1.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])")"
  done
done
unset FRAMESUM_LIB
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
