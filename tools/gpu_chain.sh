#!/bin/bash
# Chained tiles: parity (every kernel variant, multi-GPU C4 shapes), then C4 / C2 with and without.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_tx_fcs.py tests/test_multi_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_chain.log 2>&1 || { echo "PARITY FAILED"; tail -40 gpurun_out/pytest_chain.log; exit 1; }
tail -1 gpurun_out/pytest_chain.log
for v in base nochain base nochain; do
  lib=seqs_amd/lib/diag/libframesum_$v.so; [ "$v" = base ] && lib=seqs_amd/lib/libframesum.so
  timeout -k 10 200 env FRAMESUM_LIB="$GRAFT_REPO_ROOT/$lib" python bench.py --config c4 --steps 30 --warmup 5 --cpu-seconds 0 > gpurun_out/c4_$v.json 2>gpurun_out/c4_$v.err || { echo "C4 $v FAILED"; tail -5 gpurun_out/c4_$v.err; exit 1; }
  echo "$v c4 $(python -c "import json; d=json.loads(open('gpurun_out/c4_$v.json').read().strip().splitlines()[-1]); print(d['value'], d['config']['kernel_only_gibs'], d['roofline']['kernel_avg_us'])")"
done
STEPS=1000 WARM=500 CFGS=c2 bash tools/gpu_abk.sh base:0 nochain:0
