#!/bin/bash
# C4 A/B of library builds: tools/gpu_c4ab.sh base chain nocap ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  lib=seqs_amd/lib/diag/libframesum_$v.so; [ "$v" = base ] && lib=seqs_amd/lib/libframesum.so
  timeout -k 10 200 env FRAMESUM_LIB="$GRAFT_REPO_ROOT/$lib" python bench.py --config c4 --steps ${STEPS:-30} --warmup 5 --cpu-seconds 0 > gpurun_out/c4ab.json 2>gpurun_out/c4ab.err || { echo "C4 $v FAILED"; tail -5 gpurun_out/c4ab.err; exit 1; }
  echo "$v c4 $(python -c "import json; d=json.loads(open('gpurun_out/c4ab.json').read().strip().splitlines()[-1]); print(d['value'], d['config']['kernel_only_gibs'], d['roofline']['kernel_avg_us'])")"
done
