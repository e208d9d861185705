#!/bin/bash
# TX fill cost split: the product library vs diagnostic builds (FS_TXDIAG bits).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {
  timeout -k 10 120 env FRAMESUM_LIB="$1" python bench.py --cpu-seconds 0 --op fill --config c2 > gpurun_out/txd.log 2>&1 || { echo "BENCH $1 FAILED"; tail -5 gpurun_out/txd.log; exit 1; }
  echo "$2 $(python -c "import json; d=json.loads(open('gpurun_out/txd.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_us'])")"
}
L=seqs_amd/lib
for v in "$@"; do run $L/$v.so $v; done
