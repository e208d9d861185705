#!/bin/bash
# Same-box A/B of library builds (tools/env_sweep.py lib=<name>: seqs_amd/lib/ab/libframesum_<name>.so).
# usage: tools/gpu_ab.sh "<settings joined by +>" [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab; mkdir -p $O
S="$1"; R=${2:-2}
timeout -k 10 400 python tools/env_sweep.py --rounds $R --only "$S" --out $O/c2_20.jsonl || exit 1
timeout -k 10 400 python tools/env_sweep.py --rounds $R --steps 2000 --warmup 500 --only "$S" --out $O/c2_2000.jsonl || exit 1
timeout -k 10 400 python tools/env_sweep.py --rounds 1 --steps 2000 --warmup 500 --only "$S" --extra "--config c3" --out $O/c3_2000.jsonl || exit 1
