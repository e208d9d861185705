#!/bin/bash
# Round 4: the pipelined tile loop against the same library without it (seqs_amd/lib/ab/
# libframesum_nopipe.so: the loop of round 3, the global report store kept), on C2 (20 and 2,000 steps),
# 131,072-frame batches (2 tiles per wave) and C4 at N = 1 (16 tiles per wave).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 400 python tools/env_sweep.py --rounds 3 --only "base+lib=nopipe" --out $O/c2_20.jsonl || exit 1
timeout -k 10 400 python tools/env_sweep.py --rounds 2 --steps 2000 --warmup 500 --only "base+lib=nopipe" --out $O/c2_2000.jsonl || exit 1
timeout -k 10 400 python tools/env_sweep.py --rounds 2 --only "base+lib=nopipe" --extra "--frames 131072" --out $O/c2_131k.jsonl || exit 1
for r in 1 2; do for L in new nopipe; do
  if [ $L = nopipe ]; then export FRAMESUM_LIB=$GRAFT_REPO_ROOT/seqs_amd/lib/ab/libframesum_nopipe.so; else unset FRAMESUM_LIB; fi
  timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 10 --cpu-seconds 0 > $O/c4_${L}_$r.json 2>/dev/null || { echo FAIL c4; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_${L}_$r.json').read().strip().splitlines()[-1]); print('c4 $L', d['value'], d['ms_per_step'], d.get('roofline',{}).get('kernel_avg_us'))"
done; done
