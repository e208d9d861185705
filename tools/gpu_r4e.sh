#!/bin/bash
# Round 4: same-box A/B of the library against the previous build (seqs_amd/lib/ab/libframesum_old.so):
# C2 driver command and 2,000 steps, C3, the small-frame shape, C4 at N = 1.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 300 python tools/env_sweep.py --rounds 3 --only "base+lib=old" --out $O/c2_20.jsonl || exit 1
timeout -k 10 300 python tools/env_sweep.py --rounds 2 --steps 2000 --warmup 500 --only "base+lib=old" --out $O/c2_2000.jsonl || exit 1
timeout -k 10 300 python tools/env_sweep.py --rounds 2 --only "base+lib=old" --extra "--config c3" --out $O/c3_20.jsonl || exit 1
timeout -k 10 300 python tools/env_sweep.py --rounds 2 --steps 2000 --warmup 500 --only "base+lib=old" --extra "--config c3" --out $O/c3_2000.jsonl || exit 1
timeout -k 10 300 python tools/env_sweep.py --rounds 2 --only "base+lib=old" --extra "--config small" --out $O/small.jsonl || exit 1
for r in 1 2; do for L in new old; do
  if [ $L = old ]; then export FRAMESUM_LIB=$GRAFT_REPO_ROOT/seqs_amd/lib/ab/libframesum_old.so; else unset FRAMESUM_LIB; fi
  timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 10 --cpu-seconds 0 > $O/c4_${L}_$r.json 2>/dev/null || { echo FAIL c4; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_${L}_$r.json').read().strip().splitlines()[-1]); print('c4 $L', d['value'], d['ms_per_step'], d.get('roofline',{}).get('kernel_avg_us'))"
done; done
