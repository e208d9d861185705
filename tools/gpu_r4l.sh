#!/bin/bash
# Round 4: tile transitions, three forms on one box: the pipelined loop (the library), descriptors early
# but rows after the finish (seqs_amd/lib/ab/libframesum_hyb.so) and round 3's loop (libframesum_nopipe.so);
# the hybrid's multi-tile parity first.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4l; mkdir -p $O
FRAMESUM_LIB=$GRAFT_REPO_ROOT/seqs_amd/lib/ab/libframesum_hyb.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "few_workgroups or many_tiles or c2_full or partial" --timeout 300 --timeout-method thread > $O/hyb_tests.log 2>&1; rc=$?
tail -2 $O/hyb_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/hyb_tests.log | head -30; exit 1; }
timeout -k 10 400 python tools/env_sweep.py --rounds 2 --only "base+lib=hyb+lib=nopipe" --out $O/c2_20.jsonl || exit 1
timeout -k 10 400 python tools/env_sweep.py --rounds 1 --steps 2000 --warmup 500 --only "base+lib=hyb+lib=nopipe" --out $O/c2_2000.jsonl || exit 1
timeout -k 10 400 python tools/env_sweep.py --rounds 2 --only "base+lib=hyb+lib=nopipe" --extra "--frames 131072" --out $O/c2_131k.jsonl || exit 1
for L in new hyb nopipe; do
  if [ $L = new ]; then unset FRAMESUM_LIB; else export FRAMESUM_LIB=$GRAFT_REPO_ROOT/seqs_amd/lib/ab/libframesum_$L.so; fi
  timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 10 --cpu-seconds 0 > $O/c4_$L.json 2>/dev/null || { echo FAIL c4; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_$L.json').read().strip().splitlines()[-1]); print('c4 $L', d['value'], d['ms_per_step'], d.get('roofline',{}).get('kernel_avg_us'))"
done
