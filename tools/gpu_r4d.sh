#!/bin/bash
# Round 4: the pipelined tile loop of the one-pass kernel (global report store, tile-uniform loop):
# GPU suite, then the driver's command and 2,000 steps against capped grids, and C4 at N = 1.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -5 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -20; exit 1; }
timeout -k 10 600 python tools/env_sweep.py --rounds 2 --only "base+wg=192+wg=128+wg=64+wg=128,streams=8" --out $O/sweep20.jsonl || exit 1
timeout -k 10 600 python tools/env_sweep.py --rounds 1 --steps 2000 --warmup 500 --only "base+wg=128+wg=64" --out $O/sweep2000.jsonl || exit 1
for wg in 0 128; do
  timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 10 --cpu-seconds 0 --workgroups $wg > $O/c4_$wg.json 2>/dev/null || { echo FAIL c4; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_$wg.json').read().strip().splitlines()[-1]); print('c4 wg=$wg', d['value'], d['ms_per_step'], d.get('roofline',{}).get('kernel_avg_us'))"
done
timeout -k 10 600 python tools/env_sweep.py --rounds 1 --only "base+wg=64+wg=32+wg=16" --extra "--config small" --out $O/sweep_small.jsonl || exit 1
timeout -k 10 600 python tools/env_sweep.py --rounds 1 --only "base+wg=128" --extra "--config c3" --out $O/sweep_c3.jsonl || exit 1
