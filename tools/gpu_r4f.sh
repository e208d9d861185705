#!/bin/bash
# Round 4: the small-frame kernel (variant 8): GPU suite (every parity case through it too), then the
# reference's benchmark shape and C2 through every variant, same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -5 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; exit 1; }
for k in 0 8 0 8; do
  timeout -k 10 120 python bench.py --config small --kernel $k --steps 20 --warmup 5 --cpu-seconds 0 > $O/small_$k.json 2>/dev/null || { echo FAIL small $k; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/small_$k.json').read().strip().splitlines()[-1]); print('small kernel $k: %.1f GiB/s %.3g frames/s %.2f us/step kernel %.2f us' % (d['value'], d['frames_per_s'], d['ms_per_step']*1e3, d['roofline']['kernel_avg_us']))"
done
for k in 0 8; do
  timeout -k 10 120 python bench.py --config small --kernel $k --steps 2000 --warmup 500 --cpu-seconds 0 > $O/small2000_$k.json 2>/dev/null || { echo FAIL small $k; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/small2000_$k.json').read().strip().splitlines()[-1]); print('small 2000 kernel $k: %.1f GiB/s %.3g frames/s %.2f us/step kernel %.2f us' % (d['value'], d['frames_per_s'], d['ms_per_step']*1e3, d['roofline']['kernel_avg_us']))"
done
