#!/bin/bash
# Round 4, last check of the shipped tree: the whole GPU suite, smoke(), the driver's command twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/check; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$r.json 2>/dev/null || { echo FAIL bench; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/drv_$r.json').read().strip().splitlines()[-1]); print('driver cmd: %.1f GiB/s %.2f us/step kernel %.2f us c3 %.1f c5 %.1f small %.1f (%.3g frames/s)' % (d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_avg_us'], d['c3']['value'], d['c5_host']['value'], d['small']['value'], d['small']['frames_per_s']))"
done
