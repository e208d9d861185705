#!/bin/bash
# 16-lane kernel bring-up: parity (tools/w2_check.py), single-stream kernel time against the
# one-pass kernel, and bench lines (driver command and 2,000 steps) with the kernel forced.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/w2; mkdir -p $O
timeout -k 10 300 python tools/w2_check.py --time > $O/check.log 2>&1; rc=$?
cat $O/check.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit 1
for k in 6 4 6 4; do
  timeout -k 10 120 python bench.py --kernel $k --steps 20 --warmup 5 --cpu-seconds 0 --no-sub > $O/b20_$k.json 2>/dev/null || { echo FAIL b20 $k; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b20_$k.json').read().strip().splitlines()[-1]); print('kernel $k 20 steps: %.1f GiB/s %.2f us/step kernel %.2f us' % (d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_avg_us']))"
done
for k in 6 4; do
  timeout -k 10 120 python bench.py --kernel $k --steps 2000 --warmup 500 --cpu-seconds 0 --no-sub > $O/b2000_$k.json 2>/dev/null || { echo FAIL b2000 $k; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b2000_$k.json').read().strip().splitlines()[-1]); print('kernel $k 2000 steps: %.1f GiB/s %.2f us/step kernel %.2f us' % (d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_avg_us']))"
done
