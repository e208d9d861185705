#!/bin/bash
# Round 4: the 16-lane kernel bring-up (tools/gpu_w2.sh), the region's fixed costs per runtime
# wait setting (tools/sync_cost.py), and the driver's command with prepared calls.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4a; mkdir -p $O
bash tools/gpu_w2.sh || exit 1
timeout -k 10 600 python tools/sync_cost.py > $O/sync_cost.log 2>&1 || { grep -v amdgpu.ids $O/sync_cost.log; exit 1; }
grep -v amdgpu.ids $O/sync_cost.log
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-sub > $O/drv_$r.json 2>/dev/null || { echo FAIL bench; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/drv_$r.json').read().strip().splitlines()[-1]); print('driver cmd: %.1f GiB/s %.2f us/step kernel %.2f us' % (d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_avg_us']))"
done
