#!/bin/bash
# Round 4: the driver's command, three runs (the line with its C3, C5 and small-frame sub-records).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bench; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$r.json 2>$O/drv_$r.err || { echo FAIL bench; tail -5 $O/drv_$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/drv_$r.json').read().strip().splitlines()[-1]); print('driver cmd: %.1f GiB/s %.2f us/step kernel %.2f us c3 %.1f c5 %.1f small %.1f (%.3g frames/s) wall c3 %.1fs small %.1fs' % (d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_avg_us'], d['c3']['value'], d['c5_host']['value'], d['small']['value'], d['small']['frames_per_s'], d['c3']['wall_s'], d['small']['wall_s']))"
done
