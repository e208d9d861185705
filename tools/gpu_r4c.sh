#!/bin/bash
# Round 4: the driver's command (prepared calls, device kernargs), and its 20-step region
# attributed from a kernel-only rocprofv3 trace (tools/region_attr.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r4c; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-sub > $O/drv_$r.json 2>/dev/null || { echo FAIL bench; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/drv_$r.json').read().strip().splitlines()[-1]); print('driver cmd: %.1f GiB/s %.2f us/step kernel %.2f us' % (d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_avg_us']))"
done
export TMPDIR=/tmp
for r in 1 2 3; do
  rm -f $O/clk_$r.json
  (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$r -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-sub --region-clocks $O/clk_$r.json > $O/tr_$r.log 2>&1) || { echo FAIL trace; tail -5 $O/tr_$r.log; exit 1; }
  python3 tools/region_attr.py $O/tr_$r $O/clk_$r.json
done
