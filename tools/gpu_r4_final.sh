#!/bin/bash
# Round 4 final check and profile set: the whole GPU suite and smoke(), the round's profiles
# (tools/gpu_prof.sh: rocprofv3 kernel trace + stats of the bench on C2 and C3, PMC passes), the
# driver's exact command under rocprofv3 --kernel-trace --stats, then the driver's command plain
# (3 runs) and the reference's benchmark shape (--config small, small-frame kernel).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
rm -rf gpurun_out/prof
timeout -k 10 900 bash tools/gpu_prof.sh > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/driver_cmd -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/bench_driver_prof.json 2> $GRAFT_REPO_ROOT/$O/bench_driver_prof.err) || { echo FAIL driver prof; tail -5 $O/bench_driver_prof.err; exit 1; }
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$r.json 2>/dev/null || { echo FAIL bench; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/drv_$r.json').read().strip().splitlines()[-1]); print('driver cmd: %.1f GiB/s %.2f us/step kernel %.2f us c3 %.1f c5 %.1f' % (d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_avg_us'], d['c3']['value'], d['c5_host']['value']))"
done
timeout -k 10 300 python bench.py --config small --steps 20 --warmup 5 > $O/small.json 2>/dev/null || { echo FAIL small; exit 1; }
python3 -c "import json; d=json.loads(open('$O/small.json').read().strip().splitlines()[-1]); print('small: %.1f GiB/s %.3g frames/s %.2f us/step' % (d['value'], d['frames_per_s'], d['ms_per_step']*1e3))"
