#!/bin/bash
# Short-region anatomy: the C2 loop's 20-step regions plain, then under a rocprofv3 kernel trace,
# lined up with the host clocks (tools/region_trace.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python3 tools/region_trace.py ${RT_ARGS} > gpurun_out/rt_plain.log 2>&1 || { echo FAIL plain; tail gpurun_out/rt_plain.log; exit 1; }
python3 -c "
import json
r=[json.loads(l) for l in open('gpurun_out/rt_plain.log') if l.startswith('{')]
print('plain us/step', ' '.join(f\"{x['us_per_step']:.2f}\" for x in r)); print('enqueue us', ' '.join(f\"{x['host_enqueue_us']:.0f}\" for x in r))"
rm -rf gpurun_out/rt_trace
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rt_trace -- python3 tools/region_trace.py ${RT_ARGS} > gpurun_out/rt_prof.log 2>&1 || { echo FAIL prof; tail gpurun_out/rt_prof.log; exit 1; }
python3 tools/region_trace.py --analyse gpurun_out/rt_trace gpurun_out/rt_prof.log
