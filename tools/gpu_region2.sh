#!/bin/bash
# Short-region wall time under host wait modes: default, hipDeviceScheduleSpin, HSA_ENABLE_INTERRUPT=0.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
summ() { python3 -c "
import json,sys
r=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')]
print(sys.argv[2], 'us/step', ' '.join(f\"{x['us_per_step']:.2f}\" for x in r))" "$1" "$2"; }
for mode in default spin; do
  for intr in 1 0; do
    f=gpurun_out/rt_${mode}_${intr}.log
    arg=""; [ $mode = spin ] && arg=--spin
    HSA_ENABLE_INTERRUPT=$intr timeout -k 10 120 python3 tools/region_trace.py $arg $RT_ARGS > $f 2>&1 || { echo FAIL $mode $intr; tail $f; exit 1; }
    summ $f "$mode intr=$intr"
  done
done
