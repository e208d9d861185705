#!/bin/bash
# Round profile collection (rocprofv3 on the GPU box):
#  1. kernel-trace + stats of the bench command itself (c2 and c3)   -> gpurun_out/prof/<cfg>/
#  2. PMC passes, each its own run, kernel-trace only (no sys/runtime trace):
#     FETCH_SIZE, WRITE_SIZE, SQ occupancy/wait, LDS           -> gpurun_out/prof/pmc_<cfg>_<i>/
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/prof"
export TMPDIR=/tmp
cd /tmp
for cfg in c2 c3; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof/$cfg" -o run -- \
    python3 "$R/bench.py" --config $cfg --cpu-seconds 10 --no-sub > "$R/gpurun_out/prof/bench_$cfg.json" 2> "$R/gpurun_out/prof/bench_$cfg.err" \
    || { echo "rocprof bench $cfg failed"; tail -5 "$R/gpurun_out/prof/bench_$cfg.err"; exit 1; }
  tail -1 "$R/gpurun_out/prof/bench_$cfg.json"
done
for cfg in c2 c3; do
  i=0
  while read -r line; do
    i=$((i+1))
    timeout -k 10 180 rocprofv3 --pmc $line --output-format csv -d "$R/gpurun_out/prof/pmc_${cfg}_$i" -o run -- \
      python3 "$R/tools/prof_driver.py" --config $cfg --iters 20 > "$R/gpurun_out/prof/pmc_${cfg}_$i.log" 2>&1 \
      || { echo "PMC $cfg pass $i ($line) failed"; tail -5 "$R/gpurun_out/prof/pmc_${cfg}_$i.log"; exit 1; }
  done <<'LIST'
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT
TCC_HIT_sum TCC_MISS_sum
LIST
done
# the TX fill with FCS append on C2: read and write bytes per launch (the
# dirty lines its 8 written bytes per frame leave), and its kernel trace
i=0
for line in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $line --output-format csv -d "$R/gpurun_out/prof/pmc_c2fill_$i" -o run -- \
    python3 "$R/tools/prof_driver.py" --config c2 --op fill --iters 20 > "$R/gpurun_out/prof/pmc_c2fill_$i.log" 2>&1 \
    || { echo "PMC fill pass $i failed"; tail -5 "$R/gpurun_out/prof/pmc_c2fill_$i.log"; exit 1; }
done
cd "$R" && python3 tools/prof_summary.py gpurun_out/prof gpurun_out/prof/summary
