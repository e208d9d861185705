#!/bin/bash
# PMC counter passes (each its own rocprofv3 run; kernel-trace only, no sys/runtime trace).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
cd /tmp
timeout -k 10 60 rocprofv3 -L > "$R/gpurun_out/pmc/counters.txt" 2>&1 || true
i=0
while read -r line; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $line --output-format csv -d "$R/gpurun_out/pmc/p$i" -o run -- python3 "$R/tools/prof_driver.py" --iters 20 > "$R/gpurun_out/pmc/p$i.log" 2>&1 || { echo "PMC pass $i ($line) failed"; tail -5 "$R/gpurun_out/pmc/p$i.log"; }
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_VMEM
FETCH_SIZE
TCC_HIT_sum TCC_MISS_sum
LIST
ls gpurun_out/pmc 2>/dev/null | head -30
