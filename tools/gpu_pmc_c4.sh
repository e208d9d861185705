#!/bin/bash
# Instruction mix and waits of the one-pass kernel on a C4-size batch (16 tiles per wave).
set -o pipefail
R="$GRAFT_REPO_ROOT"
rm -rf "$R/gpurun_out/pmc4"; mkdir -p "$R/gpurun_out/pmc4"
export TMPDIR=/tmp
cd /tmp
i=0
while read -r line; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $line --output-format csv -d "$R/gpurun_out/pmc4/c4k0_$i" -o run -- \
    python3 "$R/tools/prof_driver.py" --config c2 --frames 1048576 --iters 6 > "$R/gpurun_out/pmc4/c4k0_$i.log" 2>&1 \
    || { echo "PMC pass $i failed"; tail -5 "$R/gpurun_out/pmc4/c4k0_$i.log"; exit 1; }
done <<'LIST'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
LIST
cd "$R" && python3 tools/pmc_print.py gpurun_out/pmc4
