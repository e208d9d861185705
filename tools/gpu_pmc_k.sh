#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) of the digest kernel per variant:
# tools/gpu_pmc_k.sh <cfg> <kernel variants...>   -> gpurun_out/pmck/<cfg>k<v>_<pass>/
set -o pipefail
R="$GRAFT_REPO_ROOT"
cfg=$1; shift
mkdir -p "$R/gpurun_out/pmck"
export TMPDIR=/tmp
cd /tmp
for k in "$@"; do
  i=0
  while read -r line; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $line --output-format csv -d "$R/gpurun_out/pmck/${cfg}k${k}_$i" -o run -- \
      python3 "$R/tools/prof_driver.py" --config $cfg --iters 20 --kernel $k > "$R/gpurun_out/pmck/${cfg}k${k}_$i.log" 2>&1 \
      || { echo "PMC $cfg k$k pass $i ($line) failed"; tail -5 "$R/gpurun_out/pmck/${cfg}k${k}_$i.log"; exit 1; }
  done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_WAVES
FETCH_SIZE
LIST
done
cd "$R" && python3 tools/pmc_print.py gpurun_out/pmck
