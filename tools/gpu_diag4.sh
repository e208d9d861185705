#!/bin/bash
# stamps (FS_STAMPS build "st") for c2/c3 + instruction-mix PMC passes on the current library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc4
for cfg in c2 c3; do
  FRAMESUM_LIB="$R/seqs_amd/lib/diag/libframesum_st.so" timeout -k 10 120 python tools/stamps.py --config $cfg > gpurun_out/stamps_$cfg.log 2>&1 || { echo "STAMPS FAILED"; tail -5 gpurun_out/stamps_$cfg.log; exit 1; }
  echo "== stamps $cfg"; grep -v amdgpu.ids gpurun_out/stamps_$cfg.log
done
export TMPDIR=/tmp
cd /tmp
for cfg in c2 c3; do
i=0
while read -r line; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $line --output-format csv -d "$R/gpurun_out/pmc4/${cfg}_$i" -o run -- python3 "$R/tools/prof_driver.py" --config $cfg --iters 20 > "$R/gpurun_out/pmc4/${cfg}_$i.log" 2>&1 || { echo "PMC pass $i failed"; tail -3 "$R/gpurun_out/pmc4/${cfg}_$i.log"; exit 1; }
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
FETCH_SIZE
LIST
done
cd "$R" && python3 tools/pmc_print.py gpurun_out/pmc4
