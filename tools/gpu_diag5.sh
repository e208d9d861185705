#!/bin/bash
# c2 stamps + instruction-mix PMC pass on the current library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc5; mkdir -p gpurun_out/pmc5
FRAMESUM_LIB="$R/seqs_amd/lib/diag/libframesum_st.so" timeout -k 10 120 python tools/stamps.py --config c2 > gpurun_out/stamps_c2.log 2>&1 || { echo "STAMPS FAILED"; tail -5 gpurun_out/stamps_c2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_c2.log | head -12
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES --output-format csv -d "$R/gpurun_out/pmc5/c2_1" -o run -- python3 "$R/tools/prof_driver.py" --config c2 --iters 20 > "$R/gpurun_out/pmc5/c2_1.log" 2>&1 || { echo "PMC failed"; tail -3 "$R/gpurun_out/pmc5/c2_1.log"; exit 1; }
cd "$R" && python3 tools/pmc_print.py gpurun_out/pmc5
