#!/bin/bash
# One PMC pass (kernel-trace only; counters: $PMC, default the instruction mix) per (library,
# kernel variant) pair on c2:
# tools/gpu_pmc_v.sh base:1 base:3 wd1:3 ...   -> gpurun_out/pmcv/<lib>-k<v>_1/
set -o pipefail
R="$GRAFT_REPO_ROOT"
rm -rf "$R/gpurun_out/pmcv"; mkdir -p "$R/gpurun_out/pmcv"
export TMPDIR=/tmp
cd /tmp
for pair in "$@"; do
  v=${pair%%:*}; k=${pair##*:}
  lib="$R/seqs_amd/lib/diag/libframesum_$v.so"; [ "$v" = base ] && lib="$R/seqs_amd/lib/libframesum.so"
  export FRAMESUM_LIB="$lib"
  timeout -s KILL 90 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY} \
    --output-format csv -d "$R/gpurun_out/pmcv/${v}-k${k}_1" -o run -- \
    python3 "$R/tools/prof_driver.py" --config c2 --iters 20 --kernel $k > "$R/gpurun_out/pmcv/${v}-k${k}.log" 2>&1 \
    || { echo "PMC $pair failed"; tail -5 "$R/gpurun_out/pmcv/${v}-k${k}.log"; exit 1; }
done
cd "$R" && python3 tools/pmc_print.py gpurun_out/pmcv
