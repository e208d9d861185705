#!/bin/bash
# C3 A/B of two libraries (prod and seqs_amd/lib/diag/libframesum_<name>.so): kernel trace + PMC
# passes of the mixed-length kernel (variant 2) on C3 with each, then bench lines interleaved.
# usage: tools/gpu_mixed_ab.sh <name>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/mixab; mkdir -p $O; export TMPDIR=/tmp
for lib in prod $1; do
  L=$PWD/seqs_amd/lib/libframesum.so; [ $lib = prod ] || L=$PWD/seqs_amd/lib/diag/libframesum_$lib.so
  i=0
  for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
           "FETCH_SIZE"; do
    i=$((i+1))
    FRAMESUM_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$O/${lib}_$i" -o run -- \
      python3 tools/prof_driver.py --config c3 --iters 20 --kernel 2 > "$O/${lib}_$i.log" 2>&1 || { echo "PMC $lib $i failed"; tail -5 "$O/${lib}_$i.log"; exit 1; }
  done
  FRAMESUM_LIB=$L timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${lib}_trace" -o run -- \
    python3 tools/prof_driver.py --config c3 --iters 50 --kernel 2 > "$O/${lib}_t.log" 2>&1 || { echo "trace $lib failed"; exit 1; }
done
python3 tools/pmc_print.py "$O" && python3 tools/trace_stats.py "$O"
REPS=2 CFGS=c3 timeout -k 10 600 bash tools/gpu_abl.sh prod $1
