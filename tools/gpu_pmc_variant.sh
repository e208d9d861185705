# Round 3: PMC passes (kernel trace only) + a kernel trace for kernel variants on C2.
# usage: tools/gpu_pmc_variant.sh <tag> <kernel> [<tag> <kernel> ...]   (FS_RX_GRID passes through)
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r3pmc"; mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
P3="FETCH_SIZE"
while [ $# -ge 2 ]; do
  tag=$1; k=$2; shift 2
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$O/${tag}_$i" -o run -- \
      python3 "$R/tools/prof_driver.py" --config ${CFG:-c2} --iters 20 --kernel $k > "$O/${tag}_$i.log" 2>&1 \
      || { echo "PMC $tag $i failed"; tail -5 "$O/${tag}_$i.log"; exit 1; }
  done
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${tag}_trace" -o run -- \
    python3 "$R/tools/prof_driver.py" --config ${CFG:-c2} --iters 50 --kernel $k > "$O/${tag}_t.log" 2>&1 \
    || { echo "trace $tag failed"; exit 1; }
done
cd "$R" && python3 tools/pmc_print.py "$O" && python3 tools/trace_stats.py "$O"
