# Streaming-kernel cost attribution: kernel time of diagnostic builds (tools/build_rx_diag.sh)
# with parts skipped, grid 1 and 2 workgroups per CU. usage: tools/gpu_r3_diag.sh d0 d1 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3diag; mkdir -p $O
for d in "$@"; do
  for g in 1 2; do
    FRAMESUM_LIB=$PWD/tools/diag_lib/libfs_$d.so FS_RX_GRID=$g timeout -k 10 120 \
      python bench.py --cpu-seconds 0 --kernel 6 --steps 1000 --warmup 300 > $O/${d}_g$g.json 2> $O/${d}_g$g.err \
      || { echo "FAIL $d g$g"; tail -3 $O/${d}_g$g.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${d}_g$g.json')); r=d['roofline']; print('$d g$g', d['value'], r['kernel_avg_us'])"
  done
done
