# Diagnostic builds of libframesum.so with parts of the streaming kernel skipped (FS_RX_DIAG
# bitmask: 1 finish, 2 combine, 4 head rows, 8 table lookups). Results are wrong by design;
# only the kernel time is read. usage: tools/build_rx_diag.sh 1 2 4 ...
set -e
cd "$(dirname "$0")/../seqs_amd/csrc"
O=/tmp/rxdiag; mkdir -p $O ../../tools/diag_lib
F="-O3 -std=c++17 -fPIC -pthread --offload-arch=gfx950"
for s in framesum_kernel.hip framesum_shard.hip framesum_tables.cpp framesum_api.cpp framesum_group.cpp; do
  [ $O/$s.o -nt $s ] || /opt/rocm/bin/hipcc $F -c $s -o $O/$s.o &
done
wait
for d in "$@"; do
  ( /opt/rocm/bin/hipcc $F -DFS_RX_DIAG=$d -c framesum_rx.hip -o $O/rx_$d.o &&
    /opt/rocm/bin/hipcc $F -shared -o ../../tools/diag_lib/libfs_d$d.so $O/rx_$d.o $O/*.hip.o $O/*.cpp.o -lrccl ) &
done
wait
ls -la ../../tools/diag_lib
