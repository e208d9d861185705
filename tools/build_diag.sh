#!/bin/bash
# Diagnostic library builds (measurement only; the one switch left is -DFS_STAMPS):
#   tools/build_diag.sh <name> "<-D flags>"  ->  seqs_amd/lib/diag/libframesum_<name>.so
set -e
cd "$(dirname "$0")/../seqs_amd/csrc"
mkdir -p ../lib/diag
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -pthread --offload-arch=gfx950 -shared $2 \
  -o ../lib/diag/libframesum_$1.so framesum_kernel.hip framesum_shard.hip framesum_tables.cpp framesum_api.cpp \
  framesum_group.cpp -lrccl
