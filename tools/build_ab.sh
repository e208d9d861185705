#!/bin/bash
# A/B build of the product library with another kernel source: seqs_amd/lib/ab/libframesum_<name>.so
# (measurement tool; tools/env_sweep.py lib=<name> runs the bench with it through FRAMESUM_LIB).
# usage: tools/build_ab.sh <name> <framesum_kernel.hip to use | git revision>
#   e.g. tools/build_ab.sh old a05f721     (that commit's kernel, this tree's host sources)
set -e
name=$1; src=$2
R=$(cd "$(dirname "$0")/.." && pwd)
d=$(mktemp -d)/a/b/csrc; mkdir -p "$d" "$d/../../include"
cp "$R"/seqs_amd/csrc/*.cpp "$R"/seqs_amd/csrc/*.h "$R"/seqs_amd/csrc/framesum_shard.hip "$d"/
cp "$R"/include/framesum.h "$d/../../include/"
if [ -f "$src" ]; then cp "$src" "$d/framesum_kernel.hip"; else git -C "$R" show "$src:seqs_amd/csrc/framesum_kernel.hip" > "$d/framesum_kernel.hip"; fi
mkdir -p "$R/seqs_amd/lib/ab"
cd "$d" && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -pthread --offload-arch=gfx950 -shared \
  -o "$R/seqs_amd/lib/ab/libframesum_$name.so" framesum_kernel.hip framesum_shard.hip framesum_tables.cpp \
  framesum_api.cpp framesum_group.cpp -lrccl
ls -la "$R/seqs_amd/lib/ab/libframesum_$name.so"
