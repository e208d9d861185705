#!/bin/bash
# Host-staged TX fill: the fill GPU tests, then old (diag "hold") against the product.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_tx_fcs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fill.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/pytest_fill.log; exit 1; }
tail -2 gpurun_out/pytest_fill.log
for rep in 1 2; do
  for v in hold base; do
    lib=seqs_amd/lib/diag/libframesum_$v.so; [ "$v" = base ] && lib=seqs_amd/lib/libframesum.so
    echo "== $v"
    FRAMESUM_LIB="$GRAFT_REPO_ROOT/$lib" timeout -k 10 200 python tools/host_fill_bench.py 2>/dev/null || { echo "FILL BENCH $v FAILED"; exit 1; }
  done
done
