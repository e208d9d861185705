#!/bin/bash
# Host-staged path: GPU tests that use it, then C5 bench lines, old (diag "hold") against the product.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
[ -n "$NOTEST" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_multi_gpu.py tests/test_c_client.py tests/test_go_binding.py tests/test_tx_fcs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_host.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/pytest_host.log; exit 1; }
[ -n "$NOTEST" ] || tail -2 gpurun_out/pytest_host.log
for rep in ${REPS:-1 2 3}; do
  for v in hold base; do
    lib=seqs_amd/lib/diag/libframesum_$v.so; [ "$v" = base ] && lib=seqs_amd/lib/libframesum.so
    FRAMESUM_LIB="$GRAFT_REPO_ROOT/$lib" timeout -k 10 200 python bench.py --config c5 --steps ${C5STEPS:-10} --warmup ${C5WARM:-3} --cpu-seconds 0 > gpurun_out/c5.json 2> gpurun_out/c5.err || { echo "C5 $v FAILED"; tail -20 gpurun_out/c5.err; exit 1; }
    echo "$v c5 $(python -c "import json; d=json.loads(open('gpurun_out/c5.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
  done
done
