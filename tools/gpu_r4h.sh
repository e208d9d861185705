#!/bin/bash
# Round 4 combined call: the final check and profile set (tools/gpu_r4_final.sh: GPU suite, smoke, profiles,
# the driver's command), then the A/Bs of the mixed kernel's pipelined pass boundary (against
# seqs_amd/lib/ab/libframesum_mixnp.so) and of the two-chain small-frame kernel (libframesum_s2.so,
# with its parity cases first).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r4_final.sh || exit 1
O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 400 python tools/env_sweep.py --rounds 2 --only "base+lib=mixnp" --extra "--config c3" --out $O/c3_20.jsonl || exit 1
timeout -k 10 400 python tools/env_sweep.py --rounds 2 --steps 2000 --warmup 500 --only "base+lib=mixnp" --extra "--config c3" --out $O/c3_2000.jsonl || exit 1
FRAMESUM_LIB=$GRAFT_REPO_ROOT/seqs_amd/lib/ab/libframesum_s2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_length_sweep.py -m gpu -x -q -k small --timeout 300 --timeout-method thread > $O/s2_tests.log 2>&1; rc=$?
tail -3 $O/s2_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/s2_tests.log | head -30; exit 1; }
timeout -k 10 400 python tools/env_sweep.py --rounds 2 --only "base+lib=s2" --extra "--config small" --out $O/small_20.jsonl || exit 1
timeout -k 10 400 python tools/env_sweep.py --rounds 2 --steps 2000 --warmup 500 --only "base+lib=s2" --extra "--config small" --out $O/small_2000.jsonl || exit 1
