#!/bin/bash
# Round 4: the mixed-length kernel's pipelined pass boundary: GPU suite, then same-box A/B against the
# build without it (seqs_amd/lib/ab/libframesum_mixnp.so) on C3 and C2.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; exit 1; }
timeout -k 10 400 python tools/env_sweep.py --rounds 3 --only "base+lib=mixnp" --extra "--config c3" --out $O/c3_20.jsonl || exit 1
timeout -k 10 400 python tools/env_sweep.py --rounds 2 --steps 2000 --warmup 500 --only "base+lib=mixnp" --extra "--config c3" --out $O/c3_2000.jsonl || exit 1
timeout -k 10 400 python tools/env_sweep.py --rounds 2 --only "base+lib=mixnp" --out $O/c2_20.jsonl || exit 1
# the small-frame kernel with two CRC chains (seqs_amd/lib/ab/libframesum_s2.so): parity through it, then A/B
FRAMESUM_LIB=$GRAFT_REPO_ROOT/seqs_amd/lib/ab/libframesum_s2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_length_sweep.py -m gpu -x -q -k small --timeout 300 --timeout-method thread > $O/s2_tests.log 2>&1; rc=$?
tail -3 $O/s2_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/s2_tests.log | head -30; exit 1; }
timeout -k 10 400 python tools/env_sweep.py --rounds 3 --only "base+lib=s2" --extra "--config small" --out $O/small_20.jsonl || exit 1
timeout -k 10 400 python tools/env_sweep.py --rounds 2 --steps 2000 --warmup 500 --only "base+lib=s2" --extra "--config small" --out $O/small_2000.jsonl || exit 1
