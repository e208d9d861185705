#!/bin/bash
# Round 4: prepared-call parity (main library), then the small-frame kernel with 37 KB of LDS (Z4 +
# byte table, 8-row slots: four workgroups per CU; seqs_amd/lib/ab/libframesum_s3.so): its parity
# cases, then A/B on the reference's benchmark shape.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "prepared" --timeout 120 --timeout-method thread > $O/prep_tests.log 2>&1; rc=$?
tail -2 $O/prep_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/prep_tests.log | head -30; exit 1; }
FRAMESUM_LIB=$GRAFT_REPO_ROOT/seqs_amd/lib/ab/libframesum_s3.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_length_sweep.py tests/test_tx_fcs.py -m gpu -x -q -k small --timeout 300 --timeout-method thread > $O/s3_tests.log 2>&1; rc=$?
tail -2 $O/s3_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/s3_tests.log | head -30; exit 1; }
timeout -k 10 400 python tools/env_sweep.py --rounds 3 --only "base+lib=s3" --extra "--config small" --out $O/small_20.jsonl || exit 1
timeout -k 10 400 python tools/env_sweep.py --rounds 2 --steps 2000 --warmup 500 --only "base+lib=s3" --extra "--config small" --out $O/small_2000.jsonl || exit 1
