cd $GRAFT_REPO_ROOT
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mixed and not pieces" > $O/t1.log 2>&1; rc=$?
tail -15 $O/t1.log
exit $rc
