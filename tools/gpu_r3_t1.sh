set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py tests/test_tx_fcs.py -k stream -x -v --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/t1.log
exit $rc
