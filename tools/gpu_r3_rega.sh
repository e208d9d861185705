set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_tx_fcs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rega_t.log 2>&1
rc=$?; tail -2 gpurun_out/rega_t.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/rega_t.log | head; exit 1; }
bash tools/gpu_stamps.sh basestamps:4 stamps:4 && bash tools/gpu_abl.sh prod base
