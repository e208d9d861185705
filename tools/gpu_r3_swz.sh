# Header-slot swizzle: one-pass parity (RX, TX, FCS), then LDS PMC on C2 and bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3s; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_tx_fcs.py tests/test_dhcp_stale.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/t.log | head; exit 1; }
bash tools/gpu_r3_pmc.sh swz 4 && bash tools/gpu_r3_gather.sh
