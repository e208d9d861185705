# Speculative first rows in the one-pass kernel: parity (every op, every kernel choice), stamps of
# both builds, same-box A/B against HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_tx_fcs.py tests/test_dhcp_stale.py tests/test_c_client.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/spec_t.log 2>&1
rc=$?; tail -2 gpurun_out/spec_t.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/spec_t.log | head -20; exit 1; }
bash tools/gpu_stamps.sh headstamps:4 stamps:4 > gpurun_out/spec_stamps.log 2>&1 || { tail -5 gpurun_out/spec_stamps.log; exit 1; }
grep -E "== |fill\+desc|realtime|wave end quantiles" gpurun_out/spec_stamps.log
REPS=2 bash tools/gpu_abl.sh prod head
