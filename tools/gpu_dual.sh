set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_tx_fcs.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dual" > gpurun_out/dual_tests.log 2>&1 || { tail -30 gpurun_out/dual_tests.log; exit 1; }
tail -3 gpurun_out/dual_tests.log
for k in 4 5 4 5; do timeout -k 10 120 python bench.py --cpu-seconds 0 --kernel $k > gpurun_out/dual_b$k.log 2>&1 || exit 1; tail -1 gpurun_out/dual_b$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('kernel $k', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'] if 'kernel_avg_us' in d['roofline'] else d['roofline'])"; done
for k in 4 5; do timeout -k 10 120 python bench.py --cpu-seconds 0 --kernel $k --steps 20 --warmup 5 > gpurun_out/dual_s$k.log 2>&1 || exit 1; tail -1 gpurun_out/dual_s$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('K=20 kernel $k', d['value'], d['ms_per_step'])"; done
