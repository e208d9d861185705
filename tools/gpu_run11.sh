#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 ./tools/hbm_read_bw > gpurun_out/hbm_98.log 2>&1 || { echo "HBM BW FAILED"; tail -5 gpurun_out/hbm_98.log; exit 1; }
cat gpurun_out/hbm_98.log
timeout -k 10 200 ./tools/hbm_read_bw 1000000000 > gpurun_out/hbm_1g.log 2>&1 || { echo "HBM BW 1G FAILED"; tail -5 gpurun_out/hbm_1g.log; exit 1; }
cat gpurun_out/hbm_1g.log
bash tools/gpu_ab.sh base nt
for st in 1 2 3; do
  timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 300 --streams $st > gpurun_out/b_s$st.log 2>&1 || { echo "BENCH streams=$st FAILED"; tail -5 gpurun_out/b_s$st.log; exit 1; }
  echo "streams=$st $(python -c "import json; d=json.loads(open('gpurun_out/b_s$st.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])")"
  timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 300 --streams $st --config c3 > gpurun_out/b3_s$st.log 2>&1 || { echo "BENCH c3 streams=$st FAILED"; tail -5 gpurun_out/b3_s$st.log; exit 1; }
  echo "c3 streams=$st $(python -c "import json; d=json.loads(open('gpurun_out/b3_s$st.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])")"
done
