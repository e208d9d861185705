# C4 through bench.py on one GPU (plain and with the 1-rank process group), the C2 line with
# --force-gather, and the multi-GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c4; mkdir -p $O
run() { local name=$1; shift; timeout -k 10 240 "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; exit 1; }; python -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-12s %9.1f GiB/s %8.5f ms/step kernel %8.3f us' % ('$name', d['value'], d['ms_per_step'], r['kernel_avg_us']), d['config'].get('kernel_only_gibs',''))"; }
run c4 python bench.py --config c4 --steps 20 --warmup 5 --cpu-seconds 0
run c4fg python bench.py --config c4 --steps 20 --warmup 5 --cpu-seconds 0 --force-gather
timeout -k 10 300 python -u -m pytest tests/test_multi_gpu.py tests/test_go_binding.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; exit $rc
