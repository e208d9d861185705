# Round-3 final check: whole GPU suite, smoke(), the driver's exact bench command (twice), C3 and
# the 1-GPU C4 line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head -20; exit 1; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
run() { local name=$1; shift; timeout -k 10 240 "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; exit 1; }; python -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-10s %9.1f GiB/s %8.5f ms/step kernel %8.3f us frac %.4f' % ('$name', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac']))"; }
run driver1 python bench.py --gpus 1 --steps 20 --warmup 5
run driver2 python bench.py --gpus 1 --steps 20 --warmup 5
run c2_2000 python bench.py --steps 2000 --warmup 500 --cpu-seconds 0
run c3 python bench.py --config c3 --steps 1000 --warmup 500 --cpu-seconds 0
run c4 python bench.py --config c4 --steps 20 --warmup 20 --cpu-seconds 0
