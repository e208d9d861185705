# The N>1 bench loop's cost on one GPU: --force-gather (a 1-rank process group: the rounds, joins
# and waits without transfers) against plain, 20 and 2,000 steps, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3g; mkdir -p $O
run() { local name=$1; shift; timeout -k 10 180 "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; exit 1; }; python -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', d['value'], d['ms_per_step'], r['kernel_avg_us'])"; }
for k in 1 2 3; do
  run plain20_$k python bench.py --steps 20 --warmup 5 --cpu-seconds 0
  run gather20_$k python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --force-gather
done
run plain2000 python bench.py --steps 2000 --warmup 500 --cpu-seconds 0
run gather2000 python bench.py --steps 2000 --warmup 500 --cpu-seconds 0 --force-gather
