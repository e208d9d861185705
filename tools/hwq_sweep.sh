# The driver's bench command and the small-frame shape under GPU_MAX_HW_QUEUES 4 (HIP's default),
# 8 and 16 (hardware queues the process's streams map to), interleaved round by round.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/hwq; mkdir -p $O
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-6s %-14s %8.1f GiB/s %6.2f us/step' % (sys.argv[2], sys.argv[3], d['value'], d['ms_per_step']*1e3) + ''.join(' | %s %.1f' % (k, d[k]['value']) for k in ('c3','small','small_host','fill','fcs') if isinstance(d.get(k), dict)))" "$@"; }
for rep in 1 2; do for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/d_${q}_$rep.json 2> $O/d_${q}_$rep.err || { echo FAIL; tail -3 $O/d_${q}_$rep.err; exit 1; }
  summ $O/d_${q}_$rep.json q=$q driver
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --config small --steps 2000 --warmup 200 --cpu-seconds 0 > $O/s_${q}_$rep.json 2> $O/s_${q}_$rep.err || { echo FAIL; tail -3 $O/s_${q}_$rep.err; exit 1; }
  summ $O/s_${q}_$rep.json q=$q small2000
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --steps 2000 --warmup 500 --cpu-seconds 0 > $O/c_${q}_$rep.json 2> $O/c_${q}_$rep.err || { echo FAIL; tail -3 $O/c_${q}_$rep.err; exit 1; }
  summ $O/c_${q}_$rep.json q=$q c2_2000
done; done
