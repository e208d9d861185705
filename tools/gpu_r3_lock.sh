# Lockstep probe (diagnostic build: a workgroup barrier after each refilled block of the one-pass
# kernel). SAFE ONLY where every wave runs the same blocks: C2 forced to the one-pass kernel
# (--kernel 4, one 25-row tile per wave). Never run it on other batches.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/lock; mkdir -p $O
L=$PWD/seqs_amd/lib/diag
FRAMESUM_LIB=$L/libframesum_lockstamps.so timeout -k 10 120 python tools/stamps.py --config c2 --kernel 4 > $O/stamps_lock.log 2>&1 || { tail -5 $O/stamps_lock.log; exit 1; }
grep -E "fill\+desc|main loop  |realtime|wave end quantiles" $O/stamps_lock.log
run() { local name=$1; shift; timeout -k 10 120 "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; exit 1; }; python -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-14s %9.1f GiB/s %8.5f ms/step kernel %8.3f us' % ('$name', d['value'], d['ms_per_step'], r['kernel_avg_us']))"; }
for rep in 1 2; do
  FRAMESUM_LIB=$L/libframesum_lockstep.so run lock_c2_$rep python bench.py --kernel 4 --steps 2000 --warmup 500 --cpu-seconds 0
  run prod_c2_$rep python bench.py --kernel 4 --steps 2000 --warmup 500 --cpu-seconds 0
  FRAMESUM_LIB=$L/libframesum_lockstep.so run lock_k20_$rep python bench.py --kernel 4 --steps 20 --warmup 5 --cpu-seconds 0
  run prod_k20_$rep python bench.py --kernel 4 --steps 20 --warmup 5 --cpu-seconds 0
done
