# Same-box A/B of the small-frame record (variant 8, bench.py --config small) between library builds:
# tools/small_ab.sh prod <name> ...  (other names: seqs_amd/lib/diag/libframesum_<name>.so); STEPS (20)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sab; mkdir -p $O
for rep in 1 2 3; do for v in "$@"; do
  L=$PWD/seqs_amd/lib/libframesum.so; [ $v != prod ] && L=$PWD/seqs_amd/lib/diag/libframesum_$v.so
  for st in ${STEPS:-20 2000}; do
    FRAMESUM_LIB=$L timeout -k 10 120 python bench.py --config small --kernel 8 --steps $st --warmup $([ $st = 20 ] && echo 5 || echo 200) --cpu-seconds 0 > $O/${v}_${st}_$rep.json 2> $O/${v}_${st}_$rep.err || { echo FAIL $v; tail -3 $O/${v}_${st}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/${v}_${st}_$rep.json').read().strip().splitlines()[-1]); print('%-8s steps %5s %8.1f GiB/s %7.2f us/step kernel %6.2f us' % ('$v', '$st', d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_avg_us']))"
  done
done; done
