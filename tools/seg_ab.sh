# round 6: C3 bench of several library builds on one box (seqs_amd/lib/ab/libframesum_<name>.so, "prod")
#   bash tools/seg_ab.sh <kernel variant> <name> [<name> ...]
cd $GRAFT_REPO_ROOT
O=gpurun_out/seg_ab; mkdir -p $O
k=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    L=$PWD/seqs_amd/lib/ab/libframesum_$v.so; [ "$v" = prod ] && L=$PWD/seqs_amd/lib/libframesum.so
    FRAMESUM_LIB=$L timeout -k 10 200 python bench.py --config ${CFG:-c3} --kernel $k --steps 1000 --warmup 500 --cpu-seconds 0 > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-10s %8.1f GiB/s kernel %7.2f us' % ('$v', d['value'], r['kernel_avg_us']))"
  done
done
