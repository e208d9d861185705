# round 6: same-box A/B of library builds (prod = seqs_amd/lib/libframesum.so, other names =
# seqs_amd/lib/ab/libframesum_<name>.so): the driver's command (C2, 20 steps), C2 at 2,000 steps and
# C3 at 1,000 steps, REPS interleaved rounds.  bash tools/lib_ab.sh prod <name> ...
cd $GRAFT_REPO_ROOT
O=gpurun_out/lib_ab; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 200 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -3 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-16s %9.1f GiB/s %8.2f us/step kernel %7.2f us' % ('$tag', d['value'], d['ms_per_step']*1e3, r['kernel_avg_us']))"; }
for rep in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    L=$PWD/seqs_amd/lib/ab/libframesum_$v.so; [ "$v" = prod ] && L=$PWD/seqs_amd/lib/libframesum.so
    for c in ${CFGS:-drv c2 c3}; do case $c in
      drv) FRAMESUM_LIB=$L run ${v}_drv python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 ;;
      c2) FRAMESUM_LIB=$L run ${v}_c2 python bench.py --steps 2000 --warmup 500 --cpu-seconds 0 ;;
      c3) FRAMESUM_LIB=$L run ${v}_c3 python bench.py --config c3 --steps 1000 --warmup 500 --cpu-seconds 0 ;;
      fill) FRAMESUM_LIB=$L run ${v}_fill python bench.py --op fill --steps 1000 --warmup 500 --cpu-seconds 0 ;;
    esac; done
  done
done
