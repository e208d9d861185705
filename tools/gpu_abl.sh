# Same-box A/B of libraries: tools/gpu_abl.sh prod base ...  ("prod" = seqs_amd/lib/libframesum.so,
# other names = seqs_amd/lib/diag/libframesum_<name>.so), two interleaved rounds of C2 (2,000 and
# 20 steps) and C3 bench lines; REPS / CFGS override.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abl; mkdir -p $O
lib() { [ "$1" = prod ] && echo "$PWD/seqs_amd/lib/libframesum.so" || echo "$PWD/seqs_amd/lib/diag/libframesum_$1.so"; }
run() { local name=$1; shift; timeout -k 10 180 "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; exit 1; }; python -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-22s %9.1f GiB/s %8.5f ms/step kernel %7.3f us' % ('$name', d['value'], d['ms_per_step'], r['kernel_avg_us']))"; }
for rep in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    L=$(lib $v)
    for c in ${CFGS:-c2 c2k20 c3}; do case $c in
      c2) FRAMESUM_LIB=$L run ${v}_c2_$rep python bench.py --steps 2000 --warmup 500 --cpu-seconds 0 ;;
      c2k20) FRAMESUM_LIB=$L run ${v}_c2k20_$rep python bench.py --steps 20 --warmup 5 --cpu-seconds 0 ;;
      c3) FRAMESUM_LIB=$L run ${v}_c3_$rep python bench.py --config c3 --steps 1000 --warmup 500 --cpu-seconds 0 ;;
    esac; done
  done
done
