# Same-box C4 (and C2) A/B of libraries: tools/gpu_c4ab.sh prod r2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/c4ab; mkdir -p $O
lib() { [ "$1" = prod ] && echo "$PWD/seqs_amd/lib/libframesum.so" || echo "$PWD/seqs_amd/lib/diag/libframesum_$1.so"; }
run() { local name=$1; shift; timeout -k 10 240 "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; exit 1; }; python -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-12s %9.1f GiB/s %8.5f ms/step kernel %8.3f us' % ('$name', d['value'], d['ms_per_step'], r['kernel_avg_us']))"; }
for rep in 1 2; do
  for v in "$@"; do
    FRAMESUM_LIB=$(lib $v) run ${v}_c4_$rep python bench.py --config c4 --steps 20 --warmup 20 --cpu-seconds 0
    FRAMESUM_LIB=$(lib $v) run ${v}_c2_$rep python bench.py --steps 2000 --warmup 500 --cpu-seconds 0
  done
done
