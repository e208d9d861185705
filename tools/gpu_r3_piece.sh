# Mixed-kernel piece geometry sweep (diagnostic builds): parity of each on the mixed cases, then
# C3 same-box A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/piece; mkdir -p $O
L=$PWD/seqs_amd/lib/diag
for v in "$@"; do
  [ "$v" = prod ] && continue
  FRAMESUM_LIB=$L/libframesum_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mixed and (c3 or piece or random or giant or tiles or edge)" > $O/t_$v.log 2>&1
  rc=$?; echo "$v parity: $(tail -1 $O/t_$v.log)"; [ $rc -eq 0 ] || { grep -E "FAILED|assert" $O/t_$v.log | head -5; exit 1; }
done
run() { local name=$1; shift; timeout -k 10 120 "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; exit 1; }; python -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-10s %9.1f GiB/s %8.5f ms/step kernel %8.3f us' % ('$name', d['value'], d['ms_per_step'], r['kernel_avg_us']))"; }
for rep in 1 2; do
  for v in "$@"; do
    lib=$L/libframesum_$v.so; [ "$v" = prod ] && lib=$PWD/seqs_amd/lib/libframesum.so
    FRAMESUM_LIB=$lib run ${v}_$rep python bench.py --config c3 --steps 1000 --warmup 500 --cpu-seconds 0
  done
done
