# round 6: the segment kernel against round 5's piece kernel on one box
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6c; mkdir -p $O
b() { timeout -k 10 200 python bench.py "$@" --cpu-seconds 0 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$*', round(d['value'],1), d['unit'].split()[0], 'kernel', r['kernel_avg_us'], 'us', r.get('kernel_chosen'))"; }
for rep in 1 2; do
  b --config c3 --kernel 2 --steps 1000 --warmup 500
  b --config c3 --kernel 3 --steps 1000 --warmup 500
done
b --config c3 --kernel 0 --steps 20 --warmup 5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
exit $rc
