#!/bin/bash
# One launcher for every GPU-box session (replaces the per-session gpu_r*.sh scripts).
#   bash tools/gpu.sh <name> <step> [<step> ...]        (run through gpurun from the repo root)
# Output goes to gpurun_out/<name>/. Steps run in order; the first failing step ends the call
# (every GPU step has its own timeout -k; nothing is retried). Steps:
#   tests[=<pytest -k expr>]   the GPU suite (or the tests matching the -k expression)
#   smoke                      __graft_entry__.smoke()
#   driver[=N]                 the driver's bench command (--gpus 1 --steps 20 --warmup 5), N runs (1)
#   bench=<args>               bench.py <args> once (e.g. bench="--config small --kernel 0")
#   prof                       tools/gpu_prof.sh: rocprofv3 trace + stats of C2 / C3, PMC passes
#   driver_prof                the driver's command under rocprofv3 --kernel-trace --stats
#   abl=<lib>,<lib>,...        tools/gpu_abl.sh on those libraries (prod = the shipped one)
#   pmc=<tag>:<kernel>[:cfg]   PMC passes + a kernel trace of one kernel variant (tools/prof_driver.py)
#   py=<script args>           python3 <script args> (a measurement tool under tools/)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
NAME=$1; shift
O=gpurun_out/$NAME; mkdir -p $O
export TMPDIR=/tmp
summ() {  # one line per bench JSON
  python3 - "$1" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
s = "%.1f %s %.2f us/step kernel %.2f us frac %.3f" % (d["value"], d["unit"].split()[0], d["ms_per_step"] * 1e3,
                                                      r.get("kernel_avg_us", 0), r.get("frac", 0))
for k in ("c3", "small", "small_host", "fill", "fcs", "c5_host"):
    if isinstance(d.get(k), dict) and "value" in d[k]:
        s += " | %s %.1f" % (k, d[k]["value"])
print(s)
EOF
}
i=0
for step in "$@"; do
  i=$((i+1))
  key=${step%%=*}; arg=""; [ "$key" != "$step" ] && arg=${step#*=}
  case $key in
  tests)
    K=(); [ -n "$arg" ] && K=(-k "$arg")
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${K[@]}" > $O/tests_$i.log 2>&1
    rc=$?; tail -2 $O/tests_$i.log
    [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests_$i.log | head -30; exit 1; } ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
    tail -1 $O/smoke.log ;;
  driver)
    for r in $(seq 1 ${arg:-1}); do
      timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_${i}_$r.json 2> $O/driver_${i}_$r.err || { echo FAIL driver; tail -5 $O/driver_${i}_$r.err; exit 1; }
      echo "driver: $(summ $O/driver_${i}_$r.json)"
    done ;;
  bench)
    timeout -k 10 400 python bench.py $arg > $O/bench_$i.json 2> $O/bench_$i.err || { echo "FAIL bench $arg"; tail -5 $O/bench_$i.err; exit 1; }
    echo "bench $arg: $(summ $O/bench_$i.json)" ;;
  prof)
    rm -rf gpurun_out/prof
    timeout -k 10 900 bash tools/gpu_prof.sh > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
    tail -4 $O/prof.log ;;
  driver_prof)
    (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/driver_cmd -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/driver_prof.json 2> $GRAFT_REPO_ROOT/$O/driver_prof.err) || { echo FAIL driver_prof; tail -5 $O/driver_prof.err; exit 1; }
    echo "driver under rocprofv3: $(summ $O/driver_prof.json)" ;;
  abl)
    timeout -k 10 1000 bash tools/gpu_abl.sh ${arg//,/ } || exit 1 ;;
  pmc)
    IFS=: read -r tag k cfg <<< "$arg"
    CFG=${cfg:-c2} timeout -k 10 600 bash tools/gpu_pmc_variant.sh $tag $k || exit 1 ;;
  py)
    timeout -k 10 600 python3 $arg > $O/py_$i.log 2>&1 || { echo "FAIL py $arg"; tail -10 $O/py_$i.log; exit 1; }
    tail -20 $O/py_$i.log ;;
  *)
    echo "unknown step $step"; exit 2 ;;
  esac
done
