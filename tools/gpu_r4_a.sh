#!/bin/bash
# Round 4, first check: the whole GPU suite (new fault-injection tests through the test library,
# the warmed 'auto' length sweep), the driver's bench command with the C3 / C5 sub-records, the
# reference-benchmark shape (--config small), and the timed region under a HIP-API + kernel trace
# lined up with the region's host clocks (tools/region_attr.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4a; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head -20; exit 1; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
T0=$(date +%s.%N)
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err || { echo FAIL driver; tail -5 $O/driver.err; exit 1; }
python3 -c "import sys,time; print('driver command wall %.1f s' % (time.time() - float(sys.argv[1])))" $T0
python - <<'EOF'
import json
d = json.loads(open("gpurun_out/r4a/driver.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("driver %.1f GiB/s %.5f ms/step kernel %.3f us frac %.4f" % (d["value"], d["ms_per_step"], r["kernel_avg_us"], r["frac"]))
print("c3", json.dumps(d.get("c3")))
print("c5", json.dumps(d.get("c5_host")))
EOF
timeout -k 10 240 python bench.py --config small --steps 20 --warmup 5 > $O/small.json 2> $O/small.err || { echo FAIL small; tail -5 $O/small.err; exit 1; }
timeout -k 10 240 python bench.py --config small --steps 2000 --warmup 500 --cpu-seconds 0 > $O/small2000.json 2> $O/small2000.err || { echo FAIL small2000; tail -5 $O/small2000.err; exit 1; }
python - <<'EOF'
import json
for f in ("small", "small2000"):
    d = json.loads(open(f"gpurun_out/r4a/{f}.json").read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, "%.1f GiB/s %.3e frames/s %.5f ms/step kernel %.3f us frac %.4f incl-meta %.1f GB/s" % (
        d["value"], d["frames_per_s"], d["ms_per_step"], r["kernel_avg_us"], r["frac"], r["achieved_incl_metadata"]),
        "cpu", json.dumps(d.get("cpu_baseline")))
EOF
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf $O/rtrace $O/clk.json
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O/rtrace -- python3 bench.py --steps 20 --warmup 5 --no-sub --cpu-seconds 0 --region-clocks $O/clk.json > $O/rtrace.log 2>&1 || { echo FAIL rtrace; tail -5 $O/rtrace.log; exit 1; }
python3 tools/region_attr.py $O/rtrace $O/clk.json | tee $O/region_attr.txt
# keep the small CSVs only (the API trace of the whole run is large)
find $O/rtrace -name "*hip_api_trace.csv" -size +20M -delete
timeout -k 10 120 tools/tile_pattern w4 > $O/tile_pattern_w4.log 2>&1 || { echo FAIL tile_pattern; tail -3 $O/tile_pattern_w4.log; exit 1; }
cat $O/tile_pattern_w4.log
echo done
