set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/hattr; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --hip-trace --output-format csv -d $O/tr -o run -- python3 tools/host_attr.py run $O/clk.json > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
tail -1 $O/run.log
python3 tools/host_attr.py attr $O/tr $O/clk.json | tee $O/attr.txt
timeout -k 10 120 python3 tools/host_attr.py run $O/clk_plain.json | tee $O/plain.txt
find $O/tr -name "*hip_api_trace.csv" -size +20M -delete
