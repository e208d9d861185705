# Round 3, second session: the profile set of the final bench (gpu_prof.sh: the bench under rocprofv3
# for C2 and C3 plus PMC passes) and a kernel trace of the driver's exact command.
set -o pipefail
R="$GRAFT_REPO_ROOT"
bash "$R/tools/gpu_prof.sh" || exit 1
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof/driver" -o run -- \
  python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$R/gpurun_out/prof/bench_driver.json" 2> "$R/gpurun_out/prof/bench_driver.err" \
  || { echo "rocprof driver command failed"; tail -5 "$R/gpurun_out/prof/bench_driver.err"; exit 1; }
tail -1 "$R/gpurun_out/prof/bench_driver.json"
