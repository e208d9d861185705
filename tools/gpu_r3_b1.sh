# Round 3: the streaming kernel (variant 6) against the round-2 default (variant 0), same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3b1; mkdir -p $O
B="python bench.py --cpu-seconds 0"
run() { local name=$1; shift; timeout -k 10 120 "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; exit 1; }; python -c "import json,sys; d=json.load(open('$O/$name.json')); r=d['roofline']; print('$name', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'])"; }
run k6_c2 $B --kernel 6 --steps 2000 --warmup 500
run k0_c2 $B --kernel 0 --steps 2000 --warmup 500
FS_RX_GRID=2 run k6g2_c2 $B --kernel 6 --steps 2000 --warmup 500
run k6_c2_20 $B --kernel 6 --steps 20 --warmup 5
run k0_c2_20 $B --kernel 0 --steps 20 --warmup 5
run k6_c3 $B --kernel 6 --config c3 --steps 1000 --warmup 500
run k0_c3 $B --kernel 0 --config c3 --steps 1000 --warmup 500
run k6_c2_s1 $B --kernel 6 --steps 2000 --warmup 500 --streams 1
run k6_c2_s2 $B --kernel 6 --steps 2000 --warmup 500 --streams 2
