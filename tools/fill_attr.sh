# where the TX fill's extra time goes (C2, 65,536 x 1500 B + 4 spare bytes).
#   write traffic: rocprofv3 --pmc WRITE_SIZE + TCC_EA0_WRREQ_sum + TCC_EA0_WRREQ_64B_sum, fill and digest
#   per-wave timeline: tools/stamps.py --op fill / digest with the FS_STAMPS build (diag/libframesum_stg.so)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fill_attr; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for op in digest fill; do
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv \
    -d $O/pmc_$op -o run -- python3 $R/tools/prof_driver.py --config c2 --op $op --iters 20 --kernel 4 > $O/pmc_$op.log 2>&1 \
    || { echo "PMC $op failed"; tail -5 $O/pmc_$op.log; exit 1; }
done
cd $R
python3 - <<'PY'
import csv, glob, os, collections
R = os.environ["GRAFT_REPO_ROOT"]
for op in ("digest", "fill"):
    f = glob.glob(f"{R}/gpurun_out/fill_attr/pmc_{op}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(f)):
        if "digest_kernel" in row.get("Kernel_Name", ""):
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    print(op, {k: round(sum(v) / max(1, len(v)) / 1, 1) for k, v in sorted(acc.items())}, "(per launch; WRITE_SIZE in KB)")
PY
for op in digest fill; do
  echo "== stamps $op"
  FRAMESUM_LIB=$R/seqs_amd/lib/diag/libframesum_stg.so timeout -k 10 200 python tools/stamps.py --config c2 --kernel 4 --op $op 2>&1 | grep -v amdgpu.ids | head -12
done
