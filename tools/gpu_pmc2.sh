#!/bin/bash
# PMC passes (kernel-trace only, separate runs) for a library variant: tools/gpu_pmc2.sh <variant> [config]
set -o pipefail
R="$GRAFT_REPO_ROOT"
V="$1"; CFG="${2:-c2}"
mkdir -p "$R/gpurun_out/pmc2"
export TMPDIR=/tmp
cd /tmp
i=0
while read -r line; do
  i=$((i+1))
  FRAMESUM_LIB="$R/seqs_amd/lib/diag/libframesum_$V.so" timeout -k 10 180 rocprofv3 --pmc $line --output-format csv -d "$R/gpurun_out/pmc2/${V}_${CFG}_$i" -o run -- python3 "$R/tools/prof_driver.py" --config $CFG --iters 20 > "$R/gpurun_out/pmc2/${V}_${CFG}_$i.log" 2>&1 || { echo "PMC pass $i ($line) failed"; tail -5 "$R/gpurun_out/pmc2/${V}_${CFG}_$i.log"; exit 1; }
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT
SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT
LIST
cd "$R" && python3 - "$V" "$CFG" <<'PY'
import sys, glob, csv, statistics
v, cfg = sys.argv[1], sys.argv[2]
per = {}
for path in glob.glob(f"gpurun_out/pmc2/{v}_{cfg}_*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(path)):
        if "digest_kernel" not in row["Kernel_Name"]:
            continue
        per.setdefault(row["Counter_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
        per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
med = {k: statistics.median(d.values()) for k, d in per.items()}
for k in sorted(med):
    print(f"{k:24s} {med[k]:16.1f}")
w = med.get("SQ_WAVES", 1)
print("per wave: valu %.0f lds %.0f salu %.0f vmem %.0f" % (med.get("SQ_INSTS_VALU",0)/w, med.get("SQ_INSTS_LDS",0)/w, med.get("SQ_INSTS_SALU",0)/w, med.get("SQ_INSTS_VMEM_RD",0)/w))
PY
