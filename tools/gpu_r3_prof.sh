# Round-3 profile set: gpu_prof.sh (bench under rocprofv3 + PMC passes, C2 and C3), C3 stamps of
# the mixed-length kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_prof.sh || exit 1
FRAMESUM_LIB=$PWD/seqs_amd/lib/diag/libframesum_stamps.so timeout -k 10 120 python tools/stamps.py --config c3 --kernel 2 > gpurun_out/stamps_c3.log 2>&1 || { tail -5 gpurun_out/stamps_c3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_c3.log | head -30
