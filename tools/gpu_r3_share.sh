# Mixed-kernel pass sharing: same-box A/B against HEAD's library (C2 2,000 / 20 steps, C3).
set -o pipefail
cd $GRAFT_REPO_ROOT
REPS=2 bash tools/gpu_abl.sh prod head
