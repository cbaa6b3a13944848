set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/prof_ablate.sh r05zc c5 "0 2 4 16 64 128"
bash tools/prof_ablate.sh r05zc c2 "0 2 4 16 64 128"
