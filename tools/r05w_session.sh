set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
EVAM_PP_LIB=$GRAFT_REPO_ROOT/ab/libevam_pp_head.so bash tools/prof_ablate.sh r05w c3 "0"
bash tools/prof_ablate.sh r05w c3 "2 4 16 6 18"
