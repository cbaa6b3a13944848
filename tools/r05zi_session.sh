set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
A="EVAM_PP_LIB=$GRAFT_REPO_ROOT/ab/libevam_pp_args32.so"
bash tools/gpu_env_ab.sh r05zi c5 "EVAM_PP_DEFAULT=1|$A"
bash tools/gpu_env_ab.sh r05zi c5 "EVAM_PP_DEFAULT=1|$A"
bash tools/gpu_env_ab.sh r05zi c2 "EVAM_PP_DEFAULT=1|$A"
bash tools/gpu_env_ab.sh r05zi c1 "EVAM_PP_DEFAULT=1|$A"
