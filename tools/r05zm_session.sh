set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_env_ab.sh r05zm c5 "EVAM_PP_DEFAULT=1|EVAM_PP_STRIP_PX=2|EVAM_PP_STRIP_NW=2|EVAM_PP_STRIP_NW=8|EVAM_PP_STRIP_TH=4|EVAM_PP_STRIP_TH=14"
