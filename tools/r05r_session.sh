set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_env_ab.sh r05r c3 "EVAM_PP_DEFAULT=1|EVAM_PP_ROI_BUF=6144|EVAM_PP_ROI_BUF=12288|EVAM_PP_ROI_TAIL=1|EVAM_PP_ROI_TAIL=8|EVAM_PP_PRIO=0"
