set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05g.log 2>&1 || { tail -40 gpurun_out/pytest_r05g.log; exit 1; }
tail -2 gpurun_out/pytest_r05g.log
bash tools/gpu_env_ab.sh r05g c3 "EVAM_PP_DEFAULT=1|EVAM_PP_ROI_PERSIST=0|EVAM_PP_ROI_WGS=3|EVAM_PP_ROI_WGS=5|EVAM_PP_ROI_WGS=6|EVAM_PP_ROI_FRAMES_XCD=0"
STEPS=200 bash tools/prof_configs.sh r05g c3
