set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05zg.log 2>&1 || { tail -40 gpurun_out/pytest_r05zg.log; exit 1; }
tail -1 gpurun_out/pytest_r05zg.log
bash tools/gpu_env_ab.sh r05zg c3 "EVAM_PP_DEFAULT=1|EVAM_PP_ROI_SORT=0 EVAM_PP_ROI_SNAKE=0"
bash tools/gpu_env_ab.sh r05zg c3 "EVAM_PP_DEFAULT=1|EVAM_PP_ROI_SORT=0 EVAM_PP_ROI_SNAKE=0"
