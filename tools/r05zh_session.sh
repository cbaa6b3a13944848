set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
EVAM_PP_ROI_SNAKE=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c3" > gpurun_out/pytest_r05zh.log 2>&1 || { tail -40 gpurun_out/pytest_r05zh.log; exit 1; }
tail -1 gpurun_out/pytest_r05zh.log
bash tools/gpu_env_ab.sh r05zh c3 "EVAM_PP_DEFAULT=1|EVAM_PP_ROI_SNAKE=2"
bash tools/gpu_env_ab.sh r05zh c3 "EVAM_PP_DEFAULT=1|EVAM_PP_ROI_SNAKE=2"
