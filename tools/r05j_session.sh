set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c3 or roi" > gpurun_out/pytest_r05j.log 2>&1 || { tail -40 gpurun_out/pytest_r05j.log; exit 1; }
tail -1 gpurun_out/pytest_r05j.log
EVAM_PP_ROI_RMAX=9 timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c3" > gpurun_out/pytest_r05j_rmax.log 2>&1 || { tail -40 gpurun_out/pytest_r05j_rmax.log; exit 1; }
tail -1 gpurun_out/pytest_r05j_rmax.log
bash tools/gpu_env_ab.sh r05j c3 "EVAM_PP_DEFAULT=1|EVAM_PP_ROI_RMAX=14|EVAM_PP_ROI_RMAX=12|EVAM_PP_ROI_RMAX=10|EVAM_PP_ROI_RMAX=8|EVAM_PP_ROI_RMAX=6"
