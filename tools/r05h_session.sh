set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "roi or c3" > gpurun_out/pytest_r05h.log 2>&1 || { tail -40 gpurun_out/pytest_r05h.log; exit 1; }
tail -2 gpurun_out/pytest_r05h.log
EVAM_PP_ROI_XCD=1 EVAM_PP_ROI_PERSIST=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c3" > gpurun_out/pytest_r05h_xcd.log 2>&1 || { tail -40 gpurun_out/pytest_r05h_xcd.log; exit 1; }
tail -2 gpurun_out/pytest_r05h_xcd.log
bash tools/gpu_env_ab.sh r05h c3 "EVAM_PP_DEFAULT=1|EVAM_PP_ROI_XCD=1|EVAM_PP_ROI_PERSIST=1"
