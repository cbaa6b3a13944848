set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "roi or c3" > gpurun_out/pytest_r05o.log 2>&1 || { tail -40 gpurun_out/pytest_r05o.log; exit 1; }
tail -1 gpurun_out/pytest_r05o.log
EVAM_PP_ROI_PX=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c3" > gpurun_out/pytest_r05o2.log 2>&1 || { tail -40 gpurun_out/pytest_r05o2.log; exit 1; }
tail -1 gpurun_out/pytest_r05o2.log
bash tools/gpu_env_ab.sh r05o c3 "EVAM_PP_DEFAULT=1|EVAM_PP_ROI_PX=2|EVAM_PP_ROI_PX=2 EVAM_PP_ROI_RMAX=0"
bash tools/gpu_env_ab.sh r05o c4 "EVAM_PP_DEFAULT=1|EVAM_PP_STRIP_PX=1"
