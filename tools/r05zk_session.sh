set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
EVAM_PP_ROI_KEY=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c3" > gpurun_out/pytest_r05zk.log 2>&1 || { tail -40 gpurun_out/pytest_r05zk.log; exit 1; }
tail -1 gpurun_out/pytest_r05zk.log
bash tools/gpu_env_ab.sh r05zk c3 "EVAM_PP_DEFAULT=1|EVAM_PP_ROI_KEY=1|EVAM_PP_ROI_TAIL=8"
bash tools/gpu_env_ab.sh r05zk c3 "EVAM_PP_DEFAULT=1|EVAM_PP_ROI_KEY=1|EVAM_PP_ROI_TAIL=8"
