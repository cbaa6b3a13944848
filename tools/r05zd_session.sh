set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
EVAM_PP_ROI_XCD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c3" > gpurun_out/pytest_r05zd.log 2>&1 || { tail -40 gpurun_out/pytest_r05zd.log; exit 1; }
tail -1 gpurun_out/pytest_r05zd.log
bash tools/gpu_env_ab.sh r05zd c3 "EVAM_PP_DEFAULT=1|EVAM_PP_ROI_XCD=1"
bash tools/gpu_env_ab.sh r05zd c3 "EVAM_PP_DEFAULT=1|EVAM_PP_ROI_XCD=1"
EVAM_PP_ROI_XCD=1 PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" bash tools/pmc.sh r05zd_xcd c3
