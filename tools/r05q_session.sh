set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r05q.log 2>&1 || { tail -40 gpurun_out/pytest_r05q.log; exit 1; }
tail -1 gpurun_out/pytest_r05q.log
bash tools/gpu_env_ab.sh r05q c3 "EVAM_PP_DEFAULT=1|EVAM_PP_LIB=$GRAFT_REPO_ROOT/ab/libevam_pp_k8.so|EVAM_PP_LIB=$GRAFT_REPO_ROOT/ab/libevam_pp_k4.so|EVAM_PP_ROI_PX=1"
