set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05x.log 2>&1 || { tail -40 gpurun_out/pytest_r05x.log; exit 1; }
tail -2 gpurun_out/pytest_r05x.log
H="EVAM_PP_LIB=$GRAFT_REPO_ROOT/ab/libevam_pp_head.so"
bash tools/gpu_env_ab.sh r05x c3 "$H|EVAM_PP_REC_DEVICE=0|EVAM_PP_DEFAULT=1"
bash tools/gpu_env_ab.sh r05x c3 "EVAM_PP_REC_DEVICE=0|EVAM_PP_DEFAULT=1"
STEPS=200 bash tools/prof_configs.sh r05x c3
