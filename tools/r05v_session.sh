set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05v.log 2>&1 || { tail -40 gpurun_out/pytest_r05v.log; exit 1; }
tail -2 gpurun_out/pytest_r05v.log
B="EVAM_PP_LIB=$GRAFT_REPO_ROOT/ab/libevam_pp_base.so"
bash tools/gpu_env_ab.sh r05v c3 "$B|EVAM_PP_DEFAULT=1"
bash tools/gpu_env_ab.sh r05v c3 "$B|EVAM_PP_DEFAULT=1"
bash tools/gpu_env_ab.sh r05v c1 "$B|EVAM_PP_DEFAULT=1"
