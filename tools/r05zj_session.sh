set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "band or c1 or wave_kernel" > gpurun_out/pytest_r05zj.log 2>&1 || { tail -40 gpurun_out/pytest_r05zj.log; exit 1; }
tail -2 gpurun_out/pytest_r05zj.log
H="EVAM_PP_LIB=$GRAFT_REPO_ROOT/ab/libevam_pp_head.so"
bash tools/gpu_env_ab.sh r05zj c1 "$H|EVAM_PP_DEFAULT=1"
bash tools/gpu_env_ab.sh r05zj c1 "$H|EVAM_PP_DEFAULT=1"
bash tools/gpu_env_ab.sh r05zj c1_i420 "$H|EVAM_PP_DEFAULT=1"
