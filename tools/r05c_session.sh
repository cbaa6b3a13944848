set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05c.log 2>&1 || { tail -30 gpurun_out/pytest_r05c.log; exit 1; }
tail -2 gpurun_out/pytest_r05c.log
for c in c1 c1_i420 c2 c3 c5; do bash tools/gpu_env_ab.sh r05c $c "EVAM_PP_DEFAULT=1|EVAM_PP_LIB=ab/libevam_pp_prev.so"; done
