set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "strip or c2 or c4 or c5 or i420 or wave_kernel_variants or full_frame" > gpurun_out/pytest_r05b.log 2>&1 || { tail -30 gpurun_out/pytest_r05b.log; exit 1; }
tail -2 gpurun_out/pytest_r05b.log
for c in c2 c2_i420 c5 c5_bgrx c4; do bash tools/gpu_env_ab.sh r05b $c "EVAM_PP_STRIP_PAIR=1|EVAM_PP_STRIP_PAIR=0"; done
