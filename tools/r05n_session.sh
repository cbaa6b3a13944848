set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_dist_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r05n.log 2>&1 || { tail -40 gpurun_out/pytest_r05n.log; exit 1; }
tail -1 gpurun_out/pytest_r05n.log
for c in c1 c1_i420; do bash tools/gpu_env_ab.sh r05n $c "EVAM_PP_DEFAULT=1|EVAM_PP_BAND_BPW=1|EVAM_PP_BAND_BPW=1 EVAM_PP_STRIP_WAVES=12"; done
