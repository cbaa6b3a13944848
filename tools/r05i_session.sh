set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05i.log 2>&1 || { tail -40 gpurun_out/pytest_r05i.log; exit 1; }
tail -2 gpurun_out/pytest_r05i.log
for c in c2 c5 c4 c2_i420; do bash tools/gpu_env_ab.sh r05i $c "EVAM_PP_DEFAULT=1|EVAM_PP_LIB=$GRAFT_REPO_ROOT/ab/libevam_pp_d3.so"; done
