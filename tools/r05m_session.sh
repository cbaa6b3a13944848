set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for c in c5 c2 c5_bgrx; do bash tools/gpu_env_ab.sh r05m $c "EVAM_PP_DEFAULT=1|EVAM_PP_STRIP_WAVES=8|EVAM_PP_STRIP_WAVES=12|EVAM_PP_STRIP_WAVES=24"; done
