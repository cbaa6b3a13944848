set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export EVAM_PP_DIAGNOSTIC_BUILD_OK=1
STEPS=200 bash tools/prof_configs.sh r05k2_default c1
for v in bnomath; do EVAM_PP_LIB=$GRAFT_REPO_ROOT/ab/libevam_pp_$v.so STEPS=200 bash tools/prof_configs.sh r05k2_$v c1; done
