set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export EVAM_PP_DIAGNOSTIC_BUILD_OK=1
STEPS=200 bash tools/prof_configs.sh r05e_default c3
for v in launch geo setup nostore nodma; do EVAM_PP_LIB=$GRAFT_REPO_ROOT/ab/libevam_pp_$v.so STEPS=200 bash tools/prof_configs.sh r05e_$v c3; done
cat gpurun_out/prof_r05e_*.txt
