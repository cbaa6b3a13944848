set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export EVAM_PP_DIAGNOSTIC_BUILD_OK=1
bash tools/gpu_env_ab.sh r05d c3 "EVAM_PP_DEFAULT=1|EVAM_PP_LIB=ab/libevam_pp_launch.so|EVAM_PP_LIB=ab/libevam_pp_geo.so|EVAM_PP_LIB=ab/libevam_pp_setup.so|EVAM_PP_LIB=ab/libevam_pp_nostore.so|EVAM_PP_LIB=ab/libevam_pp_nodma.so"
