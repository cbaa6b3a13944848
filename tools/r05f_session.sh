set -euo pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for c in c5 c1 c2 c3; do bash tools/gpu_env_ab.sh r05f $c "EVAM_PP_DEFAULT=1|HIP_FORCE_DEV_KERNARG=1|HIP_FORCE_DEV_KERNARG=0"; done
