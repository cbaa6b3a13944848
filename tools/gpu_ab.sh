#!/bin/bash
# Same-box A/B of the current build against ab/libevam_pp_head.so (alternating, rocprofv3 kernel averages)
# on the given configs, after the GPU parity suite. Usage: tools/gpu_ab.sh TAG "c2 c4 c5" [pytest -k expr]
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
TAG="$1"; CFGS="$2"; K="${3:-}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pt_$TAG.log 2>&1 || { tail -30 gpurun_out/pt_$TAG.log; exit 1; }
tail -2 gpurun_out/pt_$TAG.log
H=EVAM_PP_LIB=$ROOT/ab/libevam_pp_head.so
for c in $CFGS; do
  bash tools/sweep_env.sh $TAG $c "$H|EVAM_PP_ABLATE=0|$H|EVAM_PP_ABLATE=0|$H|EVAM_PP_ABLATE=0"
done
