#!/bin/bash
# Staged-kernel same-box A/B: ab/libevam_pp_head.so (the default build) against ab/libevam_pp_$VAR.so.
# Full GPU parity suite under the variant, then plain bench lines (alternating, no profiler) for C5, C2,
# C4, then rocprofv3 kernel times (alternating) for C5 and C2. Usage: tools/gpu_ab_staged.sh TAG VAR
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
TAG="$1"; VAR="$2"
EVAM_PP_LIB=$ROOT/ab/libevam_pp_$VAR.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1 || { tail -30 gpurun_out/pt_$TAG.log; exit 1; }
tail -1 gpurun_out/pt_$TAG.log
for c in ${CONFIGS:-c5 c2 c4}; do
  for L in head $VAR head $VAR head $VAR; do
    EVAM_PP_LIB=$ROOT/ab/libevam_pp_$L.so timeout -k 10 120 python bench.py --config $c --steps 1000 --warmup 100 --no-cpu-baseline --resident-steps 0 > gpurun_out/${TAG}_${c}_$L.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_${c}_$L.json')); print('$c $L', d['value'], d['ms_per_step'], d['host_submit_ms_per_step'], d['roofline']['frac'])"
  done
done
H=EVAM_PP_LIB=$ROOT/ab/libevam_pp_head.so
V=EVAM_PP_LIB=$ROOT/ab/libevam_pp_$VAR.so
bash tools/sweep_env.sh $TAG c5 "$H|$V|$H|$V"
bash tools/sweep_env.sh $TAG c2 "$H|$V|$H|$V"
