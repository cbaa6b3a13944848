#!/bin/bash
# C3 same-box A/B of the current build against ab/libevam_pp_head.so: ROI parity, then plain bench lines
# (alternating, no profiler) and rocprofv3 kernel times (alternating). Usage: tools/gpu_ab_c3b.sh TAG
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
TAG="${1:-ab}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "roi or churn or fullsize" > gpurun_out/pt_$TAG.log 2>&1 || { tail -30 gpurun_out/pt_$TAG.log; exit 1; }
tail -1 gpurun_out/pt_$TAG.log
for L in head new head new head new; do
  if [ $L = head ]; then export EVAM_PP_LIB=$ROOT/ab/libevam_pp_head.so; else unset EVAM_PP_LIB; fi
  timeout -k 10 120 python bench.py --config c3 --steps 1000 --warmup 100 --no-cpu-baseline --resident-steps 0 > gpurun_out/${TAG}_$L.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_$L.json')); print('$L', d['value'], d['ms_per_step'], d['host_submit_ms_per_step'], d['roofline']['frac'])"
done
unset EVAM_PP_LIB
H=EVAM_PP_LIB=$ROOT/ab/libevam_pp_head.so
bash tools/sweep_env.sh $TAG c3 "$H|EVAM_PP_ABLATE=0|$H|EVAM_PP_ABLATE=0"
