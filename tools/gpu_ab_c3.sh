#!/bin/bash
# C3 same-box A/B of the current build against ab/libevam_pp_head.so (alternating), ROI parity first,
# then write-request PMC of both. Usage: tools/gpu_ab_c3.sh TAG
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
TAG="${1:-ab}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "roi or fullsize" > gpurun_out/pt_$TAG.log 2>&1 || { tail -30 gpurun_out/pt_$TAG.log; exit 1; }
tail -2 gpurun_out/pt_$TAG.log
H=EVAM_PP_LIB=$ROOT/ab/libevam_pp_head.so
bash tools/sweep_env.sh $TAG c3 "$H|EVAM_PP_ABLATE=0|$H|EVAM_PP_ABLATE=0|$H|EVAM_PP_ABLATE=0"
PMC_GROUPS="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" bash tools/pmc.sh ${TAG}_new c3 | tail -5
PMC_GROUPS="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" EVAM_PP_LIB=$ROOT/ab/libevam_pp_head.so bash tools/pmc.sh ${TAG}_head c3 | tail -5
