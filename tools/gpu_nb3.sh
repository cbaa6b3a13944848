#!/bin/bash
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "roi or fullsize" > gpurun_out/pt_nb3.log 2>&1 || { tail -30 gpurun_out/pt_nb3.log; exit 1; }
tail -2 gpurun_out/pt_nb3.log
bash tools/sweep_env.sh nb3 c3 "EVAM_PP_ROI_NBUF=2|EVAM_PP_ROI_NBUF=3|EVAM_PP_ROI_NBUF=2|EVAM_PP_ROI_NBUF=3|EVAM_PP_ROI_NBUF=3 EVAM_PP_ROI_BUF=6144"
bash tools/gpu_occ.sh
