#!/bin/bash
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
A=EVAM_PP_LIB=$ROOT/ab/libevam_pp_s80.so; B=EVAM_PP_LIB=$ROOT/ab/libevam_pp_s80d.so
bash tools/sweep_env.sh s80 c2 "EVAM_PP_ABLATE=0|$A|$B|EVAM_PP_ABLATE=0|$A|$B|$B EVAM_PP_TH=8|$B EVAM_PP_TH=12"
bash tools/sweep_env.sh s80 c4 "EVAM_PP_ABLATE=0|$A|$B|EVAM_PP_ABLATE=0|$A|$B"
bash tools/sweep_env.sh s80 c5 "EVAM_PP_ABLATE=0|$A|$B|EVAM_PP_ABLATE=0|$A|$B"
