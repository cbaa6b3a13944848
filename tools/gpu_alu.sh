#!/bin/bash
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
V=$ROOT/ab/libevam_pp_alunorm.so
EVAM_PP_LIB=$V timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "roi or fullsize" > gpurun_out/pt_alu.log 2>&1 || { tail -30 gpurun_out/pt_alu.log; exit 1; }
tail -2 gpurun_out/pt_alu.log
bash tools/sweep_env.sh alu c3 "EVAM_PP_ABLATE=0|EVAM_PP_LIB=$V|EVAM_PP_ABLATE=0|EVAM_PP_LIB=$V|EVAM_PP_ABLATE=0|EVAM_PP_LIB=$V"
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/pl_direct.json 2>gpurun_out/pl_direct.err
python -c "import json; d=json.load(open('gpurun_out/pl_direct.json')); print('direct', d['value'])"
for i in 1 2; do timeout -k 10 300 python bench.py --via pipeline > gpurun_out/pl_dev_$i.json 2>gpurun_out/pl_dev_$i.err; python -c "import json; d=json.load(open('gpurun_out/pl_dev_$i.json')); print('pipeline', d['value'], d['config']['elapsed_s'])"; done
S=$ROOT/ab/libevam_pp_s80d.so
bash tools/sweep_env.sh s80r c2 "EVAM_PP_ABLATE=0|EVAM_PP_LIB=$S|EVAM_PP_LIB=$S EVAM_PP_STAGE_R=1|EVAM_PP_STAGE_R=1|EVAM_PP_ABLATE=0|EVAM_PP_LIB=$S|EVAM_PP_LIB=$S EVAM_PP_STAGE_R=1"
