#!/bin/bash
# Bench one workload under a list of environment settings (diagnostics / tuning).
# Usage: tools/sweep_env.sh TAG CFG "ENV1=a,ENV2=b  ENV1=c ..."   (space-separated variants, comma-joined vars)
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="$1"; CFG="$2"; VARIANTS="$3"
for v in $VARIANTS; do
  envs=$(echo "$v" | tr ',' ' ')
  [ "$v" = "base" ] && envs=""
  r=$(env $envs timeout -k 10 120 python bench.py --config "$CFG" --steps ${STEPS:-200} --warmup 50 --no-cpu-baseline)
  echo "$CFG $v $(echo "$r" | python -c 'import json,sys; d=json.load(sys.stdin); print("f/s", d["value"], "GB/s", d["roofline"]["achieved"], "ms", d["roofline"]["mean_launch_ms"])')" | tee -a "$OUT/sweep_$TAG.txt"
done
