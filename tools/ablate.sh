#!/bin/bash
# Ablation sweep (diagnostic): EVAM_PP_ABLATE bits 1=no DMA, 2=no pixel math, 4=no stores.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${1:-abl}"
for v in ${VARIANTS:-128x8x0}; do
  IFS=x read TW TH WG <<< "$v"
  for a in ${ABL:-0 2 4 8 12 16 20}; do
    r=$(EVAM_PP_ABLATE=$a EVAM_PP_TW=$TW EVAM_PP_TH=$TH EVAM_PP_WGS_PER_CU=$WG timeout -k 10 120 python bench.py --steps 100 --warmup 20 --no-cpu-baseline)
    echo "$v ablate=$a $(echo "$r" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["roofline"]["mean_launch_ms"])')" | tee -a "$OUT/ablate_$TAG.txt"
  done
done
