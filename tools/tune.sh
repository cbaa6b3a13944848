#!/bin/bash
# Tile / occupancy / staging sweep of a bench workload. Variant = TWxTHxWGS_PER_CUxREG_STAGE.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${1:-tune}"; CFG="${2:-c2}"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { tail -40 "$OUT/pytest_gpu_$TAG.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu_$TAG.log"
fi
for v in ${VARIANTS:-128x4x0x0}; do
  IFS=x read TW TH WG <<< "$v"
  r=$(EVAM_PP_TW=$TW EVAM_PP_TH=$TH EVAM_PP_WGS_PER_CU=$WG timeout -k 10 120 python bench.py --config "$CFG" --steps 100 --warmup 20 --no-cpu-baseline)
  echo "$CFG $v $(echo "$r" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["roofline"]["achieved"], d["roofline"]["mean_launch_ms"])')" | tee -a "$OUT/tune_$TAG.txt"
done
