#!/bin/bash
# ROI-kernel latency probe: kernel time vs ROI count (frames x 50) and, at a few frames, the EVAM_PP_ABLATE
# variants (2 no pixel math, 4 no stores, 16 no DMA). Prints one line per run into gpurun_out/roi_lat_TAG.txt.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${1:-lat}"; FRAMES="${2:-1 2 4 8}"; ABL="${3:-0 2 4 16 22}"
for fr in $FRAMES; do
  for a in $ABL; do
    r=$(EVAM_PP_ABLATE=$a timeout -k 10 120 python bench.py --config c3 --frames "$fr" --steps ${STEPS:-300} --warmup 50 --no-cpu-baseline)
    echo "frames $fr ablate $a $(echo "$r" | python -c 'import json,sys; d=json.load(sys.stdin); print("us", round(d["roofline"]["mean_launch_ms"]*1e3, 2), "GB/s", d["roofline"]["achieved"])')" | tee -a "$OUT/roi_lat_$TAG.txt"
  done
done
