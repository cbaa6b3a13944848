#!/bin/bash
# A/B library variants x tile heights (EVAM_PP_TH) on one bench config.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${1:-abth}"; CFG="${2:-c2}"
for th in ${THS:-8 16 32}; do
  for lib in ${LIBS:-tools/variants/*.so}; do
    res=$(EVAM_PP_TH=$th EVAM_PP_LIB="$ROOT/$lib" timeout -k 10 120 python bench.py --config "$CFG" --steps 400 --warmup 100 --no-cpu-baseline)
    echo "$CFG th=$th $(basename $lib) $(echo "$res" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["roofline"]["achieved"], d["roofline"]["mean_launch_ms"])')" | tee -a "$OUT/abth_$TAG.txt"
  done
done
