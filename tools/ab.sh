#!/bin/bash
# A/B library builds (tools/variants/*.so) on one bench config, interleaved rounds in one session.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${1:-ab}"; CFG="${2:-c2}"; ROUNDS="${ROUNDS:-2}"
for r in $(seq 1 $ROUNDS); do
  for lib in ${LIBS:-tools/variants/*.so}; do
    res=$(EVAM_PP_LIB="$ROOT/$lib" timeout -k 10 120 python bench.py --config "$CFG" --steps 200 --warmup 20 --no-cpu-baseline)
    echo "$CFG $(basename $lib) round$r $(echo "$res" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["roofline"]["achieved"], d["roofline"]["mean_launch_ms"])')" | tee -a "$OUT/ab_$TAG.txt"
  done
done
