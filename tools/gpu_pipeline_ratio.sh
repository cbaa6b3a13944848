#!/bin/bash
# Pipeline-layer overhead at equal launch size: the direct C2 line with 256 frames per step (the hub's launch
# size) next to bench.py --via pipeline --hub-batch 256 on the same box.
#   tools/gpu_pipeline_ratio.sh TAG
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
TAG="${1:-r03}"
for n in 32 256; do
  echo "[ratio] direct C2 --frames $n"; date
  timeout -k 10 240 python bench.py --frames $n --steps 200 --warmup 40 --no-cpu-baseline \
    > "$OUT/ratio_${TAG}_direct_$n.json" 2> "$OUT/ratio_${TAG}_direct_$n.err" || { tail -20 "$OUT/ratio_${TAG}_direct_$n.err"; exit 1; }
  tail -1 "$OUT/ratio_${TAG}_direct_$n.json"
done
echo "[ratio] via pipeline, hub batch 256"; date
timeout -k 10 300 python bench.py --via pipeline --hub-batch 256 --no-cpu-baseline \
  > "$OUT/ratio_${TAG}_pipeline.json" 2> "$OUT/ratio_${TAG}_pipeline.err" || { tail -20 "$OUT/ratio_${TAG}_pipeline.err"; exit 1; }
tail -1 "$OUT/ratio_${TAG}_pipeline.json"
echo "[ratio] done"; date
