#!/bin/bash
# Round-end measurement set: GPU parity suite, smoke, default bench line (C2 + CPU baseline), the other
# configs' bench lines, rocprofv3 kernel stats of every config, and the pipeline-layer leg.
# Usage: tools/gpu_final.sh TAG  -> gpurun_out/final_TAG/...
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="${1:-final}"; OUT="$ROOT/gpurun_out/final_$TAG"; mkdir -p "$OUT"
echo "[final] pytest"; date
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
echo "[final] smoke"; date
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
echo "[final] bench c2 (default)"; date
timeout -k 10 300 python bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { tail -20 "$OUT/bench_c2.err"; exit 1; }
cat "$OUT/bench_c2.json"
for c in c1 c3 c4 c5; do
  echo "[final] bench $c"; date
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { tail -20 "$OUT/bench_$c.err"; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['value'], d['roofline']['frac'], d['roofline']['mean_launch_ms'])"
done
echo "[final] pipeline leg"; date
timeout -k 10 300 python bench.py --via pipeline --frames-per-stream 4096 > "$OUT/bench_via_pipeline.json" 2> "$OUT/bench_via_pipeline.err" || { tail -20 "$OUT/bench_via_pipeline.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_via_pipeline.json')); print('pipeline', d['value'])"
echo "[final] rocprof"; date
bash tools/prof_configs.sh "f$TAG" "c1 c2 c3 c4 c5" > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
cat "$ROOT/gpurun_out/prof_f$TAG.txt"
echo "[final] done"; date
