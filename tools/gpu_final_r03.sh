#!/bin/bash
# Round-3 final measurement on one box: the GPU suite, smoke(), the driver's own bench command (C2 with the CPU
# baseline), a 1000-step bench line per config, rocprofv3 kernel stats per config, and the PMC HBM-traffic
# passes (FETCH_SIZE / WRITE_SIZE, one counter group per run) of C2-C5. Every GPU step has its own time limit
# and the first failure ends the script.
#   tools/gpu_final_r03.sh TAG
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
cd "$ROOT"
TAG="${1:-r03final}"
echo "[final] pytest -m gpu"; date
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { tail -40 "$OUT/pytest_gpu_$TAG.log"; exit 1; }
tail -1 "$OUT/pytest_gpu_$TAG.log"
echo "[final] smoke"; date
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.txt" 2>&1 || { tail -20 "$OUT/smoke_$TAG.txt"; exit 1; }
tail -1 "$OUT/smoke_$TAG.txt"
echo "[final] driver command"; date
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_${TAG}_driver.json" 2> "$OUT/bench_${TAG}_driver.err" \
  || { tail -20 "$OUT/bench_${TAG}_driver.err"; exit 1; }
tail -1 "$OUT/bench_${TAG}_driver.json"
for c in c1 c2 c3 c4 c5; do
  echo "[final] bench $c"; date
  timeout -k 10 240 python3 bench.py --config $c --steps 1000 --warmup 100 --no-cpu-baseline > "$OUT/bench_${TAG}_$c.json" \
    2> "$OUT/bench_${TAG}_$c.err" || { tail -20 "$OUT/bench_${TAG}_$c.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/bench_${TAG}_$c.json').read().splitlines()[-1]);r=d['roofline'];print('$c',d['value'],d['ms_per_step'],r['bound'],r['frac'],r.get('hbm',{}).get('frac'),r['launch_ms_p10_p50_p90'])" | tee -a "$OUT/bench_$TAG.txt"
done
STEPS=200 bash tools/prof_configs.sh "$TAG" "c1 c2 c3 c4 c5"
for c in c2 c3 c4 c5; do
  PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" bash tools/pmc.sh "${TAG}_$c" "$c"
  cp "$OUT/pmc_traffic.json" "$OUT/pmc_traffic_${TAG}_$c.json"
done
echo "[final] done"; date
