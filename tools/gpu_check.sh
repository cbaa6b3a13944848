#!/bin/bash
# One GPU session: parity tests, the default bench line, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; the first failure ends the script (set -e).
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
TAG="${1:-r01}"
echo "[gpu_check] pytest -m gpu"; date
timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { tail -40 "$OUT/pytest_gpu_$TAG.log"; exit 1; }
tail -3 "$OUT/pytest_gpu_$TAG.log"
echo "[gpu_check] bench"; date
timeout -k 10 300 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || { tail -20 "$OUT/bench_$TAG.err"; exit 1; }
cat "$OUT/bench_$TAG.json"
echo "[gpu_check] rocprofv3 kernel trace"; date
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o bench -- \
  python3 "$ROOT/bench.py" --steps 200 --warmup 50 --no-cpu-baseline > "$OUT/prof_bench_$TAG.json" 2> "$OUT/prof_$TAG.err" || { tail -20 "$OUT/prof_$TAG.err"; exit 1; }
find "$OUT/prof_$TAG" -name "*stats*" | head
echo "[gpu_check] done"; date
