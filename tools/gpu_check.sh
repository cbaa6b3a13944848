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
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { tail -40 "$OUT/pytest_gpu_$TAG.log"; exit 1; }
tail -3 "$OUT/pytest_gpu_$TAG.log"
echo "[gpu_check] bench"; date
timeout -k 10 300 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || { tail -20 "$OUT/bench_$TAG.err"; exit 1; }
cat "$OUT/bench_$TAG.json"
if [ "${DIST:-0}" = "1" ]; then
  echo "[gpu_check] bench, 2 ranks on one GPU over gloo (multi-process rehearsal)"; date
  EVAM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 100 --warmup 20 \
    > "$OUT/bench_dist2_$TAG.json" 2> "$OUT/bench_dist2_$TAG.err" || { tail -20 "$OUT/bench_dist2_$TAG.err"; exit 1; }
  cat "$OUT/bench_dist2_$TAG.json"
  EVAM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --config c4 --steps 50 --warmup 10 \
    > "$OUT/bench_dist2_c4_$TAG.json" 2> "$OUT/bench_dist2_c4_$TAG.err" || { tail -20 "$OUT/bench_dist2_c4_$TAG.err"; exit 1; }
  cat "$OUT/bench_dist2_c4_$TAG.json"
fi
if [ "${EXTRA:-0}" = "1" ]; then
  for c in c1 c3 c4 c5; do
    echo "[gpu_check] bench $c"; date
    timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 50 --no-cpu-baseline > "$OUT/bench_${c}_$TAG.json" 2> "$OUT/bench_${c}_$TAG.err" || { tail -20 "$OUT/bench_${c}_$TAG.err"; exit 1; }
    cat "$OUT/bench_${c}_$TAG.json"
  done
  echo "[gpu_check] bench host feed"; date
  timeout -k 10 300 python bench.py --feed host --steps 100 --warmup 20 --no-cpu-baseline > "$OUT/bench_host_$TAG.json" 2> "$OUT/bench_host_$TAG.err" || { tail -20 "$OUT/bench_host_$TAG.err"; exit 1; }
  cat "$OUT/bench_host_$TAG.json"
fi
echo "[gpu_check] rocprofv3 kernel trace"; date
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o bench -- \
  python3 "$ROOT/bench.py" --steps 200 --warmup 50 --no-cpu-baseline --resident-steps 0 > "$OUT/prof_bench_$TAG.json" 2> "$OUT/prof_$TAG.err" || { tail -20 "$OUT/prof_$TAG.err"; exit 1; }
find "$OUT/prof_$TAG" -name "*stats*" | head
echo "[gpu_check] done"; date
