#!/bin/bash
# Round-3 GPU session: the GPU parity suite, then bench lines of the default build on C2 / C4 / C5 and of
# each A/B setting given (env assignments, e.g. EVAM_PP_STRIP=0 or EVAM_PP_LIB=ab/libevam_pp_X.so),
# then a rocprofv3 kernel-trace summary of C2.
# Every GPU step has its own time limit; the first failure ends the script.
#   tools/gpu_r03.sh TAG [tests|notests] ["env settings of an A/B arm", ...]
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
TAG="${1:-r03}"
TESTS="${2:-tests}"
shift 2 || true
if [ "$TESTS" = "tests" ]; then
  echo "[r03] pytest -m gpu"; date
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { tail -60 "$OUT/pytest_gpu_$TAG.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu_$TAG.log"
fi
line() {  # line NAME ENV... -- ARGS...
  local name="$1"; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  echo "[r03] $name"; date
  env "${envs[@]}" timeout -k 10 240 python bench.py "$@" --no-cpu-baseline > "$OUT/bench_${TAG}_$name.json" \
    2> "$OUT/bench_${TAG}_$name.err" || { tail -20 "$OUT/bench_${TAG}_$name.err"; exit 1; }
  python3 - "$OUT/bench_${TAG}_$name.json" "$name" <<'EOF' | tee -a "$OUT/bench_$TAG.txt"
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = b["roofline"]
print(f"{sys.argv[2]:>18}: {b['value']:>12.1f} f/s  step {b['ms_per_step']*1e3:7.2f} us  launch {r['mean_launch_ms']*1e3:7.2f} us"
      f"  p10/50/90 {[round(x*1e3,2) for x in r['launch_ms_p10_p50_p90']]}  frac {r['frac'] if r['bound']=='hbm' else r['hbm']['frac']}")
EOF
}
line c2_strip -- --steps 300 --warmup 50
line c4_strip -- --config c4 --steps 150 --warmup 30
line c5_strip -- --config c5 --steps 300 --warmup 50
line c1 -- --config c1 --steps 300 --warmup 50
line c3 -- --config c3 --steps 300 --warmup 50
for e in "$@"; do
  tag="$(echo "$e" | sed 's/[ =\/]/_/g')"
  line "c2_$tag" $e -- --steps 300 --warmup 50
  line "c4_$tag" $e -- --config c4 --steps 150 --warmup 30
  line "c5_$tag" $e -- --config c5 --steps 300 --warmup 50
  line "c1_$tag" $e -- --config c1 --steps 300 --warmup 50
  line "c3_$tag" $e -- --config c3 --steps 300 --warmup 50
done
echo "[r03] rocprofv3 C2"; date
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_c2" -o run -- \
  python3 "$ROOT/bench.py" --steps 200 --warmup 50 --no-cpu-baseline --resident-steps 0 \
  > "$OUT/prof_${TAG}_c2.json" 2> "$OUT/prof_${TAG}_c2.err" || { tail -20 "$OUT/prof_${TAG}_c2.err"; exit 1; }
find "$OUT/prof_${TAG}_c2" -name "*stats*"
echo "[r03] done"; date
