#!/bin/bash
# Copy the judged outputs of one tools/gpu.sh session (gpurun_out/ is scratch) into profiles/ under the tag:
# stamp, driver / bench lines, rocprof kernel-stats CSVs and their summaries, PMC summaries, A/B tables.
#   tools/keep_profiles.sh TAG
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"; G="$ROOT/gpurun_out"; P="$ROOT/profiles"; T="$1"
cp_if() { [ -e "$1" ] && cp "$1" "$2" || true; }
cp_if "$G/stamp_$T.json" "$P/${T}_stamp.json"
for f in "$G"/bench_${T}_*.json; do [ -e "$f" ] && cp "$f" "$P/$(basename "$f" | sed "s/^bench_${T}_/${T}_bench_/")"; done
for f in "$G"/prof_${T}*.txt; do [ -e "$f" ] && cp "$f" "$P/$(basename "$f" | sed "s/^prof_${T}/${T}_prof/")"; done
for d in "$G"/prof_${T}_*/; do
  [ -d "$d" ] || continue
  n=$(basename "$d"); n=${n#prof_${T}_}
  s=$(find "$d" -name '*kernel_stats.csv' | head -1)
  [ -n "$s" ] && cp "$s" "$P/${T}_${n}_kernel_stats.csv"
done
for d in "$G"/pmc_${T}_*/; do
  [ -d "$d" ] || continue
  n=$(basename "$d"); n=${n#pmc_${T}_}
  cp_if "$d/summary.txt" "$P/${T}_pmc_${n}_summary.txt"
done
cp_if "$G/envab_$T.txt" "$P/${T}_ab.txt"
cp_if "$G/pytest_gpu_$T.log" "$P/${T}_pytest_gpu_tail.txt" && [ -e "$P/${T}_pytest_gpu_tail.txt" ] && tail -3 "$P/${T}_pytest_gpu_tail.txt" > "$P/${T}_pytest_gpu_tail.tmp" && mv "$P/${T}_pytest_gpu_tail.tmp" "$P/${T}_pytest_gpu_tail.txt"
ls "$P" | grep "^${T}_"
