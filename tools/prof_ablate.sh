#!/bin/bash
# rocprofv3 kernel durations of a workload under stage-removal diagnostic builds (the ablated launches
# compute INVALID results). Build the variants first, on the CPU side:
#   for a in 2 4 16; do tools/build_variant.sh abl$a "-DEVAM_PP_ABLATE=$a"; done
# Usage: tools/prof_ablate.sh TAG CFG "0 2 4 16" [extra bench args]   (0 = the product library)
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
TAG="$1"; CFG="$2"; ABL="$3"; shift 3
export TMPDIR=/tmp
cd /tmp
for a in $ABL; do
  d="$OUT/profabl_${TAG}_${CFG}_$a"
  # 0: the in-tree product library (or the caller's EVAM_PP_LIB variant)
  lib="$ROOT/ab/libevam_pp_abl$a.so"; [ "$a" = 0 ] && lib="${EVAM_PP_LIB:-}"
  if [ -n "$lib" ]; then export EVAM_PP_LIB="$lib"; else unset EVAM_PP_LIB; fi
  EVAM_PP_DIAGNOSTIC_BUILD_OK=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- \
    python3 "$ROOT/bench.py" --config "$CFG" --steps 200 --warmup 30 --no-cpu-baseline --resident-steps 0 "$@" \
    > "$d.json" 2> "$d.err" || { tail -5 "$d.err"; exit 1; }
  python3 - "$d" "$a" "$CFG" <<'PY' | tee -a "$OUT/profabl_$TAG.txt"
import csv, glob, sys
d, a, c = sys.argv[1:4]
for f in glob.glob(d + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "evam_pp" in r["Name"]:
            print(f"{c} ablate {a}: {r['Name'][:70]} calls {r['Calls']} avg {float(r['AverageNs'])/1e3:.2f} us "
                  f"min {float(r['MinNs'])/1e3:.2f} max {float(r['MaxNs'])/1e3:.2f}")
PY
done
