#!/bin/bash
# rocprofv3 kernel durations of one bench workload under several EVAM_PP_* knob settings (tuning sweep;
# every setting computes the same result, which the parity suite checks per forced variant).
# Usage: tools/sweep_env.sh TAG CFG "EVAM_PP_TH=4 EVAM_PP_STAGE_NBUF=3|EVAM_PP_TH=8|..." [extra bench args]
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
TAG="$1"; CFG="$2"; SETS="$3"; shift 3
export TMPDIR=/tmp
cd /tmp
IFS='|' read -ra LIST <<< "$SETS"
k=0
for s in "${LIST[@]}"; do
  d="$OUT/sweep_${TAG}_${CFG}_$k"; k=$((k + 1))
  env $s timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- \
    python3 "$ROOT/bench.py" --config "$CFG" --steps 200 --warmup 30 --no-cpu-baseline --resident-steps 0 "$@" \
    > "$d.json" 2> "$d.err" || { tail -5 "$d.err"; exit 1; }
  python3 - "$d" "$s" "$CFG" <<'PY' | tee -a "$OUT/sweep_$TAG.txt"
import csv, glob, json, sys
d, s, c = sys.argv[1:4]
b = json.load(open(d + ".json"))
for f in glob.glob(d + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "evam_pp" in r["Name"]:
            print(f"{c} [{s}]: {r['Name'][37:80]} calls {r['Calls']} avg {float(r['AverageNs'])/1e3:.2f} us "
                  f"min {float(r['MinNs'])/1e3:.2f} | step {b['ms_per_step']*1e3:.1f} us value {b['value']}")
PY
done
