#!/bin/bash
# rocprofv3 kernel-trace summary of each bench workload: the evam_pp kernel's own average duration
# next to the bench's step time (tells a host-bound step from a slow kernel).
# Usage: tools/prof_configs.sh TAG "c1 c3 c5"   -> gpurun_out/prof_TAG_<cfg>/..., prof_TAG.txt
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
TAG="${1:-prof}"; CFGS="${2:-c1 c2 c3 c4 c5}"
export TMPDIR=/tmp
cd /tmp
for c in $CFGS; do
  echo "[prof] $c"; date
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_$c" -o run -- \
    python3 "$ROOT/bench.py" --config "$c" --steps ${STEPS:-200} --warmup 50 --no-cpu-baseline --resident-steps 0 ${PROF_ARGS:-} \
    > "$OUT/prof_${TAG}_$c.json" 2> "$OUT/prof_${TAG}_$c.err" || { tail -20 "$OUT/prof_${TAG}_$c.err"; exit 1; }
  python3 - "$OUT/prof_${TAG}_$c" "$OUT/prof_${TAG}_$c.json" "$c" <<'EOF' | tee -a "$OUT/prof_$TAG.txt"
import csv, glob, json, sys
d, bj, c = sys.argv[1:4]
b = json.load(open(bj))
for f in glob.glob(d + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "evam_pp" in r["Name"]:
            avg_us = float(r["AverageNs"]) / 1e3
            ab = b.get("roofline", {}).get("algorithmic_bytes_per_launch")
            rate = f" ({ab / avg_us / 1e3:.0f} GB/s alg)" if ab else ""
            tail = (f" | bench step {b['ms_per_step'] * 1e3:.2f} us, value {b['value']}, event-based "
                    f"{b['roofline']['achieved']} GB/s" if "ms_per_step" in b else f" | value {b['value']}")
            print(f"{c}: kernel {r['Name'][:60]} calls {r['Calls']} avg {avg_us:.2f} us{rate}{tail}")
EOF
done
echo "[prof] done"; date
