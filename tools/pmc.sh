#!/bin/bash
# PMC passes over the default bench (one counter group per rocprofv3 run, kernel-trace/stats only,
# never combined with sys/runtime tracing). Output: gpurun_out/pmc_<tag>/<pass>/...counter_collection.csv
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc_${1:-r01}"; mkdir -p "$OUT"
CFG="${2:-c2}"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$ROOT/bench.py" --config "$CFG" --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/p$i.json" 2> "$OUT/p$i.err" \
    || { echo "pass $i ($grp) failed"; tail -5 "$OUT/p$i.err"; exit 1; }
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT" | tee "$OUT/summary.txt"
