#!/bin/bash
# PMC passes over the default bench, one launch at a time (--inflight 1: per-dispatch counters of one kernel; one counter group per rocprofv3 run, kernel-trace/stats only,
# never combined with sys/runtime tracing). Per run at most 8 SQ_, 4 TCC_, 4 TCP_, 2 TA_, 2 TD_, 2 GRBM_ counters. Output: gpurun_out/pmc_<tag>/<pass>/...counter_collection.csv
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc_${1:-r01}"; mkdir -p "$OUT"
CFG="${2:-c2}"
export TMPDIR=/tmp
cd /tmp
i=0
if [ -n "${PMC_GROUPS:-}" ]; then IFS=';' read -ra GROUPS_DEFAULT <<< "$PMC_GROUPS"; else
GROUPS_DEFAULT=("FETCH_SIZE" "WRITE_SIZE"
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU"
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL"
  "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"
  "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TOTAL_WAVEFRONTS_sum"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum"
  "GRBM_GUI_ACTIVE TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum")
fi
for grp in "${GROUPS_DEFAULT[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$ROOT/bench.py" --config "$CFG" --steps 20 --warmup 5 --no-cpu-baseline --resident-steps 0 --inflight 1 ${PMC_BENCH_ARGS:-} > "$OUT/p$i.json" 2> "$OUT/p$i.err" \
    || { echo "pass $i ($grp) failed"; tail -5 "$OUT/p$i.err"; exit 1; }
done
FR=$(python3 -c "import json;print(json.load(open('$OUT/p1.json'))['config']['frames_per_gpu_per_step'])")
PS=$(python3 -c "import json;print(json.load(open('$OUT/p1.json'))['config']['pool_sets'])")
python3 "$ROOT/tools/pmc_summary.py" "$OUT" "$CFG" "$FR" "$ROOT/gpurun_out/pmc_traffic.json" "$PS" | tee "$OUT/summary.txt"
# the raw per-dispatch CSVs run to tens of MB per pass; the summary keeps what is used (gpurun copies back <= 64 MiB)
rm -rf "$OUT"/p*/
