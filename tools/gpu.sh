#!/bin/bash
# One parameterised GPU session: every round-5 one-off session script was a composition of these steps
# (testk + ab, prof + ablate, pmc) and is gone; a profile's header records the steps that made it. Every GPU step runs
# under its own time limit and the first failure ends the script.
#
#   tools/gpu.sh TAG STEP [STEP ...]
#
# Steps:
#   test              pytest -m gpu (one process)                      -> gpurun_out/pytest_gpu_TAG.log
#   testk:a,b         pytest -m gpu -k "a or b" (a subset before an A/B of the knob it covers)
#   ablate:CFG:B1,B2  rocprof of stage-removal builds (EVAM_PP_ABLATE bits, tools/prof_ablate.sh)
#   smoke             __graft_entry__.smoke()                          -> gpurun_out/smoke_TAG.txt
#   driver[:N]        the driver's own bench command (C2, CPU baseline), N times -> gpurun_out/bench_TAG_driver[_k].json
#   feed:c2,c4        bench.py --feed host (PCIe-inclusive) lines -> gpurun_out/bench_TAG_feed_<cfg>.json
#   pipe[:c2,c5]      bench.py --via pipeline per config (default c2, + its rocprof kernel stats); HUB, PIPE_ARGS
#   bench:c1,c2,...   one bench line per config (BENCH_STEPS, default 1000; CPU baseline unless CPU=0)
#   prof:c1,c2,...    rocprofv3 --kernel-trace --stats per config (tools/prof_configs.sh, 200 steps, bench default:
#                     three launches in flight)
#   prof1:c1,c2,...   the same, one launch at a time (--inflight 1: the kernel-quality average) -> prof_TAG_single_*
#   pmc:c2,c3,...     FETCH_SIZE / WRITE_SIZE passes per config (tools/pmc.sh) -> pmc_traffic_TAG_<cfg>.json
#   valu:c1,...       SQ_INSTS_VALU pass per config (tools/pmc.sh)
#   stall:c1,...      stall-attribution passes per config (tools/pmc.sh, two SQ groups)
#   scalar:c1,...     scalar-issue passes (SALU counts and cycles, SALUBusy / VALUBusy)
#   hostprof:c3       host time per evam_pp_run section (needs ab/libevam_pp_hostprof.so) -> hostprof_TAG.txt
#   ab:CFG:SET1|SET2  same-box alternating env / option A/B (tools/gpu_env_ab.sh)
#   dist              bench.py under torch.distributed.run, 2 ranks sharing the GPU over gloo
#
# Every output is stamped with EVAM_SHA (pass `EVAM_SHA=$(git rev-parse HEAD)` from the container: the box has
# no .git) and with the sha256 of the kernel source and bench.py as they were on the box.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
cd "$ROOT"
TAG="$1"; shift
SRC_SHA=$(cat edge-video-analytics-microservice_amd/csrc/*.hip edge-video-analytics-microservice_amd/csrc/*.h | sha256sum | cut -c1-16)
BENCH_SHA=$(sha256sum bench.py | cut -c1-16)
echo "{\"tag\": \"$TAG\", \"git_head\": \"${EVAM_SHA:-unknown}\", \"kernel_src_sha16\": \"$SRC_SHA\", \"bench_py_sha16\": \"$BENCH_SHA\", \"date\": \"$(date -u +%FT%TZ)\"}" \
  | tee "$OUT/stamp_$TAG.json"
CPUARG=""; [ "${CPU:-1}" = "0" ] && CPUARG="--no-cpu-baseline"
for st in "$@"; do
  kind="${st%%:*}"; arg="${st#*:}"; cfgs="${arg//,/ }"
  echo "[gpu.sh] $st"; date
  case "$kind" in
    test)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { tail -40 "$OUT/pytest_gpu_$TAG.log"; exit 1; }
      tail -1 "$OUT/pytest_gpu_$TAG.log" ;;
    testk)
      # a subset of the GPU suite: testk:c3,roi -> pytest -m gpu -k "c3 or roi" (env knobs apply: VAR=... gpu.sh ...)
      k="${arg//,/ or }"
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$k" \
        > "$OUT/pytest_gpu_${TAG}_k.log" 2>&1 || { tail -40 "$OUT/pytest_gpu_${TAG}_k.log"; exit 1; }
      tail -1 "$OUT/pytest_gpu_${TAG}_k.log" ;;
    ablate)
      # stage-removal rocprof of one config: ablate:c2:0,2,4,16 (EVAM_PP_ABLATE bit sets, tools/prof_ablate.sh)
      c="${arg%%:*}"; bits="${arg#*:}"
      bash tools/prof_ablate.sh "$TAG" "$c" "${bits//,/ }" ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.txt" 2>&1 \
        || { tail -20 "$OUT/smoke_$TAG.txt"; exit 1; }
      tail -1 "$OUT/smoke_$TAG.txt" ;;
    driver)
      # driver[:N]: the driver's own command N times on this box (box variance next to the 780.7 k bar)
      n=1; [ "$arg" != "$st" ] && n="$arg"
      for k in $(seq 1 "$n"); do
        sfx=""; [ "$n" -gt 1 ] && sfx="_$k"
        timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_${TAG}_driver$sfx.json" \
          2> "$OUT/bench_${TAG}_driver$sfx.err" || { tail -20 "$OUT/bench_${TAG}_driver$sfx.err"; exit 1; }
        tail -1 "$OUT/bench_${TAG}_driver$sfx.json"
      done ;;
    feed)
      # PCIe-inclusive lines: frames start in pinned host memory (f3 host feed, touched-rows plan)
      for c in $cfgs; do
        timeout -k 10 300 python3 bench.py --config "$c" --steps 300 --warmup 30 --feed host --no-cpu-baseline \
          > "$OUT/bench_${TAG}_feed_$c.json" 2> "$OUT/bench_${TAG}_feed_$c.err" || { tail -20 "$OUT/bench_${TAG}_feed_$c.err"; exit 1; }
        tail -1 "$OUT/bench_${TAG}_feed_$c.json"
      done ;;
    pipe)
      # frames through PipelineServer (device runner, null detector / no action decoder): a throughput line per config
      # (default c2, with its rocprof kernel stats); HUB (hub batch, default 256) and PIPE_ARGS pass on to bench.py
      [ "$arg" = "$st" ] && cfgs=c2
      for c in $cfgs; do
        timeout -k 10 300 python3 bench.py --via pipeline --config "$c" --hub-batch "${HUB:-256}" ${PIPE_ARGS:-} \
          > "$OUT/bench_${TAG}_pipeline_$c.json" 2> "$OUT/bench_${TAG}_pipeline_$c.err" || { tail -20 "$OUT/bench_${TAG}_pipeline_$c.err"; exit 1; }
        tail -1 "$OUT/bench_${TAG}_pipeline_$c.json"
        if [ "$c" = c2 ] && [ -z "${PIPE_ARGS:-}" ]; then
          PROF_ARGS="--via pipeline --hub-batch ${HUB:-256}" STEPS=200 bash tools/prof_configs.sh "${TAG}_pipeline" c2
        fi
      done ;;
    bench)
      for c in $cfgs; do
        timeout -k 10 300 python3 bench.py --config "$c" --steps "${BENCH_STEPS:-1000}" --warmup 100 $CPUARG \
          ${BENCH_ARGS:-} > "$OUT/bench_${TAG}_$c.json" 2> "$OUT/bench_${TAG}_$c.err" || { tail -20 "$OUT/bench_${TAG}_$c.err"; exit 1; }
        python3 - "$OUT/bench_${TAG}_$c.json" "$c" <<'PY' | tee -a "$OUT/bench_$TAG.txt"
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1]); r = d["roofline"]; cb = d.get("cpu_baseline") or {}
print(sys.argv[2], d["value"], "f/s", d["ms_per_step"], "ms/step", r["bound"], r["frac"], "hbm", r.get("hbm", {}).get("frac"),
      "p10/50/90", r["launch_ms_p10_p50_p90"], "lat", d.get("latency", {}).get("ms_p10_p50_p90"), "cpu", cb.get("value"))
PY
      done ;;
    prof)
      STEPS=200 bash tools/prof_configs.sh "$TAG" "$cfgs" ;;
    prof1)
      PROF_ARGS="--inflight 1" STEPS=200 bash tools/prof_configs.sh "${TAG}_single" "$cfgs" ;;
    pmc)
      for c in $cfgs; do
        PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" bash tools/pmc.sh "${TAG}_$c" "$c"
        cp "$OUT/pmc_traffic.json" "$OUT/pmc_traffic_${TAG}_$c.json"
      done ;;
    valu)
      for c in $cfgs; do
        PMC_GROUPS="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" bash tools/pmc.sh "${TAG}_valu_$c" "$c"
      done ;;
    scalar)
      # scalar issue: SALU instructions and cycles, scalar-active wave cycles next to VALU, then the
      # derived SALUBusy / VALUBusy percentages (one launch at a time)
      for c in $cfgs; do
        PMC_GROUPS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE;SALUBusy VALUBusy" \
          bash tools/pmc.sh "${TAG}_scalar_$c" "$c"
      done ;;
    stall)
      # Stall attribution: WAIT_ANY (parked on s_waitcnt / barrier) + WAIT_INST_ANY (issue stall; WAIT_INST_LDS is
      # its LDS sub-bucket) + ACTIVE_INST_ANY ~ WAVE_CYCLES; LDS bank conflicts against all LDS-array cycles.
      for c in $cfgs; do
        PMC_GROUPS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD" \
          bash tools/pmc.sh "${TAG}_stall_$c" "$c"
      done ;;
    hostprof)
      # host time per section of evam_pp_run (a -DEVAM_PP_HOST_PROF build: tools/build_variant.sh hostprof
      # -DEVAM_PP_HOST_PROF before the call), one launch at a time, plus the bench's own host_us_per_call
      for c in $cfgs; do
        EVAM_PP_LIB=ab/libevam_pp_hostprof.so timeout -k 10 200 python3 bench.py --config "$c" --steps 1000 --warmup 100 \
          --no-cpu-baseline --inflight 1 > "$OUT/hostprof_${TAG}_$c.json" 2> "$OUT/hostprof_${TAG}_$c.err" \
          || { tail -20 "$OUT/hostprof_${TAG}_$c.err"; exit 1; }
        echo "$c $(grep 'host prof' "$OUT/hostprof_${TAG}_$c.err") host_us_per_call $(python3 -c "import json; print(json.loads(open('$OUT/hostprof_${TAG}_$c.json').read().splitlines()[-1])['host_us_per_call'])")" \
          | tee -a "$OUT/hostprof_$TAG.txt"
      done ;;
    ab)
      c="${arg%%:*}"; sets="${arg#*:}"
      bash tools/gpu_env_ab.sh "$TAG" "$c" "$sets" ;;
    dist)
      EVAM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 100 --warmup 20 \
        > "$OUT/bench_dist2_$TAG.json" 2> "$OUT/bench_dist2_$TAG.err" || { tail -20 "$OUT/bench_dist2_$TAG.err"; exit 1; }
      tail -1 "$OUT/bench_dist2_$TAG.json" ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "[gpu.sh] done"; date
