#!/bin/bash
# Plain bench.py lines (no profiler) of one config under several EVAM_PP_* settings, alternating, two passes.
# Usage: tools/gpu_env_ab.sh TAG CFG "SET1|SET2|..."   (a SET is space-separated VAR=VALUE pairs and/or bench.py
# options such as --inflight=1)
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
TAG="$1"; CFG="$2"; IFS='|' read -ra LIST <<< "$3"
for pass in 1 2; do
  k=0
  for s in "${LIST[@]}"; do
    f=gpurun_out/envab_${TAG}_${CFG}_${k}_$pass.json; k=$((k + 1))
    envs=(); opts=()
    for w in $s; do case "$w" in --*) opts+=("$w") ;; *) envs+=("$w") ;; esac; done
    env "${envs[@]}" timeout -k 10 120 python bench.py --config $CFG --steps ${AB_STEPS:-1000} --warmup 100 --no-cpu-baseline \
      --resident-steps 0 "${opts[@]}" > $f 2>/dev/null
    python -c "import json; d=json.load(open('$f')); print('$CFG [$s]', d['value'], d['ms_per_step'], d['roofline']['frac'], 'single', d['roofline']['single_launch']['frac'], 'host_us', d['host_us_per_call'], 'submit_ms', d['host_submit_ms_per_step'])" | tee -a gpurun_out/envab_$TAG.txt
  done
done
