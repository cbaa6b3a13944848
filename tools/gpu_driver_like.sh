#!/bin/bash
# The driver's own bench command (python3 bench.py --gpus 1 --steps 20 --warmup 5, CPU baseline included)
# and longer runs on the same box, for the step-count sensitivity of the headline.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
TAG="${1:-r03}"
for k in 1 2; do
  timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driverlike_${TAG}_$k.json 2> gpurun_out/driverlike_${TAG}_$k.err
  python3 -c "import json;d=json.loads(open('gpurun_out/driverlike_${TAG}_$k.json').read().splitlines()[-1]);print('steps 20:',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['launch_ms_p10_p50_p90'])"
done
for s in 100 1000; do
  timeout -k 10 180 python3 bench.py --gpus 1 --steps $s --warmup 20 --no-cpu-baseline > gpurun_out/driverlike_${TAG}_s$s.json 2>/dev/null
  python3 -c "import json;d=json.loads(open('gpurun_out/driverlike_${TAG}_s$s.json').read().splitlines()[-1]);print('steps $s:',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['launch_ms_p10_p50_p90'])"
done
