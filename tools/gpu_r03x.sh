#!/bin/bash
# Round-3 (x) session: bench.py launch events from launch 1 (no host-enqueue bubble in the event span):
# the driver's command three times and a 1000-step C2 line on one box.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 $([ $i -gt 1 ] && echo --no-cpu-baseline) > gpurun_out/y_drv_$i.json 2> gpurun_out/y_drv_$i.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/y_drv_$i.json').read().splitlines()[-1]);r=d['roofline'];print('driver cmd $i', d['value'], d['ms_per_step'], r['frac'], r['mean_launch_ms'], r['event_launches'], r['launch_ms_p10_p50_p90'])" | tee -a gpurun_out/y_drv.txt
done
timeout -k 10 240 python3 bench.py --config c2 --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/y_c2_1000.json 2> gpurun_out/y_c2_1000.err &&
python3 -c "import json;d=json.loads(open('gpurun_out/y_c2_1000.json').read().splitlines()[-1]);r=d['roofline'];print('c2 1000 steps', d['value'], d['ms_per_step'], r['frac'], r['mean_launch_ms'], r['event_launches'])" | tee -a gpurun_out/y_drv.txt
