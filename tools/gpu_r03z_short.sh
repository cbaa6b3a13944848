#!/bin/bash
# Final in-tree build, short: the GPU suite, smoke(), the driver's bench command, and rocprofv3 kernel stats of C2.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/z_pytest.log 2>&1 && tail -1 gpurun_out/z_pytest.log &&
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/z_smoke.txt 2>&1 && tail -1 gpurun_out/z_smoke.txt &&
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/z_driver.json 2> gpurun_out/z_driver.err && tail -1 gpurun_out/z_driver.json &&
STEPS=200 bash tools/prof_configs.sh r03z "c2 c1"
