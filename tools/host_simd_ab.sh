#!/bin/bash
# C3 host-path A/B of EVAM_PP_HOST_SIMD (pass 1 on AVX2) on one box: the GPU ROI subset, then alternating
# 1000-step C3 bench lines with their host_us_per_call. Output: gpurun_out/hs_ab.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "roi or c3" -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_hs.log 2>&1 && tail -1 gpurun_out/pytest_hs.log \
  || { tail -30 gpurun_out/pytest_hs.log; exit 1; }
for pass in 1 2 3; do for v in 0 1; do
  EVAM_PP_HOST_SIMD=$v timeout -k 10 120 python bench.py --config c3 --steps 1000 --warmup 100 --no-cpu-baseline \
    --resident-steps 0 > gpurun_out/hs_${v}_$pass.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/hs_${v}_$pass.json')); print('c3 HOST_SIMD=$v', d['value'], d['ms_per_step'], d['roofline']['frac'], 'host_us_per_call', d['host_us_per_call'], 'host_submit', d['host_submit_ms_per_step'])" | tee -a gpurun_out/hs_ab.txt
done; done
