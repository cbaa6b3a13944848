#!/bin/bash
# Round-3 (x) session: strip-kernel LUT by LDS-DMA (no ring drain at the LUT barrier); parity, then same-box A/B
# against the previous build in ab/libevam_pp_old.so.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fullsize.py \
  tests/test_gpu_parity.py tests/test_abi.py > gpurun_out/x2_tests.log 2>&1 && tail -3 gpurun_out/x2_tests.log &&
bash tools/gpu_env_ab.sh lut c5 "EVAM_PP_LIB=ab/libevam_pp_old.so|EVAM_PP_ROI=1" &&
bash tools/gpu_env_ab.sh lut c2 "EVAM_PP_LIB=ab/libevam_pp_old.so|EVAM_PP_ROI=1" &&
bash tools/gpu_env_ab.sh lut c4 "EVAM_PP_LIB=ab/libevam_pp_old.so|EVAM_PP_ROI=1"
