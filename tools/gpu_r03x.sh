#!/bin/bash
# Round-3 (x) session: strip / band prologues with every kernel-argument load before the first DMA in one batch
# (variant build ab/libevam_pp_batched.so): its parity through the strip and band kernels, then same-box A/B
# against the in-tree build.
set -o pipefail
mkdir -p gpurun_out
EVAM_PP_LIB=ab/libevam_pp_batched.so timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py tests/test_gpu_parity.py > gpurun_out/x4_tests.log 2>&1 && tail -3 gpurun_out/x4_tests.log &&
bash tools/gpu_env_ab.sh kb c5 "EVAM_PP_ROI=1|EVAM_PP_LIB=ab/libevam_pp_batched.so" &&
bash tools/gpu_env_ab.sh kb c1 "EVAM_PP_ROI=1|EVAM_PP_LIB=ab/libevam_pp_batched.so" &&
bash tools/gpu_env_ab.sh kb c2 "EVAM_PP_ROI=1|EVAM_PP_LIB=ab/libevam_pp_batched.so"
