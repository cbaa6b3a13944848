#!/bin/bash
# Round-3 (x) session: ROI / strip prologue barriers (LDS-only) and the ROI tail split, parity then same-box A/B
# against the HEAD build in ab/libevam_pp_old.so.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fullsize.py \
  "tests/test_gpu_parity.py" -k "roi or c3 or c5 or c2 or c4 or c1" > gpurun_out/x_tests.log 2>&1 && tail -3 gpurun_out/x_tests.log &&
bash tools/gpu_env_ab.sh bar c3 "EVAM_PP_LIB=ab/libevam_pp_old.so|EVAM_PP_ROI_TAIL=1|EVAM_PP_ROI_TAIL=2|EVAM_PP_ROI_TAIL=4" &&
bash tools/gpu_env_ab.sh bar c5 "EVAM_PP_LIB=ab/libevam_pp_old.so|EVAM_PP_ROI=1" &&
bash tools/gpu_env_ab.sh bar c2 "EVAM_PP_LIB=ab/libevam_pp_old.so|EVAM_PP_ROI=1"
