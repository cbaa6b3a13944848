#!/bin/bash
# Round-3 (x) session: ROI kernel chroma terms shared by both vertical taps when a whole wave reads one chroma row;
# ROI parity, then same-box A/B against the previous build (ab/libevam_pp_prev.so), plus C5 ring-depth knobs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fullsize.py \
  tests/test_gpu_parity.py -k "roi or c3" > gpurun_out/x3_tests.log 2>&1 && tail -3 gpurun_out/x3_tests.log &&
bash tools/gpu_env_ab.sh csame c3 "EVAM_PP_LIB=ab/libevam_pp_prev.so|EVAM_PP_ROI=1" &&
bash tools/gpu_env_ab.sh d c5 "EVAM_PP_STRIP_D=2|EVAM_PP_STRIP_D=3|EVAM_PP_STRIP_D=1|EVAM_PP_STRIP_WAVES=24"
