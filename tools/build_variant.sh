#!/bin/bash
# Build a variant of libevam_pp.so with extra compile definitions for same-box A/B runs
# (select it with EVAM_PP_LIB=ab/libevam_pp_NAME.so). Usage: tools/build_variant.sh NAME "-DFOO=1 ..."
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$ROOT/ab"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wall -Wno-unused-function $2 \
  -I "$ROOT/include" -o "$ROOT/ab/libevam_pp_$1.so" "$ROOT/edge-video-analytics-microservice_amd/csrc/evam_pp.hip"
echo "built ab/libevam_pp_$1.so"
