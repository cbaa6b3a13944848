#!/bin/bash
# Build libevam_pp.so from the kernel sources of git revision REV into ab/libevam_pp_NAME.so, for same-box A/B runs
# against the working tree (EVAM_PP_LIB=ab/libevam_pp_NAME.so). Usage: tools/build_rev.sh REV NAME
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
T=$(mktemp -d); trap 'rm -rf "$T"' EXIT
mkdir -p "$T/include" "$T/pkg/csrc" "$ROOT/ab"
git -C "$ROOT" archive "$1" include edge-video-analytics-microservice_amd/csrc | tar -x -C "$T"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wall -Wno-unused-function \
  -I "$T/include" -o "$ROOT/ab/libevam_pp_$2.so" "$T/edge-video-analytics-microservice_amd/csrc/evam_pp.hip"
echo "built ab/libevam_pp_$2.so from $1"
