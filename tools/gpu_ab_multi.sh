#!/bin/bash
# Same-box A/B of several configs: tools/gpu_env_ab.sh (alternating arms, two passes) per config.
#   tools/gpu_ab_multi.sh TAG "c2 c5 ..." "SET1|SET2|..."
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
for c in $2; do
  bash tools/gpu_env_ab.sh "$1" "$c" "$3"
done
