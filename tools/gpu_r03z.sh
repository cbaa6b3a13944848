#!/bin/bash
# Variant A/B (tools/gpu_r03x.sh), then the final measurement of the in-tree build (tools/gpu_final_r03.sh r03z).
# A failed A/B (a parity mismatch of the variant) still lets the final run; a timeout, abort or crash does not.
bash tools/gpu_r03x.sh; rc=$?
echo "[r03z] variant A/B exit $rc"
case $rc in 124|134|137|139) exit $rc ;; esac
bash tools/gpu_final_r03.sh r03z
