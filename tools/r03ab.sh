#!/bin/bash
# GPU box: A/B of the stereo loads/stores with 32-bit offsets (base) against
# the previous commit's msgpu TU (old).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 bash tools/lib_ab.sh base old base old 2>&1 || exit $?
