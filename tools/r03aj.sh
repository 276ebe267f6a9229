#!/bin/bash
# GPU box: k_gen_normal capped at 112 VGPRs (MSG_GEN_VGPRS=56: the attribute
# counts half the unified register file on gfx950; 4 spilled VGPRs) so that a
# 64-VGPR k_ola_env wave fits beside four generator waves on a SIMD, against
# the uncapped product (119 VGPRs: 32 free per SIMD), alternating.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 bash tools/lib_ab.sh base g112 base g112 > gpurun_out/r03aj_ab.txt 2>&1; rc=$?
cat gpurun_out/r03aj_ab.txt; exit $rc
