#!/bin/bash
# GPU box: k_fir8p phase stamps against the number of persistent workgroups
# (MSGPU_FIR8P_CUS): does a block's segment-load phase shrink when fewer CUs
# share HBM (bandwidth share) or stay (latency)?
set -o pipefail
mkdir -p gpurun_out
for c in 256 128 64 16 8; do
  echo "=== $c workgroups"
  MSGPU_FIR8P_CUS=$c MSGPU_LIB=$PWD/audio-suite_amd/msgpu/libmsgpu_firstamps.so timeout -k 10 200 python tools/fir8_stamps.py C3 256 || exit $?
done
