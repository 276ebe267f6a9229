#!/bin/bash
# stereo max pass in 16-frame runs (experiment library st16): GPU suite on it, then A/B
mkdir -p gpurun_out
MSGPU_LIB=$PWD/audio-suite_amd/msgpu/libmsgpu_st16.so timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
  > gpurun_out/r05af_gpu_tests.txt 2>&1; rc=$?; echo "suite rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r05af_gpu_tests.txt | tail -5
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/ab_env.sh r05af "base||base" "st16||st16" "base2||base" "st16b||st16" || exit $?
bash tools/ab_cfg.sh r05af C5 6 "base||base" "st16||st16"
