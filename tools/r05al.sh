#!/bin/bash
# ER gains drawn on the device (k_er_gains): GPU suite, then H48 / C3 A/B against host-drawn gains (MSGPU_ER_DEV=0)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q -s --timeout 250 --timeout-method thread \
  > gpurun_out/r05al_gpu_tests.txt 2>&1; rc=$?; echo "suite rc=$rc"; grep -E "FAILED|passed|failed|host-drawn" gpurun_out/r05al_gpu_tests.txt | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/ab_cfg.sh r05al H48 50 "dev||base" "host|MSGPU_ER_DEV=0|base" "dev2||base" "host2|MSGPU_ER_DEV=0|base" || exit $?
bash tools/ab_env.sh r05al "c3||base" "c3host|MSGPU_ER_DEV=0|base"
