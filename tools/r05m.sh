#!/bin/bash
mkdir -p gpurun_out
T=${1:-r05m}
timeout -k 10 500 python -u -m pytest tests -m gpu -q -s --timeout 250 --timeout-method thread \
  > gpurun_out/${T}_gpu_tests.txt 2>&1; rc=$?; echo "suite rc=$rc"; grep -E "FAILED|passed|failed|Error|FIR4C" gpurun_out/${T}_gpu_tests.txt | tail -14
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/ab_env.sh ${T} "base||base" "base2||base" || exit $?
bash tools/ab_cfg.sh ${T} H48 50 "c1||base" "c0|MSGPU_FIR4C=0|base" "c1b||base" "c0b|MSGPU_FIR4C=0|base" || exit $?
bash tools/ab_cfg.sh ${T} C5 6 "base||base"
