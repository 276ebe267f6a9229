#!/bin/bash
# round 5: fused overlap-add (DIF split folded in, chosen per batch) -- tests, C3 against the previous library, C5
mkdir -p gpurun_out
T=${1:-r05t}
timeout -k 10 200 python -u -m pytest tests/test_gpu_long_filters.py -m gpu -q -s --timeout 150 --timeout-method thread \
  -k "early or ola_fused or persistent" > gpurun_out/${T}_test.txt 2>&1; rc=$?; echo "test rc=$rc"; tail -3 gpurun_out/${T}_test.txt
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/ab_env.sh ${T} "new||base" "old||old" "ola|MSGPU_OLA_FIR_DENSITY=1e9|base" "new2||base" "old2||old" "ola2|MSGPU_OLA_FIR_DENSITY=1e9|base" || exit $?
bash tools/ab_cfg.sh ${T} C5 6 "c5||base" "c5old||old" "c5off|MSGPU_OLA_FIR=0|base"
