#!/bin/bash
# round 5: k_fir8p split into plain / fused-overlap-add instantiations -- tests, C3 and C5
mkdir -p gpurun_out
T=${1:-r05q}
timeout -k 10 200 python -u -m pytest tests/test_gpu_long_filters.py -m gpu -q -s --timeout 150 --timeout-method thread \
  -k "early or ola_fused or persistent" > gpurun_out/${T}_test.txt 2>&1; rc=$?; echo "test rc=$rc"; tail -3 gpurun_out/${T}_test.txt
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/ab_env.sh ${T} "c3||base" "c3b||base" || exit $?
bash tools/ab_cfg.sh ${T} C5 6 "c5||base" "c5b||base"
