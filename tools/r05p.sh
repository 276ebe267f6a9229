#!/bin/bash
# round 5: filter spectra before the generator -- bit-identity, then A/B on C3 / C5
mkdir -p gpurun_out
T=${1:-r05p}
timeout -k 10 200 python -u -m pytest tests/test_gpu_long_filters.py -m gpu -q -s --timeout 150 --timeout-method thread \
  -k "early or ola_fused" > gpurun_out/${T}_test.txt 2>&1; rc=$?; echo "test rc=$rc"; tail -3 gpurun_out/${T}_test.txt
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/ab_cfg.sh ${T} C5 6 "late|MSGPU_H_EARLY=0|base" "early||base" "late2|MSGPU_H_EARLY=0|base" "early2||base" || exit $?
bash tools/ab_env.sh ${T} "c3late|MSGPU_H_EARLY=0|base" "c3early||base" "c3late2|MSGPU_H_EARLY=0|base" "c3early2||base"
