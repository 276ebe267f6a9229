#!/bin/bash
# GPU box: GPU suite on the product (one wave per event, walk split from the
# emission) and on the K = 2 / 4 waves-per-event generator builds, then an A/B.
set -o pipefail
mkdir -p gpurun_out
for v in base k2 k4; do
  if [ $v != base ]; then export MSGPU_LIB=$PWD/audio-suite_amd/msgpu/libmsgpu_$v.so; else unset MSGPU_LIB; fi
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/r03ac_tests_$v.txt 2>&1 || { echo "== $v FAILED"; tail -25 gpurun_out/r03ac_tests_$v.txt; exit 1; }
  echo "== $v: $(tail -1 gpurun_out/r03ac_tests_$v.txt)"
done
unset MSGPU_LIB
timeout -k 10 700 bash tools/lib_ab.sh base k2 k4 base k2 k4 2>&1 || exit $?
