#!/bin/bash
# GPU box: GPU suite, then A/B of k_spec3 with 2 / 3 / 4 events per workgroup.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r03y_gpu_tests.txt 2>&1
rc=$?
echo "== suite rc=$rc"; tail -2 gpurun_out/r03y_gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
MSGPU_LIB=$PWD/audio-suite_amd/msgpu/libmsgpu_ev4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03y_ev4_tests.txt 2>&1 || exit $?
tail -1 gpurun_out/r03y_ev4_tests.txt
timeout -k 10 600 bash tools/lib_ab.sh base ev3 ev4 base ev3 ev4 2>&1 || exit $?
