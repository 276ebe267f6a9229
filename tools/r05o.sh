#!/bin/bash
# round 5: overlap-add fused into k_fir8p -- bit-identity, then the suite, then A/B on C3 / C5
mkdir -p gpurun_out
T=${1:-r05o}
timeout -k 10 200 python -u -m pytest tests/test_gpu_long_filters.py -m gpu -q -s --timeout 150 --timeout-method thread \
  -k "ola_fused or fir4_spectra" > gpurun_out/${T}_ola_test.txt 2>&1; rc=$?; echo "ola test rc=$rc"; tail -4 gpurun_out/${T}_ola_test.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest tests -m gpu -q -s --timeout 250 --timeout-method thread \
  > gpurun_out/${T}_gpu_tests.txt 2>&1; rc=$?; echo "suite rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${T}_gpu_tests.txt | tail -8
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/ab_env.sh ${T} "c3def||base" "c3ola|MSGPU_OLA_FIR_DENSITY=1e9|base" "c3def2||base" "c3ola2|MSGPU_OLA_FIR_DENSITY=1e9|base" || exit $?
bash tools/ab_cfg.sh ${T} C5 6 "off|MSGPU_OLA_FIR=0|base" "def||base" "off2|MSGPU_OLA_FIR=0|base" "def2||base"
