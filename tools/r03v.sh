#!/bin/bash
# GPU box: GPU suite (product), then A/B of k_spec3 split pass-2 twiddles with the
# generator's 4.2 KB LDS mode (co-residence beside k_spec3) against the previous layout.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r03v_gpu_tests.txt 2>&1
rc=$?
echo "== suite rc=$rc"; tail -2 gpurun_out/r03v_gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
MSGPU_LIB=$PWD/audio-suite_amd/msgpu/libmsgpu_cores.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03v_cores_tests.txt 2>&1 || exit $?
tail -1 gpurun_out/r03v_cores_tests.txt
timeout -k 10 500 bash tools/lib_ab.sh base cores old base cores old 2>&1 || exit $?
