#!/bin/bash
# GPU box: GPU suite on the product library, then an A/B of k_gen_normal variants.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r03l_gpu_tests.txt 2>&1
rc=$?
echo "== suite rc=$rc"; tail -3 gpurun_out/r03l_gpu_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 bash tools/lib_ab.sh base noslow base 2>&1
