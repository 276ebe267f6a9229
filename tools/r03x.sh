#!/bin/bash
# GPU box: GPU suite, then A/B of k_spec3 with two events per workgroup (the
# second's grain prefetched) against one event per workgroup.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r03x_gpu_tests.txt 2>&1
rc=$?
echo "== suite rc=$rc"; tail -2 gpurun_out/r03x_gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash tools/lib_ab.sh base nopair base nopair 2>&1 || exit $?
