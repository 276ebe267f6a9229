#!/bin/bash
# GPU box (round 4): the GPU suite with the k_fir8 filter-length fix.
set -o pipefail
tag=${1:-r04a}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -v -s -x --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.txt 2>&1
rc=$?
echo "== suite rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/${tag}_gpu_tests.txt | tail -6
exit $rc
