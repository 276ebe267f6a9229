#!/bin/bash
# GPU box: GPU suite, A/B of the FIR exchange layouts, SQ counters of the product library.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r03p_gpu_tests.txt 2>&1
rc=$?
echo "== suite rc=$rc"; tail -3 gpurun_out/r03p_gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash tools/lib_ab.sh base base 2>&1 || exit $?
bash tools/pmc_sq2.sh r03p || exit $?
grep -A22 "^k_fir8<0>" gpurun_out/r03p_sq_summary.txt | grep -E "INSTS_VALU|BANK|IDX_ACTIVE|WAIT_ANY/|insts per"
