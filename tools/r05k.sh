#!/bin/bash
# round-5 GPU session: the >2^29-frame test, the GPU suite, the default bench line,
# the FIR engine comparison (k_fir8p vs k_fir4 vs k_fir2 at C3)
mkdir -p gpurun_out
T=${1:-r05k}
timeout -k 10 300 python -u -m pytest tests/test_gpu_long_output.py -x -q -s --timeout 250 --timeout-method thread \
  > gpurun_out/${T}_long.txt 2>&1; rc=$?; echo "long rc=$rc"; tail -4 gpurun_out/${T}_long.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread \
  > gpurun_out/${T}_gpu_tests.txt 2>&1; rc=$?; echo "suite rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/${T}_gpu_tests.txt | tail -8
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit $?
python3 tools/brief.py gpurun_out/${T}_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/${T}_bench.json')); r=d['roofline']
print('roofline', r['kernel'], r['frac'], 'stage', r['fir_rfft_stage'])"
bash tools/ab_env.sh ${T}fir "fir8p||base" "fir4|MSGPU_FIR8=0|base" "fir2|MSGPU_FIR8=0 MSGPU_FIR4=0|base"
