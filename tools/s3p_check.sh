#!/bin/bash
# GPU box: k_spec3p (MSGPU_SPEC3P=1) against the two-event chain -- bits on the
# mixed batch and on C3 / C4, the spectral tests under the persistent form,
# then the isolated / timed A/B on C3 and C4.
set -o pipefail
mkdir -p gpurun_out
L=audio-suite_amd/msgpu/libmsgpu.so
timeout -k 10 300 python tools/bits_ab.py "$L,MSGPU_SPEC3P=0" "$L,MSGPU_SPEC3P=1" > gpurun_out/r06u_bits.json 2> gpurun_out/r06u_bits.log
echo "bits rc=$?"; cat gpurun_out/r06u_bits.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_long_filters.py -k 'spec3_persistent or fir8_persistent' -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/r06u_tests0.txt 2>&1; echo "persist test rc=$?"; tail -3 gpurun_out/r06u_tests0.txt
MSGPU_SPEC3P=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k 'spec3 or C3 or C4' -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06u_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06u_tests.txt
[ $rc -gt 1 ] && exit $rc
bash tools/ab_env.sh r06u 'p0|MSGPU_SPEC3P=0|base' 'p1|MSGPU_SPEC3P=1|base' 'p0b|MSGPU_SPEC3P=0|base' 'p1b|MSGPU_SPEC3P=1|base'
