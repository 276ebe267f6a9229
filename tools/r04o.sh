#!/bin/bash
# GPU box: C5 stream-gate sweep.  Stages (msgpu.hip stage_mark): 2 generator,
# 3 spectral, 4 overlap-add, 5 filter spectra, 8 FIR kernels, 6 stereo.  A gate
# W,R makes each context wait before its stage W until the previous context has
# begun stage R.  8,6 serialises the FIR kernels of the three streams (each
# waits for the previous sub-batch's stereo stage), so the CU-exclusive k_fir8
# blocks no longer queue behind each other's and the other stages' waves.
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, args...
  local t=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu --iso-steps 0 --from-dicts-steps 0 --points= "$@" > gpurun_out/r04o_$t.json 2> gpurun_out/r04o_$t.log || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r04o_$t.json')); print('$t', d['ms_per_step'], d['checked']['all_ok'])"
}
run C5_u --config C5 --steps 3 --gate none
run C5_g86 --config C5 --steps 3 --gate 8,6
run C5_g29 --config C5 --steps 3 --gate 2,9
run C5_g48 --config C5 --steps 3 --gate 4,8
run C5_g86_s2 --config C5 --steps 3 --gate 8,6 --streams 2
run C3_g24 --config C3 --steps 20
run C3_g86 --config C3 --steps 20 --gate 8,6
run C4_g24 --config C4 --steps 30
run C4_g86 --config C4 --steps 30 --gate 8,6
