#!/bin/bash
# GPU box: sampled stage profiling (bench PROFILE_EVERY = 4) -- H48 and C3 lines,
# and the stage-time GPU tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -k "stage or profil or h48" -x -q --timeout 200 --timeout-method thread > gpurun_out/r06pe_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r06pe_tests.txt
[ $rc -gt 1 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --config H48 --no-cpu --points= --fir-points= --steps 50 --from-dicts-steps 0 \
    --iso-steps 0 > gpurun_out/r06pe_h48_$i.json 2> gpurun_out/r06pe_h48_$i.log || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r06pe_h48_$i.json')); s=d['stage_ms']
print('H48', d['ms_per_step'], d['checked']['all_ok'], d.get('stage_sampling'), {k: s[k] for k in ('generate','spectral','fir_kernel','stereo','total','host_plan_wall')})"
done
timeout -k 10 200 python bench.py --no-cpu --points= --fir-points= --steps 40 --from-dicts-steps 0 --iso-steps 0 \
  > gpurun_out/r06pe_c3.json 2> gpurun_out/r06pe_c3.log || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/r06pe_c3.json')); s=d['stage_ms']
print('C3', d['ms_per_step'], d['checked']['all_ok'], d['roofline']['frac'], {k: s[k] for k in ('generate','spectral','overlap_add','fir_kernel','stereo','total')})"
