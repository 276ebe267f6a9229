#!/bin/bash
# A/B of msg_gate schedules between the two streams' contexts on the default
# bench workload.   usage (on the box): bash tools/gate_ab.sh none 2,6 [...]
set -e
mkdir -p gpurun_out
for g in "$@"; do
  timeout -k 10 200 python bench.py --no-cpu --points= --gate "$g" > gpurun_out/gate_${g/,/_}.json 2>/dev/null
  python3 -c "
import json;d=json.load(open('gpurun_out/gate_${g/,/_}.json'));t=d['stage_ms']
print('gate $g', 'step', d['ms_per_step'], 'Msamples/s', d['value'], 'ok', d['checked']['all_ok'])
print('  timed', {k: t[k] for k in ('generate','spectral','overlap_add','fir_kernel','fir_h','stereo')})"
done
