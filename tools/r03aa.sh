#!/bin/bash
# GPU box: H48 with the one-partition 65 536-point FIR (default) against the
# 32 768 / 16 384-point kernels (MSGPU_FIR8=0), alternating.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for f in 1 0; do
    MSGPU_FIR8=$f timeout -k 10 200 python bench.py --config H48 --points= --no-cpu --steps 50 > gpurun_out/h48_fir8_$f.json 2>/dev/null || exit $?
    python3 -c "
import json;d=json.load(open('gpurun_out/h48_fir8_$f.json'));t=d['stage_ms'];i=d['roofline_isolated']['stage_ms'] if d.get('roofline_isolated') else {}
print('MSGPU_FIR8=$f step', d['ms_per_step'], 'value', d['value'], 'ok', (d['checked'] or {}).get('all_ok'), 'iso fir', i.get('fir_kernel'), 'iso fir_h', i.get('fir_h'), 'iso total', i.get('total'))"
  done
done
