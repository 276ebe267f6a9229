#!/bin/bash
# A/B the product library against tuning builds (build.py --exp-tu ... --out
# libmsgpu_<name>.so) on the default bench workload, one bench per variant.
#   usage (on the box): bash tools/lib_ab.sh base NAME [NAME|base ...]
set -e
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" != base ]; then export MSGPU_LIB=$PWD/audio-suite_amd/msgpu/libmsgpu_$v.so; else unset MSGPU_LIB; fi
  timeout -k 10 200 python bench.py --no-cpu --points= --fir-points= > gpurun_out/ab_$v.json 2>/dev/null
  python3 -c "
import json;d=json.load(open('gpurun_out/ab_$v.json'));i=d['roofline_isolated']['stage_ms'];t=d['stage_ms']
print('$v', 'step', d['ms_per_step'], 'ok', d['checked']['all_ok'])
print('  iso  ', {k: i[k] for k in ('generate','spectral','overlap_add','fir_kernel','fir_h','stereo')})
print('  timed', {k: t[k] for k in ('generate','spectral','overlap_add','fir_kernel','fir_h','stereo')})"
done
