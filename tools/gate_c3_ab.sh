#!/bin/bash
# GPU box: C3's stream gate re-measured on the round-6 kernels, alternating pairs.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for g in 2,4 none; do
    timeout -k 10 200 python bench.py --no-cpu --points= --fir-points= --steps 40 --from-dicts-steps 0 --iso-steps 0 \
      --gate $g > gpurun_out/r06g3_${g/,/_}_$i.json 2> gpurun_out/r06g3_${g/,/_}_$i.log || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/r06g3_${g/,/_}_$i.json'))
print('C3 gate $g', $i, d['ms_per_step'], d['checked']['all_ok'])"
  done
done
