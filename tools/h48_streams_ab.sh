#!/bin/bash
# GPU box: H48 ungated with 2 / 3 / 4 streams (sub-batches of 512 / 341 / 256), alternating.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for cfg in "3 341" "2 512" "4 256"; do
    set -- $cfg
    timeout -k 10 200 python bench.py --config H48 --no-cpu --points= --fir-points= --steps 50 --from-dicts-steps 0 \
      --iso-steps 0 --gate none --streams $1 --sub $2 > gpurun_out/r06hs_$1_$i.json 2> gpurun_out/r06hs_$1_$i.log || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/r06hs_$1_$i.json'))
print('H48 streams $1 sub $2', $i, d['ms_per_step'], d['checked']['all_ok'])"
  done
done
