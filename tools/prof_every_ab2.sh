#!/bin/bash
# GPU box: H48 with stage events on every batch (1), every 4th, every 16th and
# none (0), alternating, same session.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for k in 1 4 16 0; do
    MSGPU_BENCH_PROFILE_EVERY=$k timeout -k 10 200 python bench.py --config H48 --no-cpu --points= --fir-points= \
      --steps 50 --from-dicts-steps 0 --iso-steps 0 > gpurun_out/r06pe2_${k}_$i.json 2> gpurun_out/r06pe2_${k}_$i.log || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/r06pe2_${k}_$i.json'))
print('H48 every $k', $i, d['ms_per_step'], d['checked']['all_ok'])"
  done
done
