#!/bin/bash
# GPU box: the 2,4 stream gate against none on the short-step points (H48, C4),
# alternating, three pairs each.
set -o pipefail
mkdir -p gpurun_out
run() {
  cfg=$1; tag=$2; shift 2
  timeout -k 10 200 python bench.py --config $cfg --no-cpu --points= --fir-points= --steps 50 --from-dicts-steps 0 \
    --iso-steps 0 "$@" > gpurun_out/r06g2_${cfg}_$tag.json 2> gpurun_out/r06g2_${cfg}_$tag.log || return $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r06g2_${cfg}_$tag.json'))
print('$cfg $tag', d['ms_per_step'], d['checked']['all_ok'], d['config'].get('stream_gate'))"
}
for cfg in H48 C4; do
  for i in 1 2 3; do
    run $cfg gate$i || exit 1
    run $cfg none$i --gate none || exit 1
  done
done
