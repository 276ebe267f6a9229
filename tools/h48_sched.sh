#!/bin/bash
# GPU box: H48's sub-batch size / stream count / gate (the step is a per-stream
# latency chain of ~20 small kernels, not throughput), alternating configurations.
set -o pipefail
mkdir -p gpurun_out
run() {
  tag=$1; shift
  timeout -k 10 200 python bench.py --config H48 --no-cpu --points= --fir-points= --steps 50 --from-dicts-steps 0 \
    --iso-steps 0 "$@" > gpurun_out/r06h48s_$tag.json 2> gpurun_out/r06h48s_$tag.log || return $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r06h48s_$tag.json'))
print('$tag', '$*', d['ms_per_step'], d['checked']['all_ok'], d['config'].get('sub_batches_per_gpu'), d['config'].get('stream_gate'))"
}
for i in 1 2; do
  run base$i || exit 1
  run s171_$i --sub 171 || exit 1
  run s128_$i --sub 128 || exit 1
  run s256x4_$i --sub 256 --streams 4 || exit 1
  run s171x6_$i --sub 171 --streams 6 || exit 1
  run nogate$i --gate none || exit 1
done
