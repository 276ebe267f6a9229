#!/bin/bash
# GPU box: sub-batch sizes for C3 and C4 on the round-6 kernels (3 streams, default gate), alternating.
set -o pipefail
mkdir -p gpurun_out
run() {
  cfg=$1; sub=$2; i=$3
  timeout -k 10 200 python bench.py --config $cfg --no-cpu --points= --fir-points= --steps 30 --from-dicts-steps 0 \
    --iso-steps 0 --sub $sub > gpurun_out/r06ss_${cfg}_${sub}_$i.json 2> gpurun_out/r06ss_${cfg}_${sub}_$i.log || return $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r06ss_${cfg}_${sub}_$i.json'))
print('$cfg sub $sub', $i, d['ms_per_step'], d['checked']['all_ok'], d['config'].get('sub_batches_per_gpu'))"
}
for i in 1 2; do
  for sub in 342 256 205 171; do run C3 $sub $i || exit 1; done
  for sub in 171 128 256; do run C4 $sub $i || exit 1; done
done
