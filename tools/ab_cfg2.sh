#!/bin/bash
# GPU box: library A/B on one config: bash tools/ab_cfg2.sh TAG CFG STEPS lib1 lib2 ... (base = product)
set -o pipefail
mkdir -p gpurun_out
tag=$1; cfg=$2; steps=$3; shift 3
for i in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = base ]; then le=""; else le="MSGPU_LIB=$PWD/audio-suite_amd/msgpu/libmsgpu_$lib.so"; fi
    env $le timeout -k 10 400 python bench.py --config $cfg --no-cpu --points= --fir-points= --steps $steps \
      --from-dicts-steps 0 > gpurun_out/${tag}_${cfg}_${lib}_$i.json 2> gpurun_out/${tag}_${cfg}_${lib}_$i.log || exit $?
    echo -n "$cfg $lib $i: "; python3 tools/brief.py gpurun_out/${tag}_${cfg}_${lib}_$i.json | tr '\n' ' '; echo
  done
done
