#!/bin/bash
# A/B of env settings on one bench config (no CPU baseline, no points).
#   usage (on the box): bash tools/ab_cfg.sh TAG CONFIG STEPS 'label|ENV=V ...|libname' ...
mkdir -p gpurun_out
tag=$1; cfg=$2; steps=$3; shift 3
for spec in "$@"; do
  IFS='|' read -r label envs lib <<< "$spec"
  if [ "$lib" != base ] && [ -n "$lib" ]; then libenv="MSGPU_LIB=$PWD/audio-suite_amd/msgpu/libmsgpu_$lib.so"; else libenv=""; fi
  echo "=== $cfg $label ($envs $libenv)"
  env $envs $libenv timeout -k 10 300 python bench.py --no-cpu --points= --fir-points= --config $cfg --steps $steps --from-dicts-steps 0 \
      > gpurun_out/${tag}_${cfg}_$label.json 2> gpurun_out/${tag}_${cfg}_$label.log
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -5 gpurun_out/${tag}_${cfg}_$label.log; exit $rc; fi
  python3 tools/brief.py gpurun_out/${tag}_${cfg}_$label.json
done
