#!/bin/bash
# A/B of libraries / env settings on the default C3 bench (no CPU baseline, no points).
#   usage (on the box): bash tools/ab_env.sh TAG 'label|ENV=V ...|libname' ...
# libname: msgpu/libmsgpu_<libname>.so, or 'base' for the product library.
mkdir -p gpurun_out
tag=$1; shift
for spec in "$@"; do
  IFS='|' read -r label envs lib <<< "$spec"
  if [ "$lib" != base ] && [ -n "$lib" ]; then libenv="MSGPU_LIB=$PWD/audio-suite_amd/msgpu/libmsgpu_$lib.so"; else libenv=""; fi
  echo "=== $label ($envs $libenv)"
  env $envs $libenv timeout -k 10 200 python bench.py --no-cpu --points= --fir-points= --steps 40 --from-dicts-steps 0 \
      > gpurun_out/${tag}_$label.json 2> gpurun_out/${tag}_$label.log
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -5 gpurun_out/${tag}_$label.log; exit $rc; fi
  python3 tools/brief.py gpurun_out/${tag}_$label.json
done
