#!/bin/bash
# C5 sub-batch size A/B
mkdir -p gpurun_out
run() { local l=$1; shift
  timeout -k 10 300 python bench.py --config C5 --no-cpu --points= --steps 6 --from-dicts-steps 0 --iso-steps 0 "$@" \
      > gpurun_out/r05ag_$l.json 2> gpurun_out/r05ag_$l.log || return $?
  python3 -c "import json;d=json.loads(open('gpurun_out/r05ag_$l.json').read().strip().split(chr(10))[-1]);print('$l', d['ms_per_step'], d['value'], d['checked']['all_ok'] if d.get('checked') else '')"; }
run s171 && run s256 --sub 256 && run s171b && run s256b --sub 256 && run s128 --sub 128
