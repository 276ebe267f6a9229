#!/bin/bash
# C3 sub-batch size / gate sweep (A/B only)
mkdir -p gpurun_out
run() {   # label, bench args...
  local l=$1; shift
  timeout -k 10 200 python bench.py --no-cpu --points= --steps 40 --from-dicts-steps 0 --iso-steps 0 "$@" \
      > gpurun_out/r05z_$l.json 2> gpurun_out/r05z_$l.log || return $?
  python3 -c "import json;d=json.loads(open('gpurun_out/r05z_$l.json').read().strip().split(chr(10))[-1]);print('$l', d['ms_per_step'], d['value'])"
}
run def && run s171 --sub 171 && run s256 --sub 256 && run s512 --sub 512 --streams 2 && run def2 && run s171b --sub 171 && run s256b --sub 256 && run s171g0 --sub 171 --gate none
