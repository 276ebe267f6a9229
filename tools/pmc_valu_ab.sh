#!/bin/bash
# SQ_INSTS_VALU / SQ_INSTS_SALU / SQ_WAVES of the bench kernels for the product
# library and tuning builds (one PMC pass each, single stream).
#   usage (on the box): bash tools/pmc_valu_ab.sh base NAME [...]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" != base ]; then export MSGPU_LIB=$R/audio-suite_amd/msgpu/libmsgpu_$v.so; else unset MSGPU_LIB; fi
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES \
      --output-format csv -d "$O/valu_$v" -o run -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --iso-steps 0 --points= --streams 1 > "$O/valu_$v.log" 2>&1
  cd "$R"
  echo "== $v"; python3 tools/pmc_summary.py "$O/valu_$v" 2>&1 | grep -A6 "k_gen_normal<false>" | grep -E "k_gen|INSTS|WAVES|per wave"
done
