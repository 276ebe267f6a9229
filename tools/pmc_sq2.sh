#!/bin/bash
# Two SQ counter passes (<= 8 SQ counters each) over a short C3 bench, one stream.
#   usage (on the box): bash tools/pmc_sq2.sh TAG [bench args...]
set -e
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
    --output-format csv -d "$O/${tag}_sqA" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --iso-steps 0 --points= --streams 1 "$@" > "$O/${tag}_sqA.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU \
    --output-format csv -d "$O/${tag}_sqB" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --iso-steps 0 --points= --streams 1 "$@" > "$O/${tag}_sqB.log" 2>&1
cd "$R"
python3 tools/pmc_summary.py "$O/${tag}_sqA" "$O/${tag}_sqB" > "$O/${tag}_sq_summary.txt" 2>&1 || true
