#!/bin/bash
# SQ stall/issue counters of the bench kernels (one PMC pass, <= 8 SQ counters).
#   usage (on the box): bash tools/pmc_sq.sh TAG [bench args...]
set -e
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    --output-format csv -d "$O/${tag}_sq" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --iso-steps 0 --points= --fir-points= --streams 1 "$@" > "$O/${tag}_sq.log" 2>&1
cd "$R"
python3 tools/pmc_summary.py "$O/${tag}_sq" > "$O/${tag}_sq_summary.txt" 2>&1 || true
