#!/bin/bash
# Profile the default bench workload on the gpurun box and leave the summaries
# under gpurun_out/<tag>_*:  kernel stats (rocprofv3 --kernel-trace --stats),
# two separate PMC passes (FETCH_SIZE, WRITE_SIZE) and the per-launch HBM
# traffic derived from them (tools/pmc_traffic.py).  The profiled launches are
# those of the timed region only (--iso-steps 0): BATCH = presets per launch
# (1024 presets on the default 2 streams -> 512).
#   usage (on the box): bash tools/profile.sh TAG [bench args...]
set -e
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${tag}_prof" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu --iso-steps 0 --points= "$@" > "$O/${tag}_prof.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/${tag}_pmc_fetch" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --iso-steps 0 --points= "$@" > "$O/${tag}_pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/${tag}_pmc_write" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --iso-steps 0 --points= "$@" > "$O/${tag}_pmc_write.log" 2>&1
cd "$R"
python3 tools/pmc_traffic.py "$O/${tag}_pmc_fetch" "$O/${tag}_pmc_write" --config "${CONFIG:-C3}" \
    --batch "${BATCH:-512}" --out "$O/${tag}_traffic.json"
