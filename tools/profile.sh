#!/bin/bash
# Profile the default bench workload on the gpurun box and leave the summaries
# under gpurun_out/<tag>_*:
#   * rocprofv3 --kernel-trace --stats of the bench command itself (C3 only, no
#     CPU baseline, no isolated pass: every launch is a timed-region sub-batch),
#     with that run's own bench line (<tag>_prof_bench.json), so the event-timed
#     stage windows in the line and the rocprof kernel averages come from the
#     same launches;
#   * two separate PMC passes (FETCH_SIZE, WRITE_SIZE) and the per-launch HBM
#     traffic derived from them (tools/pmc_traffic.py).
# BATCH = presets per launch (1024 presets on the default 3 streams -> 341).
#   usage (on the box): bash tools/profile.sh TAG [bench args...]
set -e
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${tag}_prof" -o run -- \
    python3 "$R/bench.py" --no-cpu --iso-steps 0 --points= --fir-points= "$@" > "$O/${tag}_prof_bench.json" 2> "$O/${tag}_prof.log"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/${tag}_pmc_fetch" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --iso-steps 0 --points= --fir-points= "$@" > "$O/${tag}_pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/${tag}_pmc_write" -o run -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --iso-steps 0 --points= --fir-points= "$@" > "$O/${tag}_pmc_write.log" 2>&1
cd "$R"
python3 tools/pmc_traffic.py "$O/${tag}_pmc_fetch" "$O/${tag}_pmc_write" --config "${CONFIG:-C3}" \
    --batch "${BATCH:-341}" --out "$O/${tag}_traffic.json"
python3 tools/prof_agree.py "$O/${tag}_prof_bench.json" "$O/${tag}_prof" > "$O/${tag}_agree.txt"
