#!/bin/bash
# GPU box: rocprofv3 kernel stats and HBM traffic (two PMC passes) of the
# standalone FIR at 16 k and 64 k taps (tools/fir_bench.py: 1024 signals of
# 384 000 samples, the SURVEY 8(d) taps) under gpurun_out/<tag>_fir_*.
#   usage (on the box): bash tools/prof_fir.sh TAG
set -e
tag=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${tag}_fir_prof" -o run -- \
    python3 "$R/tools/fir_bench.py" --taps 16384,65536 --steps 10 > "$O/${tag}_fir_bench.jsonl" 2> "$O/${tag}_fir_prof.log"
for k in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $k --output-format csv -d "$O/${tag}_fir_pmc_$k" -o run -- \
      python3 "$R/tools/fir_bench.py" --taps 16384,65536 --steps 2 --warmup 1 > "$O/${tag}_fir_pmc_$k.log" 2>&1
done
cd "$R"
python3 tools/pmc_traffic.py "$O/${tag}_fir_pmc_FETCH_SIZE" "$O/${tag}_fir_pmc_WRITE_SIZE" --config FIR \
    --batch 1024 --out "$O/${tag}_traffic_FIR.json"
python3 - "$O" "$tag" <<'PY'
import csv, glob, json, sys
O, tag = sys.argv[1:3]
f = glob.glob(f"{O}/{tag}_fir_prof/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print("  ", r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e6, 4), "ms avg")
t = json.load(open(f"{O}/{tag}_traffic_FIR.json"))
for k, v in t["kernels"].items():
    print("  traffic", k[:60], v.get("hbm_bytes_per_launch"))
PY
