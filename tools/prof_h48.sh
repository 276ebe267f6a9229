#!/bin/bash
# GPU box: H48 kernel trace (per-batch launches and their durations in the timed region)
set -o pipefail
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r06y}
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${tag}_H48" -o run -- \
  python3 "$R/bench.py" --config H48 --no-cpu --iso-steps 0 --points= --fir-points= --steps 20 --from-dicts-steps 0 \
  > "$R/gpurun_out/${tag}_H48_bench.json" 2> "$R/gpurun_out/${tag}_H48.log" || exit $?
cd "$R"
python3 - "$tag" <<'PY'
import csv, glob, json, sys
tag = sys.argv[1]
d = json.load(open(f"gpurun_out/{tag}_H48_bench.json"))
print("H48 step", d["ms_per_step"])
f = glob.glob(f"gpurun_out/{tag}_H48/**/*kernel_stats.csv", recursive=True)[0]
tot = 0
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"])):
    print("  %-60s %6s %9.4f %9.4f %5.1f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["MinNs"]) / 1e6, float(r["Percentage"])))
PY
