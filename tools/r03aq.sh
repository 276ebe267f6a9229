#!/bin/bash
# GPU box: rocprofv3 kernel stats of the C4 and C5 bench configurations (the
# DESIGN section 4 table), each run's own bench line beside it.
set -o pipefail
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in C4 C5; do
  steps=10; [ $c = C5 ] && steps=3
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r03aq_$c" -o run -- \
      python3 "$R/bench.py" --config $c --no-cpu --iso-steps 0 --points= --steps $steps > "$R/gpurun_out/r03aq_${c}_bench.json" 2> "$R/gpurun_out/r03aq_$c.log") || exit $?
  python3 - $c <<'PY'
import csv, glob, json, sys
c = sys.argv[1]
d = json.load(open(f"gpurun_out/r03aq_{c}_bench.json"))
print(c, "step", d["ms_per_step"], "value", round(d["value"]), "ok", d["checked"]["all_ok"], "sub", d["config"].get("sub_batches_per_gpu"))
f = glob.glob(f"gpurun_out/r03aq_{c}/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print("  ", r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), round(float(r["Percentage"]), 1))
PY
done
