#!/bin/bash
# GPU box: the round's profile set under gpurun_out/<tag>_*:
#   C3   kernel stats + FETCH/WRITE traffic + bench/rocprof agreement (tools/profile.sh)
#   C3   SQ issue/stall counters, one stream (tools/pmc_sq.sh)
#   C4, C5 kernel stats of their own bench runs (the DESIGN section 4 table)
#   C5   FETCH/WRITE traffic per 171-preset launch
#   usage (on the box): bash tools/prof_round.sh TAG
set -o pipefail
tag=${1:-r04p}
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/profile.sh "$tag" || exit $?
bash tools/pmc_sq.sh "$tag" || exit $?
for c in C4 C5; do
  steps=10; [ $c = C5 ] && steps=3
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${tag}_$c" -o run -- \
      python3 "$R/bench.py" --config $c --no-cpu --iso-steps 0 --points= --fir-points= --steps $steps \
      > "$R/gpurun_out/${tag}_${c}_bench.json" 2> "$R/gpurun_out/${tag}_$c.log") || exit $?
  python3 - "$tag" $c <<'PY'
import csv, glob, json, sys
tag, c = sys.argv[1:3]
d = json.load(open(f"gpurun_out/{tag}_{c}_bench.json"))
print(c, "step", d["ms_per_step"], "value", round(d["value"]), "ok", d["checked"]["all_ok"], "sub", d["config"].get("sub_batches_per_gpu"))
f = glob.glob(f"gpurun_out/{tag}_{c}/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    print("  ", r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), round(float(r["Percentage"]), 1))
PY
done
cd /tmp
for k in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $k --output-format csv -d "$R/gpurun_out/${tag}_C5_pmc_$k" -o run -- \
      python3 "$R/bench.py" --config C5 --steps 1 --warmup 1 --no-cpu --iso-steps 0 --points= --fir-points= \
      > "$R/gpurun_out/${tag}_C5_pmc_$k.log" 2>&1 || exit $?
done
cd "$R"
python3 tools/pmc_traffic.py "gpurun_out/${tag}_C5_pmc_FETCH_SIZE" "gpurun_out/${tag}_C5_pmc_WRITE_SIZE" --config C5 \
    --batch 171 --out "gpurun_out/${tag}_traffic_C5.json"
echo "== C3 agree"; cat "gpurun_out/${tag}_agree.txt" | tail -12
echo "== SQ"; tail -20 "gpurun_out/${tag}_sq_summary.txt"
