#!/bin/bash
# same-box kernel durations of two libraries (rocprofv3 kernel stats of the C3 bench)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
for lib in base old base2 old2; do
  case $lib in base*) unset MSGPU_LIB ;; *) export MSGPU_LIB=$R/audio-suite_amd/msgpu/libmsgpu_old.so ;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/r05s_$lib" -o run -- \
      python3 "$R/bench.py" --no-cpu --points= --steps 20 --from-dicts-steps 0 > "$O/r05s_$lib.json" 2> "$O/r05s_$lib.log" || exit $?
  f=$(ls "$O"/r05s_$lib/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find "$O/r05s_$lib" -name "*kernel_stats.csv" | head -1)
  echo "== $lib"; python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print(f"{r['Name'][:40]:40s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.1f} pct {float(r['Percentage']):5.1f}")
PY
done
