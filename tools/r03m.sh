#!/bin/bash
# GPU box: standalone FIR bench (msg_fir on k_fir8 / k_fir4 / k_fir2 / delay line) and its kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/fir_bench.py --cpu > gpurun_out/r03m_fir_bench.jsonl || exit $?
cat gpurun_out/r03m_fir_bench.jsonl
R=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r03m_fir_prof" -o run -- \
   python3 "$R/tools/fir_bench.py" --steps 3 > "$R/gpurun_out/r03m_fir_prof.log" 2>&1 || exit $?
cd "$R"
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r03m_fir_prof/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e6, 4))
PY
