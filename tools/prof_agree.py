#!/usr/bin/env python3
"""Event-timed stage windows of a bench line against the rocprofv3 kernel averages
of the same run (tools/profile.sh).  Prints, per stage, the line's per-launch
window (ms) and the summed rocprof average of the stage's kernels (ms).

    python tools/prof_agree.py BENCH_LINE.json ROCPROF_DIR
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import STAGE_KERNEL  # noqa: E402


def main():
    line = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    f = glob.glob(os.path.join(sys.argv[2], "**", "*kernel_stats.csv"), recursive=True)[0]
    avg = {}
    for r in csv.DictReader(open(f)):
        name = r["Name"][5:] if r["Name"].startswith("void ") else r["Name"]
        avg[name] = (float(r["AverageNs"]) / 1e6, int(r["Calls"]))
    print(f"bench line: {line['ms_per_step']} ms/step, roofline kernel {line['roofline']['kernel']} "
          f"{line['roofline']['kernel_ms']} ms")
    print(f"{'stage':12s} {'event-timed ms':>15s} {'rocprof avg ms':>15s}  kernels (calls)")
    for stage, prefixes in STAGE_KERNEL.items():
        ks = [(n, a, c) for n, (a, c) in avg.items() if n.startswith(tuple(prefixes))]
        tot = sum(a for _, a, _ in ks)
        ev = line["stage_ms"].get(stage)
        print(f"{stage:12s} {ev if ev is not None else float('nan'):15.4f} {tot:15.4f}  "
              + ", ".join(f"{n.split('(')[0]} ({c})" for n, _, c in ks))


if __name__ == "__main__":
    main()
