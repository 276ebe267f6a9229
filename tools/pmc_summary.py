#!/usr/bin/env python3
"""Per-kernel mean of every PMC counter in rocprofv3 counter CSVs (any number of dirs).

    python tools/pmc_summary.py gpurun_out/pmcA gpurun_out/pmcB [--kernel k_fir2]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(list))
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
            for row in csv.DictReader(open(f, newline="")):
                k = row["Kernel_Name"]
                k = k[5:] if k.startswith("void ") else k
                if a.kernel and a.kernel not in k:
                    continue
                acc[k.split("(")[0]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        if k.startswith("__amd"):
            continue
        print(k)
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:16.1f}")
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            w = m["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if c in m:
                    print(f"   {c + '/WAVE_CYCLES':40s} {m[c] / w:8.3f}")
        if "SQ_WAVES" in m and "SQ_INSTS_VALU" in m:
            print(f"   VALU insts per wave {m['SQ_INSTS_VALU'] / m['SQ_WAVES']:.0f}")


if __name__ == "__main__":
    main()
