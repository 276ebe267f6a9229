#!/usr/bin/env python3
"""Per-launch HBM traffic of each kernel from two rocprofv3 PMC passes.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run -- python3 bench.py ...
    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write \
        --config C3 --batch 1024 --out profiles/traffic.json

FETCH_SIZE and WRITE_SIZE are kilobytes (1024 B) per dispatch.  gfx950
correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the
bytes of wide coalesced streaming reads, so it is doubled; WRITE_SIZE is exact
for 16-B-per-lane streaming stores.  Both passes must run the same workload.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def read_counter(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    per = defaultdict(list)
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                name = row["Kernel_Name"]
                if name.startswith("void "):
                    name = name[5:]
                per[name].append(float(row["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--config", required=True)
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch = read_counter(a.fetch_dir, "FETCH_SIZE")
    write = read_counter(a.write_dir, "WRITE_SIZE")
    kernels = {}
    for name in sorted(set(fetch) | set(write)):
        if name.startswith("__amd_rocclr"):
            continue
        f = fetch.get(name, [])
        w = write.get(name, [])
        fk = sum(f) / len(f) if f else None
        wk = sum(w) / len(w) if w else None
        rec = {"launches_fetch_pass": len(f), "launches_write_pass": len(w),
               "fetch_size_kb": fk, "write_size_kb": wk}
        if fk is not None and wk is not None:
            rec["read_bytes"] = 2.0 * fk * 1024.0      # gfx950: FETCH_SIZE x2
            rec["write_bytes"] = wk * 1024.0
            rec["hbm_bytes_per_launch"] = rec["read_bytes"] + rec["write_bytes"]
        kernels[name] = rec
    out = {"config": a.config, "batch": a.batch,
           "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count), write = WRITE_SIZE KiB",
           "kernels": kernels}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, r in kernels.items():
        print(f"{r.get('hbm_bytes_per_launch', 0) / 1e6:12.1f} MB/launch  {k[:90]}")


if __name__ == "__main__":
    main()
