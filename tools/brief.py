#!/usr/bin/env python3
"""One-line summary of a bench JSON line (C3 step, stage windows, isolated stages, points)."""
import json
import sys

try:
    d = json.load(open(sys.argv[1]))
except Exception as e:  # noqa: BLE001
    print("no line:", e)
    sys.exit(0)
K = ("generate", "spectral", "overlap_add", "fir_kernel", "fir_h", "stereo", "total")
print("step", d["ms_per_step"], "value", d["value"], "ok", (d.get("checked") or {}).get("all_ok"))
print("  timed", {k: d["stage_ms"].get(k) for k in K})
i = d.get("roofline_isolated") or {}
print("  iso  ", {k: (i.get("stage_ms") or {}).get(k) for k in K}, "frac", i.get("kernels_frac"))
for k, v in (d.get("points") or {}).items():
    iso = (v.get("roofline_isolated") or {}).get("stage_ms") or {}
    print(" ", k, "step", v["ms_per_step"], "value", v["value"], "ok", (v.get("check") or {}).get("all_ok"),
          "iso", {a: iso.get(a) for a in K})
