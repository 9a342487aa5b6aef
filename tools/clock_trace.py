#!/usr/bin/env python3
"""Per-dispatch clock of the LDS passes from one rocprofv3 --pmc run that collected GRBM_GUI_ACTIVE (GPU-active
cycles) and SQ_BUSY_CU_CYCLES: cycles / dispatch duration = the clock the chip held during that dispatch.

Shows the warm-up transient of a run of back-to-back 512³ solves (the analytic-start pass is compute-bound, so its
time follows the clock the power controller grants; the 5-step passes are memory-bound and move less).

Usage: python tools/clock_trace.py gpurun_out/clk [--cus 256] [--md]
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import re


def short(name: str) -> str:
    m = re.search(r"k_(\w+)<([^>]*)>", name)
    if m:
        return f"{m.group(1)}<{m.group(2).replace(' ', '')}>"
    return name.split("(")[0][-40:]


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("path")
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--md", action="store_true", help="markdown table")
    a = ap.parse_args()
    files = [a.path] if os.path.isfile(a.path) else sorted(
        glob.glob(os.path.join(a.path, "**", "*counter_collection.csv"), recursive=True))
    disp = collections.OrderedDict()
    for f in files:
        for r in csv.DictReader(open(f)):
            if "leapfrog" not in r["Kernel_Name"]:
                continue
            key = (f, r["Dispatch_Id"])
            d = disp.setdefault(key, {"name": short(r["Kernel_Name"]), "start": int(r["Start_Timestamp"]),
                                      "dur_us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
            d[r["Counter_Name"]] = float(r["Counter_Value"])
    rows = sorted(disp.values(), key=lambda d: d["start"])
    if a.md:
        print("| # | pass | µs | GRBM_GUI_ACTIVE MHz | CU-busy MHz |")
        print("|---|---|---|---|---|")
    for i, d in enumerate(rows):
        dur = d["dur_us"]
        gui = d.get("GRBM_GUI_ACTIVE", 0.0) / dur if dur else 0.0
        cu = d.get("SQ_BUSY_CU_CYCLES", 0.0) / a.cus / dur if dur else 0.0
        if a.md:
            print(f"| {i} | `{d['name']}` | {dur:.1f} | {gui:.0f} | {cu:.0f} |")
        else:
            print(f"{i:3d} {d['name']:34s} {dur:8.1f} us  gui {gui:6.0f} MHz  cu-busy {cu:6.0f} MHz")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
