#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc CSV output (run_counter_collection.csv of one or more runs) per kernel: mean counter
value per dispatch, plus derived ratios. Usage: python tools/pmc_summary.py gpurun_out/pmc/*/run_counter_collection.csv"""
import collections
import csv
import glob
import os
import re
import sys


def short(name: str) -> str:
    n = name.replace("void ", "")
    for ns in ("wave3d::(anonymous namespace)::", "wave3d::tbk::", "wave3d::p2k::", "wave3d::"):
        n = n.replace(ns, "")
    m = re.match(r"([A-Za-z_0-9]+(<[^>]*>)?)", n)
    return m.group(1) if m else n[:60]


def expand(paths):
    """Files as given; a directory stands for every *counter_collection.csv below it (rocprofv3 -d DIR)."""
    out = []
    for p in paths:
        if os.path.isdir(p):
            out += sorted(glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True))
        else:
            out.append(p)
    if not out:
        raise SystemExit(f"pmc_summary: no counter_collection.csv under {paths}")
    return out


def main(paths):
    paths = expand(paths)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k].append((float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3)
    print("| kernel | counter | mean per dispatch |")
    print("|---|---|---|")
    for k in sorted(agg):
        if k.startswith("__amd"):
            continue
        for c, v in sorted(agg[k].items()):
            print(f"| `{k}` | {c} | {sum(v) / len(v):.4g} |")
        a = {c: sum(v) / len(v) for c, v in agg[k].items()}
        if "SQ_WAVE_CYCLES" in a and a["SQ_WAVE_CYCLES"]:
            w = a["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in a:
                    print(f"| `{k}` | {c} / WAVE_CYCLES | {a[c] / w:.3f} |")
        if "TCC_HIT_sum" in a and "TCC_MISS_sum" in a:
            print(f"| `{k}` | L2 hit rate | {a['TCC_HIT_sum'] / (a['TCC_HIT_sum'] + a['TCC_MISS_sum']):.3f} |")
        print(f"| `{k}` | mean dispatch µs (under profiler) | {sum(dur[k]) / len(dur[k]):.1f} |")


if __name__ == "__main__":
    main(sys.argv[1:])
