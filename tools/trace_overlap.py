#!/usr/bin/env python3
"""Overlap of halo copies with the LDS passes in a rocprofv3 trace (--kernel-trace --memory-copy-trace, CSV).

For the copy-engine ("sdma") transport the halo regions move as hipMemcpyDeviceToDeviceNoCU copies; this tool reports,
from the trace of a run, how much of the copy time ran while a k_leapfrog_tb pass was on the GPU (the point of the
transport: no compute unit is taken from the pass), and a per-kind time table.

    python tools/trace_overlap.py gpurun_out/trace_sdma        # a rocprofv3 -d directory (searched recursively)
"""
from __future__ import annotations

import csv
import glob
import os
import re
import sys
from collections import defaultdict


def _rows(d: str, suffix: str) -> list[dict]:
    out = []
    for p in sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def _short(name: str) -> str:
    n = name.replace("wave3d::(anonymous namespace)::", "").replace("wave3d::", "").replace("void ", "")
    m = re.match(r"([A-Za-z_0-9:]+)(<[^>]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:60]


def _merge(iv: list[tuple[int, int]]) -> list[tuple[int, int]]:
    out: list[tuple[int, int]] = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], b))
        else:
            out.append((a, b))
    return out


def _overlap(a: tuple[int, int], merged: list[tuple[int, int]]) -> int:
    s = 0
    for x, y in merged:
        lo, hi = max(a[0], x), min(a[1], y)
        if hi > lo:
            s += hi - lo
    return s


def analyse(d: str) -> dict:
    kern = _rows(d, "kernel_trace.csv")
    copies = _rows(d, "memory_copy_trace.csv")
    passes = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kern if "k_leapfrog_tb" in r["Kernel_Name"]]
    merged = _merge(passes)
    per_kind = defaultdict(lambda: [0, 0])
    for r in kern:
        k = _short(r["Kernel_Name"])
        per_kind[k][0] += 1
        per_kind[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot = ov = 0
    nbytes = 0
    for r in copies:
        a = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        tot += a[1] - a[0]
        ov += _overlap(a, merged)
        nbytes += int(r.get("Bytes", 0) or 0)
        k = "copy " + r.get("Direction", "?")
        per_kind[k][0] += 1
        per_kind[k][1] += a[1] - a[0]
    return {"copies": len(copies), "copy_ns": tot, "copy_ns_during_pass": ov, "copy_bytes": nbytes,
            "pass_ns": sum(b - a for a, b in merged), "per_kind": dict(per_kind)}


def main(argv: list[str]) -> int:
    if not argv:
        print(__doc__)
        return 2
    r = analyse(argv[0])
    print(f"| item | value |\n|---|---|")
    print(f"| memory copies | {r['copies']} ({r['copy_bytes'] / 1e6:.1f} MB) |")
    print(f"| copy time | {r['copy_ns'] / 1e6:.3f} ms |")
    frac = r["copy_ns_during_pass"] / r["copy_ns"] if r["copy_ns"] else 0.0
    print(f"| copy time while a k_leapfrog_tb pass ran | {r['copy_ns_during_pass'] / 1e6:.3f} ms ({100 * frac:.1f} %) |")
    print(f"| k_leapfrog_tb busy time (union) | {r['pass_ns'] / 1e6:.3f} ms |")
    print("\n| kind | count | total ms |\n|---|---|---|")
    for k, (n, t) in sorted(r["per_kind"].items(), key=lambda kv: -kv[1][1]):
        print(f"| `{k}` | {n} | {t / 1e6:.3f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
