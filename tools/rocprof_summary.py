#!/usr/bin/env python3
"""Summarise a rocprofv3 run (rocpd SQLite ``*_results.db`` or ``*_kernel_stats.csv``) into a markdown table.

    python tools/rocprof_summary.py gpurun_out/prof/run_results.db [--bytes-per-node 24 --nodes 511**3] > profiles/x.md

With --bytes-per-node/--nodes the leapfrog rows also get an effective-bandwidth column (compulsory bytes / kernel time).
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import sqlite3
import sys


def from_db(path: str):
    c = sqlite3.connect(path)
    q = ("select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
         "max(grid_x*grid_y*grid_z/(workgroup_x*workgroup_y*workgroup_z)), max(workgroup_x*workgroup_y*workgroup_z), "
         "max(vgpr_count), max(sgpr_count), max(lds_size), max(scratch_size) from kernels group by name "
         "order by sum(duration) desc")
    return [dict(name=r[0], calls=r[1], total_ns=r[2], avg_ns=r[3], min_ns=r[4], max_ns=r[5], wgs=r[6], wg=r[7],
                 vgpr=r[8], sgpr=r[9], lds=r[10], scratch=r[11]) for r in c.execute(q)]


def from_csv(path: str):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append(dict(name=r["Name"], calls=int(r["Calls"]), total_ns=float(r["TotalDurationNs"]),
                             avg_ns=float(r["AverageNs"]), min_ns=float(r["MinNs"]), max_ns=float(r["MaxNs"])))
    return rows


def short(name: str) -> str:
    n = name.replace("wave3d::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0] if "(" in n and not n.startswith("void") else n.split("(wave3d")[0].replace("void ", "")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--bytes-per-node", type=float, default=0.0)
    ap.add_argument("--nodes", type=str, default="0")
    ap.add_argument("--match", default="leapfrog")
    a = ap.parse_args()
    p = a.path
    if os.path.isdir(p):
        cands = glob.glob(os.path.join(p, "**", "*results.db"), recursive=True) or \
            glob.glob(os.path.join(p, "**", "*kernel_stats.csv"), recursive=True)
        p = cands[0]
    rows = from_db(p) if p.endswith(".db") else from_csv(p)
    nodes = float(eval(a.nodes, {"__builtins__": {}}))  # e.g. 511**3
    total = sum(r["total_ns"] for r in rows)
    print(f"source: `{os.path.basename(p)}`  total kernel time {total / 1e6:.3f} ms\n")
    hdr = "| kernel | calls | total ms | avg µs | min µs | max µs | % | WGs | WG size | VGPR | LDS B | scratch |"
    if a.bytes_per_node and nodes:
        hdr += " eff. TB/s (avg) |"
    print(hdr)
    print("|" + "---|" * (hdr.count("|") - 1))
    for r in rows:
        line = (f"| `{short(r['name'])}` | {r['calls']} | {r['total_ns'] / 1e6:.3f} | {r['avg_ns'] / 1e3:.1f} | "
                f"{r['min_ns'] / 1e3:.1f} | {r['max_ns'] / 1e3:.1f} | {100 * r['total_ns'] / total:.1f} | "
                f"{r.get('wgs', '')} | {r.get('wg', '')} | {r.get('vgpr', '')} | {r.get('lds', '')} | "
                f"{r.get('scratch', '')} |")
        if a.bytes_per_node and nodes:
            bw = a.bytes_per_node * nodes / (r["avg_ns"] * 1e-9) / 1e12 if a.match in r["name"] else float("nan")
            line += f" {bw:.2f} |" if bw == bw else " |"
        print(line)
    return 0


if __name__ == "__main__":
    sys.exit(main())
