#!/usr/bin/env python3
"""Overlap of halo copies with the LDS passes in a rocprofv3 trace (--kernel-trace --memory-copy-trace, CSV).

For the copy-engine ("sdma") transport the halo regions move as hipMemcpyDeviceToDeviceNoCU copies; this tool reports,
from the trace of a run, how much of the copy time ran while a k_leapfrog_tb pass was on the GPU (the point of the
transport: no compute unit is taken from the pass), and a per-kind time table.

    python tools/trace_overlap.py gpurun_out/trace_sdma        # a rocprofv3 -d directory (searched recursively)
    python tools/trace_overlap.py gpurun_out/trace_sdma --json run.json --solves 12

The memory-copy CSV of rocprofv3 (ROCm 7.2) carries no size column, so the copy volume comes from the solver's own
schedule: ``--json`` names the ``bin/wave3d --json`` output of the traced run (``halo_bytes`` = bytes this rank sends
per solve, GpuSolver::traffic) and ``--solves`` the number of solves in the trace (warmup included). A CSV that does
carry a size column (``Bytes`` / ``Size`` / ``Copy_Bytes``) is summed directly.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
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
    passes = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kern
              if "k_leapfrog_tb" in r["Kernel_Name"] or "k_leapfrog_p2" in r["Kernel_Name"]]
    merged = _merge(passes)
    # RCCL's own copy kernels (the rccl transport, or --fake-traffic): how much of their time ran beside a pass
    rccl = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kern if "nccl" in r["Kernel_Name"].lower()]
    rccl_ns = sum(b - a for a, b in rccl)
    rccl_ov = sum(_overlap(a, merged) for a in rccl)
    per_kind = defaultdict(lambda: [0, 0])
    for r in kern:
        k = _short(r["Kernel_Name"])
        per_kind[k][0] += 1
        per_kind[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot = ov = 0
    nbytes = 0
    size_key = next((k for k in ("Bytes", "Size", "Copy_Bytes") if copies and k in copies[0]), None)
    for r in copies:
        a = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        tot += a[1] - a[0]
        ov += _overlap(a, merged)
        if size_key:
            nbytes += int(r.get(size_key, 0) or 0)
        k = "copy " + r.get("Direction", "?")
        per_kind[k][0] += 1
        per_kind[k][1] += a[1] - a[0]
    return {"copies": len(copies), "copy_ns": tot, "copy_ns_during_pass": ov,
            "copy_bytes": nbytes if size_key else None,
            "pass_ns": sum(b - a for a, b in merged), "per_kind": dict(per_kind),
            "rccl_kernels": len(rccl), "rccl_ns": rccl_ns, "rccl_ns_during_pass": rccl_ov}


def copy_volume(r: dict, json_path: str | None, solves: int | None) -> str:
    """The copy-volume cell: bytes from the trace itself, else from the solver's schedule (--json/--solves)."""
    if r["copy_bytes"] is not None:
        return f"{r['copy_bytes'] / 1e6:.1f} MB (trace)"
    if json_path and solves:
        with open(json_path) as f:
            halo = float(json.load(f)["halo_bytes"])
        return f"{halo * solves / 1e6:.1f} MB ({solves} solves x {halo / 1e6:.2f} MB from the schedule)"
    return "size not in the trace (pass --json/--solves)"


def main(argv: list[str]) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("trace_dir")
    ap.add_argument("--json", help="bin/wave3d --json output of the traced run (halo_bytes per solve)")
    ap.add_argument("--solves", type=int, help="solves in the trace (warmup included)")
    a = ap.parse_args(argv)
    r = analyse(a.trace_dir)
    print(f"| item | value |\n|---|---|")
    print(f"| memory copies | {r['copies']} ({copy_volume(r, a.json, a.solves)}) |")
    print(f"| copy time | {r['copy_ns'] / 1e6:.3f} ms |")
    frac = r["copy_ns_during_pass"] / r["copy_ns"] if r["copy_ns"] else 0.0
    print(f"| copy time while a k_leapfrog_tb/p2 pass ran | {r['copy_ns_during_pass'] / 1e6:.3f} ms ({100 * frac:.1f} %) |")
    print(f"| k_leapfrog_tb/p2 busy time (union) | {r['pass_ns'] / 1e6:.3f} ms |")
    if r["rccl_kernels"]:
        rf = r["rccl_ns_during_pass"] / r["rccl_ns"] if r["rccl_ns"] else 0.0
        print(f"| RCCL kernels | {r['rccl_kernels']}, {r['rccl_ns'] / 1e6:.3f} ms |")
        print(f"| RCCL kernel time while a pass ran | {r['rccl_ns_during_pass'] / 1e6:.3f} ms ({100 * rf:.1f} %) |")
    print("\n| kind | count | total ms |\n|---|---|---|")
    for k, (n, t) in sorted(r["per_kind"].items(), key=lambda kv: -kv[1][1]):
        print(f"| `{k}` | {n} | {t / 1e6:.3f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
