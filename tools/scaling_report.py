#!/usr/bin/env python3
"""Markdown speedup / efficiency table from JSON lines written by bench.py (--out) or scripts/run_cpu_sweep.sh.

Conventions follow the reference (readme.md:84-114): S = T_1 / T_p, E = S / p with p the number of workers (GPUs,
threads or ranks). For bench.py lines the time is ms_per_step (one full 512^3 K=20 solve) and the reference's own
numbers (0.752 s / 0.505 s on P100) are shown next to ours.
"""
import json
import sys
from collections import defaultdict

REF = {1: 0.752, 2: 0.505}


def main(path):
    rows = [json.loads(l) for l in open(path) if l.strip().startswith("{")]
    if not rows:
        print("no rows")
        return 0
    if "ms_per_step" in rows[0]:
        base = next((r for r in rows if r["n_gpus"] == 1), rows[0])
        t1 = base["ms_per_step"] / 1e3
        print("| GPUs | wall-clock s | GCell/s | speedup | efficiency | reference (P100) s | vs reference |")
        print("|---|---|---|---|---|---|---|")
        for r in sorted(rows, key=lambda r: r["n_gpus"]):
            p, t = r["n_gpus"], r["ms_per_step"] / 1e3
            ref = REF.get(p)
            print(f"| {p} | {t:.5f} | {r['value']:.1f} | {t1 / t:.2f} | {t1 / t / p:.2f} | "
                  f"{ref if ref else '—'} | {f'{ref / t:.1f}x' if ref else '—'} |")
        return 0
    groups = defaultdict(list)
    for r in rows:
        groups[(r.get("mode", "?"), r["N"])].append(r)
    for (mode, N), rs in sorted(groups.items()):
        rs.sort(key=lambda r: r["workers"])
        t1 = rs[0]["solve_s"] * rs[0]["workers"] if rs[0]["workers"] == 1 else rs[0]["solve_s"]
        print(f"\n{mode}, {N}^3:\n\n| workers | time s | speedup | efficiency | GCell/s |")
        print("|---|---|---|---|---|")
        for r in rs:
            s = t1 / r["solve_s"]
            print(f"| {r['workers']} | {r['solve_s']:.4f} | {s:.2f} | {s / r['workers']:.2f} | "
                  f"{r.get('gcell_per_s', 0):.3f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "scaling.jsonl"))
