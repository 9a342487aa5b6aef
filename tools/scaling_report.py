#!/usr/bin/env python3
"""Markdown speedup / efficiency table (and optional figure) from JSON lines written by bench.py (--out) or
scripts/run_cpu_sweep.sh.

Conventions follow the reference (readme.md:84-114): S = T_1 / T_p, E = S / p with p the number of workers (GPUs,
threads or ranks). For bench.py lines the time is ms_per_step (one full 512^3 K=20 solve) and the reference's own
numbers (0.752 s / 0.505 s on P100) are shown next to ours.

    python tools/scaling_report.py results.jsonl [--plot fig.png]

--plot draws the reference's two panels (iamge1.png / report.pdf p.18 Fig. 4.1: speedup and efficiency against the
number of workers, one line per implementation); for bench.py lines it draws GCell/s and efficiency per GPU count with
the reference's P100 points for comparison.
"""
import argparse
import json
import sys
from collections import defaultdict

REF = {1: 0.752, 2: 0.505}
REF_GCELL = {p: 512**3 * 20 / t / 1e9 for p, t in REF.items()}


def _bench_records(obj, out):
    """Every bench.py line inside a (possibly nested) JSON object: the driver's SCALE_rNN.json / BENCH_rNN.json files
    wrap the lines (e.g. under "parsed"), a --out file holds them one per line."""
    if isinstance(obj, dict):
        if "n_gpus" in obj and "ms_per_step" in obj:
            out.append(obj)
            return
        for v in obj.values():
            _bench_records(v, out)
    elif isinstance(obj, list):
        for v in obj:
            _bench_records(v, out)


def load(path):
    text = open(path).read()
    try:  # one JSON document (driver records)
        doc = json.loads(text)
    except json.JSONDecodeError:
        doc = None
    if isinstance(doc, (dict, list)):
        rows = []
        _bench_records(doc, rows)
        if rows or isinstance(doc, list):
            return _dedupe(rows)
        return [doc] if "workers" in doc else []
    return [json.loads(l) for l in text.splitlines() if l.strip().startswith("{")]


def _dedupe(rows):
    """One line per GPU count (a driver record may repeat a line as "parsed" and inside "run"); the last wins."""
    by = {}
    for r in rows:
        by[(r.get("metric"), r["n_gpus"])] = r
    return list(by.values())


def gpu_rows(rows):
    base = next((r for r in rows if r["n_gpus"] == 1), rows[0])
    t1 = base["ms_per_step"] / 1e3
    out = []
    for r in sorted(rows, key=lambda r: r["n_gpus"]):
        p, t = r["n_gpus"], r["ms_per_step"] / 1e3
        out.append(dict(p=p, t=t, gcell=r["value"], speedup=t1 / t, eff=t1 / t / p, ref=REF.get(p)))
    return out


def cpu_groups(rows):
    """Per (mode, N): speedup against the sequential run of that N (the 1-thread OpenMP line; the reference divides
    every version by its sequential program's time, readme.md:86-100), else against the group's first point."""
    groups = defaultdict(list)
    seq = {}
    for r in rows:
        groups[(r.get("mode", "?"), r["N"])].append(r)
        if r.get("mode") == "openmp" and r["workers"] == 1:
            seq[r["N"]] = r["solve_s"]
    out = {}
    for key, rs in sorted(groups.items()):
        rs.sort(key=lambda r: r["workers"])
        t1 = seq.get(key[1], rs[0]["solve_s"] * rs[0]["workers"] if rs[0]["workers"] == 1 else rs[0]["solve_s"])
        out[key] = [dict(p=r["workers"], t=r["solve_s"], speedup=t1 / r["solve_s"],
                         eff=t1 / r["solve_s"] / r["workers"], gcell=r.get("gcell_per_s", 0.0)) for r in rs]
    return out


def print_tables(rows):
    if "ms_per_step" in rows[0]:
        print("| GPUs | wall-clock s | GCell/s | speedup | efficiency | reference (P100) s | vs reference |")
        print("|---|---|---|---|---|---|---|")
        for g in gpu_rows(rows):
            ref = g["ref"]
            vs = f"{ref / g['t']:.1f}x" if ref else "—"
            print(f"| {g['p']} | {g['t']:.5f} | {g['gcell']:.1f} | {g['speedup']:.2f} | {g['eff']:.2f} | "
                  f"{ref if ref else '—'} | {vs} |")
        ph = [r for r in sorted(rows, key=lambda r: r["n_gpus"]) if r.get("phases_ms")]
        if ph:  # the reference's per-GPU-count time breakdown (report.pdf p.16 §4.4: compute / copies / MPI)
            print("\nPhase breakdown (device ms per solve, max over ranks, traced solve of the timed schedule; exchange "
                  "overlaps compute when the schedule overlaps):\n")
            print("| GPUs | schedule | compute | of which shells | exchange | error check | error-log gather |")
            print("|---|---|---|---|---|---|---|")
            for r in ph:
                p = r["phases_ms"]
                print(f"| {r['n_gpus']} | {r.get('config', {}).get('schedule', '')} | {p.get('compute', 0):.3f} | "
                      f"{p.get('shell', 0):.3f} | {p.get('exchange', 0):.3f} | {p.get('check', 0):.3f} | "
                      f"{p.get('gather', p.get('gather_host', 0)):.3f} |")
        return
    for (mode, N), rs in cpu_groups(rows).items():
        print(f"\n{mode}, {N}^3:\n\n| workers | time s | speedup | efficiency | GCell/s |")
        print("|---|---|---|---|---|")
        for r in rs:
            print(f"| {r['p']} | {r['t']:.4f} | {r['speedup']:.2f} | {r['eff']:.2f} | {r['gcell']:.3f} |")


def plot(rows, path):
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    fig, (a1, a2) = plt.subplots(1, 2, figsize=(11, 4.2))
    if "ms_per_step" in rows[0]:
        g = gpu_rows(rows)
        ps = [r["p"] for r in g]
        a1.plot(ps, [r["gcell"] for r in g], "o-", label="MI355X (this framework)")
        a1.plot(list(REF_GCELL), list(REF_GCELL.values()), "s--", label="P100 reference (readme.md:99-100)")
        a1.set_yscale("log")
        a1.set_ylabel("GCell-updates/s (512³, K=20, fp64)")
        a2.plot(ps, [r["eff"] for r in g], "o-", label="MI355X strong-scaling efficiency")
        a2.axhline(1.0, color="gray", lw=0.5)
        a2.set_ylabel("efficiency  T₁ / (p·T_p)")
        for a in (a1, a2):
            a.set_xlabel("GPUs")
            a.set_xticks(ps)
    else:
        for (mode, N), rs in cpu_groups(rows).items():
            ps = [r["p"] for r in rs]
            a1.plot(ps, [r["speedup"] for r in rs], "o-", label=f"{mode} {N}³")
            a2.plot(ps, [r["eff"] for r in rs], "o-", label=f"{mode} {N}³")
        top = max(r["p"] for rs in cpu_groups(rows).values() for r in rs)
        a1.plot([1, top], [1, top], ":", color="gray", label="ideal")
        a1.set_ylabel("speedup  T₁ / T_p")
        a2.set_ylabel("efficiency  S / p")
        for a in (a1, a2):
            a.set_xlabel("workers (threads or ranks)")
    for a in (a1, a2):
        a.grid(alpha=0.3)
        a.legend(fontsize=8)
    fig.tight_layout()
    fig.savefig(path, dpi=110)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("path", nargs="?", default="scaling.jsonl")
    ap.add_argument("--plot", default="", help="also write the speedup / efficiency figure (PNG) here")
    a = ap.parse_args(argv)
    rows = load(a.path)
    if not rows:
        print("no rows")
        return 0
    print_tables(rows)
    if a.plot:
        plot(rows, a.plot)
        print(f"\nfigure: {a.plot}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
