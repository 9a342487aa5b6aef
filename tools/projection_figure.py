#!/usr/bin/env python3
"""Compute-only strong-scaling projection of the 512³ K=20 solve from one-GPU measurements.

    python tools/projection_figure.py gpurun_out/fakesweep.jsonl [--plot profiles/figs/gpu_compute_projection.png]

Input: the JSON lines of ``scripts/gpu.sh fakesweep`` — the 1-GPU solve, and one rank of P timed alone with
``--fake-rank r/P`` (its real box, ghosts and passes, no transport traffic) for the sequential slab and block schedules.
A point's time is the max over the sampled ranks; each P keeps its fastest schedule.

This prices the compute side of a multi-GPU solve only: the halo traffic over xGMI (and the overlap that hides part of
it) is not in it, so the numbers are an upper bound on what an 8-GPU node can reach, not a measurement of one.
Schedules whose name contains "sdma" (round 4) are fake ranks WITH their copy-engine traffic (mean of the timed
solves): every message of the rank goes through this one GPU's SDMA engines, where a node gives each neighbour link
its own — a pessimistic bracket. They form a second curve and never enter the compute-only one. The
measured curve comes from the driver's SCALE records (tools/scaling_report.py). The panels mirror the reference's
speedup / efficiency figure (readme.md:102-108, iamge1.png).
"""
from __future__ import annotations

import argparse
import json
from collections import defaultdict

CELLS = 512 ** 3 * 20
REF_S = {1: 0.752, 2: 0.505}  # the reference's P100 total times (readme.md:99-100)


def load(path):
    pts = defaultdict(dict)  # P -> schedule -> max over ranks of solve_s
    for line in open(path):
        line = line.strip()
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        sched = d.get("schedule", "single")
        pts[d["P"]][sched] = max(pts[d["P"]].get(sched, 0.0), float(d["solve_s"]))
    return pts


def _kind(sched: str) -> str:
    return "sdma" if "sdma" in sched else "rccl" if "traffic" in sched else ""


def table(pts, traffic=False):
    """Fastest schedule per P among the compute-only ones (traffic falsy), the copy-engine ones (True or "sdma") or the
    ones with their RCCL messages sent to themselves ("rccl", round 5 --fake-traffic); P = 1 is the one-GPU solve."""
    want = "sdma" if traffic is True else (traffic or "")
    t1 = min(v for k, v in pts[1].items() if not _kind(k))
    rows = []
    for P in sorted(pts):
        cand = {k: v for k, v in pts[P].items() if P == 1 or _kind(k) == want}
        if not cand:
            continue
        sched, t = min(cand.items(), key=lambda kv: kv[1])
        rows.append({"P": P, "schedule": sched, "t": t, "gcell": CELLS / t / 1e9, "speedup": t1 / t,
                     "eff": t1 / t / P, "all": dict(sorted(cand.items()))})
    return rows


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("path")
    ap.add_argument("--plot", default="")
    a = ap.parse_args(argv)
    pts = load(a.path)
    rows = table(pts)
    trows = table(pts, traffic=True)
    trows = trows if len(trows) > 1 else []
    rrows = table(pts, traffic="rccl")
    rrows = rrows if len(rrows) > 1 else []
    for title, rr in (("compute only", rows), ("with copy-engine traffic on one GPU's engines", trows),
                      ("with the rank's RCCL messages sent to itself (--fake-traffic; no xGMI hop)", rrows)):
        if not rr:
            continue
        print(f"\n{title}\n")
        print("| GPUs | fastest schedule | per-rank ms | GCell/s | speedup | efficiency | schedules (ms) | P100 reference |")
        print("|---|---|---|---|---|---|---|---|")
        for r in rr:
            alls = ", ".join(f"{k} {v * 1e3:.3f}" for k, v in r["all"].items())
            ref = f"{REF_S[r['P']]} s" if r["P"] in REF_S else "—"
            print(f"| {r['P']} | {r['schedule']} | {r['t'] * 1e3:.3f} | {r['gcell']:.0f} | {r['speedup']:.2f} | "
                  f"{r['eff']:.2f} | {alls} | {ref} |")
    if a.plot:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        ps = [r["P"] for r in rows]
        fig, (a1, a2) = plt.subplots(1, 2, figsize=(11, 4.2))
        a1.plot(ps, [r["speedup"] for r in rows], "o-", label="MI355X, per-rank compute (fake rank, no traffic)")
        if trows:
            a1.plot([r["P"] for r in trows], [r["speedup"] for r in trows], "^-",
                    label="MI355X, fake rank + its copy-engine traffic (one GPU's engines)")
        if rrows:
            a1.plot([r["P"] for r in rrows], [r["speedup"] for r in rrows], "v-",
                    label="MI355X, fake rank + its RCCL messages to itself")
        a1.plot([1, ps[-1]], [1, ps[-1]], ":", color="gray", label="ideal")
        a1.plot(list(REF_S), [REF_S[1] / REF_S[p] for p in REF_S], "s--", label="P100 reference (readme.md:99-100)")
        a1.set_xlabel("GPUs")
        a1.set_ylabel("speedup vs 1 GPU")
        a1.set_title("512³ K=20 fp64: one-GPU projection")
        a1.legend(fontsize=8)
        a2.plot(ps, [r["eff"] for r in rows], "o-", label="MI355X, per-rank compute")
        if trows:
            a2.plot([r["P"] for r in trows], [r["eff"] for r in trows], "^-", label="MI355X, + copy-engine traffic")
        if rrows:
            a2.plot([r["P"] for r in rrows], [r["eff"] for r in rrows], "v-", label="MI355X, + RCCL self-traffic")
        a2.plot(list(REF_S), [REF_S[1] / REF_S[p] / p for p in REF_S], "s--", label="P100 reference")
        a2.set_xlabel("GPUs")
        a2.set_ylabel("efficiency")
        a2.set_ylim(0, 1.1)
        a2.set_title("not a multi-GPU measurement: halo traffic excluded")
        a2.legend(fontsize=8)
        fig.tight_layout()
        fig.savefig(a.plot, dpi=110)
        print(f"\nfigure: {a.plot}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
