#!/usr/bin/env python3
"""GPU robustness sweep: every (N, L, tau, K, check_every, temporal) below solved on the GPU and compared with the
closed-form oracle (models/wave3d.py::oracle_errors) and with the CPU solver (bit-exact errors).

    python tools/oracle_sweep.py [--json out.jsonl]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mpi_cuda_amd import ProblemSpec  # noqa: E402
from mpi_cuda_amd.models.wave3d import oracle_errors  # noqa: E402
from mpi_cuda_amd.solver import Solver  # noqa: E402

CASES = [
    # N, L, tau, K, check_every, temporal
    (64, 1.0, 1e-3, 1, 1, 4), (64, 1.0, 1e-3, 2, 1, 4), (64, 1.0, 1e-3, 3, 1, 4), (65, 1.0, 1e-3, 7, 3, 4),
    (100, math.pi, 1e-3, 20, 2, 4), (127, 1.0, 1e-3, 50, 2, 4), (128, 1.0, 1e-3, 50, 0, 3), (129, 1.0, 1e-3, 33, 5, 2),
    (257, 1.0, 1e-3, 20, 2, 4), (300, math.pi, 2e-3, 41, 4, 4), (512, 1.0, 1e-3, 20, 2, 4), (640, 1.0, 5e-4, 24, 2, 4),
]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    bad = 0
    out = []
    for N, L, tau, K, ce, temporal in CASES:
        spec = ProblemSpec(N=N, tau=tau, K=K, L=L, check_every=ce)
        r = Solver(spec, backend="hip", device=0, temporal=temporal).run()
        ref = oracle_errors(spec)
        worst = 0.0
        for n, m, e in zip(r.steps, r.max_err, r.rms_err):
            om, oe = ref[n]
            worst = max(worst, abs(m - om) / om, abs(e - oe) / oe)
        cpu = Solver(spec, backend="cpu").run() if N <= 300 else None
        exact = cpu is None or (cpu.max_err == r.max_err and all(
            math.isclose(x, y, rel_tol=1e-12) for x, y in zip(cpu.rms_err, r.rms_err)))
        ok = r.finite and worst < 1e-4 and exact and r.steps == [n for n in range(1, K + 1)
                                                              if (ce and n % ce == 0) or n == K]
        bad += not ok
        row = dict(N=N, L=round(L, 6), tau=tau, K=K, check_every=ce, temporal=temporal, steps=len(r.steps),
                   oracle_rel=worst, cpu_bitexact=None if cpu is None else exact, ok=ok, solve_ms=r.solve_s * 1e3)
        out.append(row)
        print(json.dumps(row), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            f.write("\n".join(json.dumps(r) for r in out) + "\n")
    print("FAILED" if bad else "all ok", bad)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
