#!/usr/bin/env python3
"""Per-rank solve times of the Python Solver(runtime="process") against the native CLI.

Run under torch.distributed.run (gloo for the rendezvous); every rank builds Solver(..., runtime="process") — its
production GpuSolver in a bin/wave3d --serve child — and times REPS solves after WARM warmups; rank 0 prints one JSON
line with the per-solve times (max over ranks) and whether the solves were graph-captured.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/proc_runtime_bench.py \\
        --N 512 --transport sdma --no-rccl --reps 20 --warmup 8
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch.distributed as dist

    from mpi_cuda_amd import ProblemSpec
    from mpi_cuda_amd.solver import Solver

    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=512)
    ap.add_argument("--tau", type=float, default=1e-3)
    ap.add_argument("--K", type=int, default=20)
    ap.add_argument("--transport", default="sdma")
    ap.add_argument("--decomp", default="slab")
    ap.add_argument("--no-rccl", action="store_true")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    a = ap.parse_args()
    dist.init_process_group("gloo")
    s = Solver(ProblemSpec(N=a.N, tau=a.tau, K=a.K), backend="hip", transport=a.transport, decomp=a.decomp,
               device=0 if a.no_rccl else None, rccl=not a.no_rccl, overlap=not a.no_overlap, runtime="process")
    rs = [s.run() for _ in range(a.warmup + a.reps)][a.warmup:]
    t = [r.solve_s for r in rs]
    if dist.get_rank() == 0:
        print(json.dumps({"runtime": "process", "N": a.N, "world": s.world, "transport": s.transport,
                          "schedule": s.schedule, "graph": all(r.extra["graph"] for r in rs),
                          "best_s": min(t), "median_s": statistics.median(t), "mean_s": statistics.mean(t),
                          "final_max_err": rs[-1].max_err[-1]}), flush=True)
    s.close()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
