"""Python CLI: ``python -m mpi_cuda_amd N tau K [L] [options]`` — same positional interface and output lines as the
reference programs (`wave`, `wave3dOMP`, `onlyMPI`, `mpiomp`, `mpigpu-1`; report.pdf p.15 §4.2.4, p.20-24 §5.x) and
as the native ``bin/wave3d``.

Launch several ranks with torchrun (the `mpirun -np P` analogue):

    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 -m mpi_cuda_amd 512 0.001 20 1              # 4 GPUs, RCCL
    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 -m mpi_cuda_amd 128 0.001 20 --backend cpu  # MPI analogue

``--checkpoint PREFIX`` dumps u^{K−1} and u^K (utils/dump.py format) so that ``--resume PREFIX`` can continue a run
from step K to a larger K on any backend and decomposition; the native CLI has the same flags.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="python -m mpi_cuda_amd", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("N", type=int, help="intervals per axis ((N+1)^3 nodes)")
    ap.add_argument("tau", type=float, help="time step")
    ap.add_argument("K", type=int, help="number of steps")
    ap.add_argument("L", type=float, nargs="?", default=1.0, help="cube edge (default 1)")
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "cpu", "torch"])
    ap.add_argument("--transport", default="auto", choices=["auto", "rccl", "torch", "loopback", "rccl-self", "push",
                                                               "push-ipc", "sdma", "sdma-ipc", "native", "none"])
    ap.add_argument("--world", type=int, default=0,
                    help="ranks of an in-process group on one GPU (transport loopback, or rccl-self: RCCL send/recv)")
    ap.add_argument("--decomp", default="slab", help="slab | block | PxQxR")
    ap.add_argument("--check-every", type=int, default=2)
    ap.add_argument("--threads", type=int, default=0, help="OpenMP threads of the CPU backend")
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=0)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-temporal", action="store_true")
    ap.add_argument("--temporal", type=int, default=5, help="at most this many steps per HBM pass (2..5)")
    ap.add_argument("--no-tb", action="store_true", help="two-step register-queue passes instead of the LDS kernel")
    ap.add_argument("--timers", action="store_true")
    ap.add_argument("--json", default="")
    ap.add_argument("--dump", default="", help="write u^K to PREFIX[.rankR].bin/.json")
    ap.add_argument("--checkpoint", default="", help="write u^{K-1}, u^K to PREFIX.prev / PREFIX.cur dumps")
    ap.add_argument("--resume", default="", help="continue from a --checkpoint PREFIX (any backend/transport)")
    ap.add_argument("--force", action="store_true", help="run even if the CFL condition is violated")
    ap.add_argument("--quiet", action="store_true")
    return ap


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    import torch
    import torch.distributed as dist

    from . import ProblemSpec
    from .parallel.rccl import init_process_group
    from .solver import Solver
    from .utils import dump as dumpio
    from .utils.report import gcell_per_s

    spec = ProblemSpec(N=a.N, tau=a.tau, K=a.K, L=a.L, check_every=a.check_every)
    if not spec.cfl_ok:
        print(f"wave3d: CFL violated: courant = tau*sqrt(3)/h = {spec.courant:.4f} > 1 (tau_max = {spec.tau_max:.3e})",
              file=sys.stderr)
        if not a.force:
            return 2
    backend = a.backend
    if backend == "auto":
        backend = "hip" if torch.cuda.is_available() else "cpu"
    rank, world, local = init_process_group("gloo" if backend != "hip" or a.transport != "torch" else "nccl")
    transport = a.transport
    kw = dict(backend=backend, transport=transport, decomp=a.decomp, overlap=not a.no_overlap,
              graph=not a.no_graph, threads=a.threads, force=a.force, temporal=1 if a.no_temporal else a.temporal, tb=not a.no_tb)
    if backend == "hip":
        kw["device"] = local if a.world == 0 else 0
        kw["timers"] = a.timers
    if a.world:
        kw.update(transport=transport if transport in ("rccl-self", "push", "sdma") else "loopback", rank=0,
                  world=a.world)
    s = Solver(spec, **kw)
    if a.resume:
        prev, meta = dumpio.load(a.resume + ".prev")
        cur, meta_c = dumpio.load(a.resume + ".cur")
        for m in (meta, meta_c):  # the checkpoint must be of THIS problem (tau and L were not compared)
            for key, want in (("N", a.N), ("tau", a.tau), ("L", a.L)):
                got = m.get(key)
                if got is None or not math.isclose(float(got), float(want), rel_tol=1e-15, abs_tol=0.0):
                    print(f"wave3d: resume: checkpoint {key} = {got} differs from the run's {want}", file=sys.stderr)
                    return 2
        s.set_state(prev, cur, int(meta_c["step"]))
    r = None
    times = []
    for i in range(a.warmup + a.repeat):
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        r = s.run()
        if i >= a.warmup:
            times.append(time.perf_counter() - t0)
    t = torch.tensor([min(times)], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    best = float(t[0])
    if rank == 0:
        if not a.quiet:
            print(f"wave3d: N={a.N} tau={a.tau:g} K={a.K} L={a.L:g} backend={s.backend} transport={s.transport} "
                  f"ranks={s.world} decomp={'x'.join(map(str, s.dims))}")
            for line in r.lines():
                print(line)
        cells = spec.cell_updates if not a.resume else float(a.N) ** 3 * (a.K - int(meta_c["step"]))
        print(f"Total time: {best:.6f} s, {cells / best / 1e9:.2f} GCell/s")
        ph = r.extra.get("phases")
        if a.timers and ph:
            print("Phases (device ms): " + ", ".join(f"{k} {v:.3f}" for k, v in ph.items()))
        if a.json:
            with open(a.json, "w") as f:
                json.dump({"backend": s.backend, "transport": s.transport, "N": a.N, "tau": a.tau, "K": a.K, "L": a.L,
                           "ranks": s.world, "dims": list(s.dims), "solve_s": best,
                           "gcell_per_s": gcell_per_s(a.N, a.K, best),
                           "steps": [[n, m, e] for n, m, e in zip(r.steps, r.max_err, r.rms_err)]}, f)
    if a.dump or a.checkpoint:
        def write(prefix, which):
            if s.transport in ("loopback", "rccl-self", "push", "sdma"):
                if rank == 0:
                    dumpio.save(prefix, s.global_field(which).numpy(), N=a.N, L=a.L, tau=a.tau,
                                step=a.K - which)
                return
            f = s.owned_field(which)
            off = s.native.plan.box[0::2] if s.transport == "torch" else (0, 0, 0)
            dumpio.save(prefix, f.numpy(), N=a.N, L=a.L, tau=a.tau, step=a.K - which, offset=off, rank=rank,
                        world=s.world, dims=s.dims)

        if a.dump:
            write(a.dump, 0)
        if a.checkpoint:
            write(a.checkpoint + ".cur", 0)
            write(a.checkpoint + ".prev", 1)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0 if r.finite else 3


if __name__ == "__main__":
    sys.exit(main())
