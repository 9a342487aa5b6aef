"""Decomposed solver driven from Python over torch.distributed (gloo on CPU, RCCL or host-staged gloo on GPU).

Same kernels and same decomposition as the native GpuSolver, different transport and a Python step loop. It is the
CPU analogue of the reference's MPI (`mpi`/`onlyMPI`) and MPI+OpenMP (`mpiomp`) programs (readme.md:38-48,
report.pdf p.12-14 §4.2.2-4.2.3) and the transport A/B baseline for the native RCCL path.

Per step (report.pdf p.5 §2.2): exchange ghosts of u^n → update u^{n+1} in place over u^{n−1} (+ error partials on
check steps) → swap. The first exchange is unnecessary because u⁰ and u¹ ghosts are analytic.
"""
from __future__ import annotations

import math
import time

import torch
import torch.distributed as dist

from .._native import load
from ..models.wave3d import ProblemSpec
from ..ops import stencil as ops
from .decomp import plan as make_plan
from .halo import TorchHaloExchange


class TorchDistSolver:
    def __init__(self, spec: ProblemSpec, rank: int = 0, world: int = 1, decomp: str = "slab", device="cpu",
                 group=None, stage_via_host: bool = False, threads: int = 0):
        C = load()
        self.spec = spec
        self.rank, self.world = rank, world
        self.device = torch.device(device)
        self.group = group
        if threads and self.device.type == "cpu":
            C.cpu_set_threads(threads)
        self.problem = spec.native()
        self.coeffs = C.Coeffs.from_problem(self.problem)
        self.plan = make_plan(spec.N, world, rank, decomp, spec.tau, spec.K, spec.L)
        self.layout = self.plan.layout
        self.full = C.compute_box(self.layout)
        self.s = ops.sin_table_ext(self.problem, device=self.device)
        self.u = [ops.alloc_field(self.layout, self.device), ops.alloc_field(self.layout, self.device)]
        self.halo = TorchHaloExchange(self.layout, self.plan.halo, self.device, group, stage_via_host)
        self.final = 1

    def _ct(self, n: int) -> float:
        return math.cos(self.spec.a_t * (n * self.spec.tau))

    def set_state(self, prev: torch.Tensor, cur: torch.Tensor, step: int) -> None:
        """Resume from global (N+1)³ fields u^{step-1}, u^{step} (a checkpoint, utils/dump.py): the next run() continues
        from `step` to spec.K instead of starting from the initial condition."""
        if not 1 <= step < self.spec.K:
            raise ValueError(f"resume step {step} must be in [1, K={self.spec.K})")
        self._state = (prev, cur, int(step))

    def _load_state(self) -> int:
        prev, cur, step = self._state
        lay = self.layout
        n = self.spec.N + 1
        for src, dst in ((prev, self.u[0]), (cur, self.u[1])):
            g = ops.grid_view(lay, dst)
            g.zero_()
            # local grid index i <-> global node g0 - 1 + i (ghosts included), clipped to the domain
            sl = []
            gl = []
            for g0, nn in ((int(lay.gx0), int(lay.nx)), (int(lay.gy0), int(lay.ny)), (int(lay.gz0), int(lay.nz))):
                lo = max(0, 1 - g0)
                hi = min(nn + 2, n + 1 - g0)
                sl.append(slice(lo, hi))
                gl.append(slice(g0 - 1 + lo, g0 - 1 + hi))
            g[sl[0], sl[1], sl[2]] = src[gl[0], gl[1], gl[2]].to(dst.device, torch.float64)
        return step

    def run(self) -> dict:
        spec = self.spec
        checks = spec.check_steps()
        local = {}
        t0 = time.perf_counter()
        n0 = 1
        if getattr(self, "_state", None) is not None:
            n0 = self._load_state()
            checks = [n for n in checks if n > n0]
        else:
            ops.init_first(self.layout, self.coeffs, self.s, self.u[0], self.u[1])
            if 1 in checks:
                local[1] = ops.error(self.layout, self.u[1], self.full, self.s, self._ct(1))
        cur, old = 1, 0
        for n in range(n0, spec.K):
            if n > n0:
                self.halo.exchange(self.u[cur])
            chk = (n + 1) in checks
            r = ops.leapfrog(self.layout, self.coeffs, self.u[cur], self.u[old], [self.full], self.s,
                             self._ct(n + 1), chk)
            if chk:
                local[n + 1] = r if r is not None else (0.0, 0.0)
            cur, old = old, cur
        self.final = cur
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        steps = sorted(local)
        mine = torch.tensor([[local[n][0], local[n][1]] for n in steps], dtype=torch.float64)
        if self.world > 1:
            gathered = [torch.zeros_like(mine) for _ in range(self.world)]
            dist.all_gather(gathered, mine, group=self.group)
        else:
            gathered = [mine]
        denom = float(spec.N - 1) ** 3
        mx, rms = [], []
        for i, _ in enumerate(steps):
            m, s = 0.0, 0.0
            for g in gathered:  # fixed rank order
                m = max(m, float(g[i, 0]))
                s += float(g[i, 1])
            mx.append(m)
            rms.append(math.sqrt(s / denom))
        dt = time.perf_counter() - t0
        return {"steps": steps, "max_err": mx, "rms_err": rms, "solve_s": dt,
                "finite": all(math.isfinite(v) for v in mx + rms)}

    def owned_field(self, which: int = 0) -> torch.Tensor:
        """Owned nodes (nx, ny, nz) of u^K (which=0) or u^{K-1} (which=1), on the CPU."""
        lay = self.layout
        u = self.u[self.final if which == 0 else 1 - self.final]
        g = ops.grid_view(lay, u)
        return g[1:1 + int(lay.nx), 1:1 + int(lay.ny), 1:1 + int(lay.nz)].detach().cpu().clone()
