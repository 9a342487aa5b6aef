"""The 3D wave-equation "model": problem definition, analytic solution, closed-form discrete oracle and an independent
PyTorch fp64 reference solver.

Reference behaviour (AICCer1/MPI-CUDA; the programs are not in the snapshot, the documents are — SURVEY.md §0.1):

* PDE u_tt = Δu on [0,L]³, homogeneous Dirichlet BCs, u(t=0) = φ, u_t(t=0) = 0              report.pdf p.4 §1
* analytic u_a = sin(πx/L)·sin(πy/L)·sin(πz/L)·cos(a_t t), a_t = π·√3/L                    report.pdf p.4 §1
* grid x_i = i·h, h = L/N, nodes 0..N; leapfrog with the 7-point Laplacian;
  u¹ = u⁰ + τ²/2·Δ_h u⁰                                                                        report.pdf p.5 §2-2.2
* "Max Error" = L∞ over the nodes, "L2 Error" = RMS over the (N−1)³ interior nodes           report.pdf p.6 §3.1.2,
                                                                                               SURVEY.md §1.3 VERIFIED
* golden log (512³, τ=1e-3, K=20, L=1)                                                        report.pdf p.15-16 §4.3

The closed-form oracle: φ is a discrete eigenfunction of Δ_h with eigenvalue −λ, so the discrete
solution is exactly cos(nθ)·φ with cos θ = 1 − τ²λ/2. The error at step n is d_n·|φ| with d_n = |cos nθ − cos(a_t nτ)|,
giving L∞ = d_n·max|φ| and RMS = d_n·(Σφ²/(N−1)³)^½ — evaluated here in 50-digit arithmetic (mpmath), because the
two cosines cancel in fp64.
"""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass, field

import numpy as np
import torch

# Golden per-step log of the reference's GPU program, 1 and 2 GPUs identical (report.pdf p.15-16 §4.3.1-4.3.2).
REFERENCE_LOG_512 = [
    (2, 3.967859e-11, 1.406978e-11),
    (4, 1.587058e-10, 5.627573e-11),
    (6, 3.570526e-10, 1.266079e-10),
    (8, 6.346724e-10, 2.250497e-10),
    (10, 9.915001e-10, 3.515776e-10),
    (12, 1.427449e-09, 5.061618e-10),
    (14, 1.942419e-09, 6.887656e-10),
    (16, 2.536286e-09, 8.993458e-10),
    (18, 3.208909e-09, 1.137852e-09),
    (20, 3.960129e-09, 1.404229e-09),
]


@dataclass
class ProblemSpec:
    """N intervals per axis ((N+1)³ nodes), time step tau, K steps, cube edge L (positional CLI ``N tau K [L]``)."""

    N: int = 512
    tau: float = 1e-3
    K: int = 20
    L: float = 1.0
    check_every: int = 2
    extra: dict = field(default_factory=dict)

    def __post_init__(self) -> None:
        if self.N < 2:
            raise ValueError("N must be >= 2")
        if not (self.tau > 0 and math.isfinite(self.tau)):
            raise ValueError("tau must be > 0")
        if self.K < 1:
            raise ValueError("K must be >= 1")
        if not (self.L > 0 and math.isfinite(self.L)):
            raise ValueError("L must be > 0")

    @property
    def h(self) -> float:
        return self.L / self.N

    @property
    def a_t(self) -> float:
        return math.pi * math.sqrt(3.0 / (self.L * self.L))

    @property
    def courant(self) -> float:
        """τ·√3/h — the 3-D 7-point leapfrog is stable iff this is ≤ 1."""
        return self.tau * math.sqrt(3.0) / self.h

    @property
    def cfl_ok(self) -> bool:
        return self.courant <= 1.0

    @property
    def tau_max(self) -> float:
        return self.h / math.sqrt(3.0)

    @property
    def cell_updates(self) -> float:
        """N³·K — the reference-derived GCell/s numerator."""
        return float(self.N) ** 3 * self.K

    def check_steps(self) -> list[int]:
        ce = self.check_every
        return [n for n in range(1, self.K + 1) if (ce > 0 and n % ce == 0) or n == self.K]

    def native(self):
        from .._native import load

        return load().Problem(self.N, self.tau, self.K, self.L)

    def as_dict(self) -> dict:
        d = asdict(self)
        d.pop("extra", None)
        return d


def sin_table(spec: ProblemSpec) -> np.ndarray:
    """sin(π x_i / L), i = 0..N, boundary entries exactly 0 (same values the kernels use)."""
    i = np.arange(spec.N + 1, dtype=np.float64)
    s = np.sin(np.pi * (i * spec.h) / spec.L)
    s[0] = 0.0
    s[-1] = 0.0
    return s


def analytic(spec: ProblemSpec, n: int, dtype=torch.float64, device="cpu") -> torch.Tensor:
    """u_a at step n on the full (N+1)³ node grid."""
    s = torch.as_tensor(sin_table(spec), dtype=dtype, device=device)
    ct = math.cos(spec.a_t * (n * spec.tau))
    return ((s[:, None, None] * s[None, :, None]) * ct) * s[None, None, :]  # stencil.hpp::analytic_row order


# ----------------------------------------------------------------------------------------------------------------
# closed-form oracle
# ----------------------------------------------------------------------------------------------------------------
def oracle_errors(spec: ProblemSpec, steps: list[int] | None = None, dps: int = 50) -> dict[int, tuple[float, float]]:
    """Exact (L∞, RMS-interior) error of the discrete scheme at each step, from the closed form of SURVEY.md §1.6."""
    import mpmath as mp

    mp.mp.dps = dps
    N = spec.N
    L = mp.mpf(spec.L)
    h = L / N
    tau = mp.mpf(spec.tau)
    lam = 3 * (4 / h**2) * mp.sin(mp.pi * h / (2 * L)) ** 2
    cos_theta = 1 - tau**2 * lam / 2
    theta = mp.acos(cos_theta)
    a_t = mp.pi * mp.sqrt(3 / L**2)
    # max_i |sin(π i/N)|³ and Σ_interior φ² = (Σ_i sin²(π i/N))³
    s_max = max(abs(mp.sin(mp.pi * i / N)) for i in range(N + 1))
    s2 = mp.fsum(mp.sin(mp.pi * i / N) ** 2 for i in range(1, N))
    rms_fac = mp.sqrt(s2**3 / mp.mpf(N - 1) ** 3)
    out = {}
    for n in steps if steps is not None else spec.check_steps():
        d = abs(mp.cos(n * theta) - mp.cos(a_t * n * tau))
        out[n] = (float(d * s_max**3), float(d * rms_fac))
    return out


# ----------------------------------------------------------------------------------------------------------------
# independent PyTorch fp64 reference solver (second oracle; runs on CPU or GPU)
# ----------------------------------------------------------------------------------------------------------------
def d2sum_torch(u: torch.Tensor) -> torch.Tensor:
    """h²·Δ_h on the interior of a full node grid: the sum of the three second differences (stencil.hpp::d2sum, same
    operation order as the native kernels)."""
    c = u[1:-1, 1:-1, 1:-1]
    c2 = 2.0 * c
    return ((u[2:, 1:-1, 1:-1] - c2 + u[:-2, 1:-1, 1:-1]) + (u[1:-1, 2:, 1:-1] - c2 + u[1:-1, :-2, 1:-1])
            + (u[1:-1, 1:-1, 2:] - c2 + u[1:-1, 1:-1, :-2]))


def fma_torch(a: float, b: torch.Tensor, c: torch.Tensor) -> torch.Tensor:
    """a·b + c rounded once (stencil.hpp's fused leapfrog / first step; torch has no fused multiply-add): the
    elementwise IEEE fma of the native binding, on a host copy."""
    from mpi_cuda_amd._native import load

    bb, cc = torch.broadcast_tensors(b, c)
    bn = bb.detach().to("cpu", torch.float64).contiguous().numpy().ravel()
    cn = cc.detach().to("cpu", torch.float64).contiguous().numpy().ravel()
    an = np.full_like(bn, a)
    r = np.asarray(load().fma_array(an, bn, cn)).reshape(tuple(bb.shape))
    return torch.from_numpy(r).to(b.device)


def laplacian_torch(u: torch.Tensor, h: float) -> torch.Tensor:
    """7-point Δ_h on the interior of a full node grid."""
    return d2sum_torch(u) * (1.0 / (h * h))


def torch_reference_solve(spec: ProblemSpec, device="cpu", return_fields: bool = False):
    """Plain PyTorch fp64 implementation of report.pdf p.5 §2.2. Returns {step: (Linf, RMS)} (+ (u^K, u^{K-1}))."""
    tau2 = spec.tau * spec.tau
    u0 = analytic(spec, 0, device=device)
    u0[0], u0[-1] = 0.0, 0.0
    u0[:, 0], u0[:, -1] = 0.0, 0.0
    u0[:, :, 0], u0[:, :, -1] = 0.0, 0.0
    u1 = torch.zeros_like(u0)
    ih2 = 1.0 / (spec.h * spec.h)
    lam, half_lam = tau2 * ih2, (0.5 * tau2) * ih2  # problem.hpp::Coeffs: the coefficients of d2sum
    u1[1:-1, 1:-1, 1:-1] = fma_torch(half_lam, d2sum_torch(u0), u0[1:-1, 1:-1, 1:-1])
    denom = float(spec.N - 1) ** 3
    errs = {}
    checks = set(spec.check_steps())

    def err(u, n):
        e = (u[1:-1, 1:-1, 1:-1] - analytic(spec, n, device=device)[1:-1, 1:-1, 1:-1]).abs()
        return float(e.max()), math.sqrt(float((e * e).sum()) / denom)

    if 1 in checks:
        errs[1] = err(u1, 1)
    prev, cur = u0, u1
    for n in range(1, spec.K):
        nxt = torch.zeros_like(cur)
        c = cur[1:-1, 1:-1, 1:-1]
        nxt[1:-1, 1:-1, 1:-1] = fma_torch(lam, d2sum_torch(cur), 2.0 * c - prev[1:-1, 1:-1, 1:-1])
        prev, cur = cur, nxt
        if n + 1 in checks:
            errs[n + 1] = err(cur, n + 1)
    if return_fields:
        return errs, cur, prev
    return errs
