"""mpi_cuda_amd — MI355X-native 3D wave-equation solver framework.

Capabilities of AICCer1/MPI-CUDA (sequential / OpenMP / MPI / MPI+OpenMP / MPI+CUDA leapfrog solvers for
u_tt = Δu with Dirichlet BCs and on-the-fly analytic error checks), re-designed for MI355X:

* ``ops``       hand-written CDNA4 HIP kernels (init+first step, 2.5-D leapfrog with fused error epilogue, halo
                pack/unpack, deterministic reductions) and their PyTorch fp64 reference ops;
* ``parallel``  slab / 3-D block domain decomposition, halo exchange over RCCL (native, C++) or torch.distributed
                (gloo on CPU, RCCL on GPU), bootstrap helpers;
* ``models``    the problem definition, the analytic solution and the closed-form discrete oracle;
* ``utils``     reference-compatible log lines, JSON reports, field dumps, timers;
* ``solver``    the high-level ``solve()`` entry point used by ``bench.py`` and the CLI.

The package name keeps the reference's repository name; ``mpi-cuda_amd`` at the repo root is a symlink to it.
"""
from __future__ import annotations

__version__ = "0.1.0"

from .models.wave3d import ProblemSpec  # noqa: E402,F401
from .solver import SolveResult, solve  # noqa: E402,F401
