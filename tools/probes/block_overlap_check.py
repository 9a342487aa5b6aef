"""Bit-exactness matrix of the 3-D block deep-tb schedules on one GPU (in-process groups): transport × overlap ×
decomposition, against the single-GPU solve. Prints one line per case (max |diff| of u^K and the L-inf log)."""
import sys

import torch

sys.path.insert(0, ".")
from mpi_cuda_amd import ProblemSpec  # noqa: E402
from mpi_cuda_amd.solver import Solver  # noqa: E402

cases = [(27, "3x3x3", 100), (8, "2x2x2", 100), (27, "3x3x3", 140), (12, "3x2x2", 100), (9, "1x3x3", 100)]
for world, decomp, N in cases:
    spec = ProblemSpec(N=N, tau=1e-3, K=20)
    ref = Solver(spec, backend="hip", device=0, temporal=1)
    r1 = ref.run()
    f0 = ref.global_field(0)
    for transport in ("loopback", "sdma"):
        for overlap in (True, False):
            g = Solver(spec, backend="hip", transport=transport, world=world, rank=0, decomp=decomp, device=0,
                       overlap=overlap)
            r = g.run()
            d = (g.global_field(0) - f0).abs()
            bad = (d != 0).nonzero()
            where = ""
            if len(bad):
                where = f" first {bad[0].tolist()} planes x {sorted(set(bad[:, 0].tolist()))[:8]}"
            print(f"{decomp} N={N} {transport} overlap={overlap}: max|diff| {d.max().item():.3e} "
                  f"({len(bad)} nodes){where} log {'same' if r.max_err == r1.max_err else 'DIFF'}", flush=True)
