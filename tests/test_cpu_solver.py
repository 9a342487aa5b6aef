"""CPU path (the reference's sequential `wave` and OpenMP `wave3dOMP` programs): config #1 (128³, τ=1e-3, K=20)
against the closed-form oracle, bit-exactness vs the PyTorch reference, thread-count invariance."""
import math

import pytest
import torch

from mpi_cuda_amd import ProblemSpec, solve
from mpi_cuda_amd.models.wave3d import oracle_errors, torch_reference_solve
from mpi_cuda_amd.solver import Solver


def test_config1_128_matches_oracle_digits():
    """128³ L∞ 2.820954e-07 / RMS 1.009161e-07."""
    r = solve(ProblemSpec(N=128, tau=1e-3, K=20), backend="cpu")
    assert r.lines()[-1] == "Step 20, t = 0.020000, Max Error = 2.820954e-07, L2 Error = 1.009161e-07"
    o = oracle_errors(ProblemSpec(N=128, tau=1e-3, K=20))
    for n, m, e in zip(r.steps, r.max_err, r.rms_err):
        assert math.isclose(m, o[n][0], rel_tol=1e-6) and math.isclose(e, o[n][1], rel_tol=1e-6)


@pytest.mark.parametrize("N,K,L", [(20, 7, 1.0), (33, 5, math.pi)])
def test_cpu_fields_bitexact_vs_torch_reference(N, K, L):
    spec = ProblemSpec(N=N, tau=1e-3, K=K, L=L, check_every=1)
    s = Solver(spec, backend="cpu")
    r = s.run()
    errs, uk, ukm1 = torch_reference_solve(spec, return_fields=True)
    assert torch.equal(s.owned_field(0), uk)
    assert torch.equal(s.owned_field(1), ukm1)
    for n, m in zip(r.steps, r.max_err):
        assert m == errs[n][0]


def test_thread_count_invariance():
    spec = ProblemSpec(N=48, tau=1e-3, K=8)
    res = []
    for t in (1, 3, 8):
        s = Solver(spec, backend="cpu", threads=t)
        r = s.run()
        res.append((r.max_err, r.rms_err, s.owned_field(0)))
    for other in res[1:]:
        assert other[0] == res[0][0] and other[1] == res[0][1]
        assert torch.equal(other[2], res[0][2])


def test_cfl_guard_and_blowup_detection():
    with pytest.raises(ValueError):
        Solver(ProblemSpec(N=64, tau=0.02, K=30), backend="cpu")
    r = solve(ProblemSpec(N=64, tau=0.02, K=400, check_every=100), backend="cpu", force=True)
    assert not r.finite or r.max_err[-1] > 1e3


def test_run_batch_falls_back_to_run_on_cpu():
    """Solver.run_batch(n) on a backend without a batched native path: n ordinary solves, each the run() log."""
    from mpi_cuda_amd import ProblemSpec
    from mpi_cuda_amd.solver import Solver

    s = Solver(ProblemSpec(N=24, tau=1e-3, K=6, check_every=1), backend="cpu")
    r1 = s.run()
    rs = s.run_batch(3)
    assert len(rs) == 3
    for r in rs:
        assert r.steps == r1.steps and r.max_err == r1.max_err and r.rms_err == r1.rms_err
