"""Spec + oracle tests: the closed form reproduces the reference's printed log."""
import math

import pytest

from mpi_cuda_amd import ProblemSpec
from mpi_cuda_amd.models.wave3d import REFERENCE_LOG_512, oracle_errors, torch_reference_solve


def test_oracle_reproduces_reference_log_512():
    o = oracle_errors(ProblemSpec(N=512, tau=1e-3, K=20, L=1.0))
    for n, m, r in REFERENCE_LOG_512:
        tol = 5e-6 if n == 2 else 5e-7  # printed-digit rounding + fp64 rounding of the reference's own run (Appendix B)
        assert abs(o[n][0] / m - 1) < tol
        assert abs(o[n][1] / r - 1) < tol


@pytest.mark.parametrize("N,L,linf,rms", [(128, 1.0, 2.820954e-07, 1.009161e-07), (256, 1.0, 5.958803e-08, 2.119160e-08),
                                          (128, math.pi, 2.996306e-08, 1.071891e-08),
                                          (512, math.pi, 1.732130e-09, 6.141989e-10)])
def test_oracle_other_configs(N, L, linf, rms):
    o = oracle_errors(ProblemSpec(N=N, tau=1e-3, K=20, L=L), steps=[20])[20]
    assert abs(o[0] / linf - 1) < 1e-6 and abs(o[1] / rms - 1) < 1e-6


def test_reference_sweep_rms_values():
    """δ printed in the OpenMP/MPI sweep tables (report.pdf p.7-8): 1.00e-07 (rounded), 2.12e-08, 1.40e-09; L=π:
    1.07e-08, 2.62e-09, 6.14e-10 — the RMS-over-interior convention."""
    for L, vals in ((1.0, (1.0e-07, 2.12e-08, 1.40e-09)), (math.pi, (1.07e-08, 2.62e-09, 6.14e-10))):
        for N, v in zip((128, 256, 512), vals):
            rms = oracle_errors(ProblemSpec(N=N, tau=1e-3, K=20, L=L), steps=[20])[20][1]
            assert abs(rms - v) <= 0.011 * v


@pytest.mark.parametrize("N,L,K", [(24, 1.0, 8), (31, math.pi, 6)])
def test_torch_reference_solver_matches_oracle(N, L, K):
    spec = ProblemSpec(N=N, tau=1e-3, K=K, L=L, check_every=1)
    e = torch_reference_solve(spec)
    o = oracle_errors(spec)
    for n in e:
        assert math.isclose(e[n][0], o[n][0], rel_tol=1e-6)
        assert math.isclose(e[n][1], o[n][1], rel_tol=1e-6)


def test_cfl_limits():
    assert ProblemSpec(N=512, tau=1e-3).cfl_ok
    assert ProblemSpec(N=577, tau=1e-3).cfl_ok
    assert not ProblemSpec(N=578, tau=1e-3).cfl_ok
    assert not ProblemSpec(N=2048, tau=1e-3).cfl_ok
    assert ProblemSpec(N=2048, tau=2.5e-4).cfl_ok
    assert abs(ProblemSpec(N=2048).tau_max - 2.8189e-4) < 1e-7


def test_spec_validation():
    with pytest.raises(ValueError):
        ProblemSpec(N=1)
    with pytest.raises(ValueError):
        ProblemSpec(tau=0)
    with pytest.raises(ValueError):
        ProblemSpec(K=0)
    assert ProblemSpec(K=20).check_steps() == list(range(2, 21, 2))
    assert ProblemSpec(K=7, check_every=3).check_steps() == [3, 6, 7]
