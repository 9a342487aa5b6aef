"""CPU validation of the deep temporal-blocking kernel's algorithm and address arithmetic (tools/tb_emulate.py
mirrors csrc/src/kernels_leapfrog_tb.hip): an S-step pass equals S native CPU leapfrog steps bit for bit, every global
and sin-table access stays inside its allocation."""
import math
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
import tb_emulate  # noqa: E402

from mpi_cuda_amd.ops import stencil as ops  # noqa: E402


@pytest.mark.parametrize("S", [2, 3, 4])
@pytest.mark.parametrize("N", [20, 45])
def test_tb_emulation_matches_cpu_steps(C, S, N):
    prob = C.Problem(N, 1e-3 * 40 / N, 20, 1.0)
    co = C.Coeffs.from_problem(prob)
    lay = C.make_layout(prob, C.rank_box(prob, C.Dims(1, 1, 1), 0))
    box = C.compute_box(lay)
    torch.manual_seed(N + S)

    def rand_field():
        g = torch.zeros((int(lay.nx) + 2, int(lay.ny) + 2, int(lay.nz) + 2), dtype=torch.float64)
        g[2:-2, 2:-2, 2:-2] = torch.randn(int(lay.nx) - 2, int(lay.ny) - 2, int(lay.nz) - 2, dtype=torch.float64)
        return ops.from_grid(lay, g)

    prev, cur = rand_field(), rand_field()
    s = ops.sin_table_ext(prob)
    ct = [math.cos(prob.a_t * (3 + k) * prob.tau) for k in range(1, S + 1)]
    a, b = prev.clone(), cur.clone()
    e_cpu = {}
    for k in range(1, S + 1):
        e_cpu[k] = ops.leapfrog(lay, co, b, a, [box], s, ct[k - 1], check=True)
        a, b = b, a
    o1 = np.zeros(int(lay.total))
    o2 = np.zeros(int(lay.total))
    e = tb_emulate.run_pass(lay, co, prev.numpy(), cur.numpy(), o1, o2, box, s.numpy(), S, (box.x0, box.x1), ct,
                            (1 << S) - 1)
    assert np.array_equal(ops.to_grid(lay, torch.from_numpy(o1)).numpy(), ops.to_grid(lay, a).numpy())
    assert np.array_equal(ops.to_grid(lay, torch.from_numpy(o2)).numpy(), ops.to_grid(lay, b).numpy())
    for k in range(1, S + 1):
        assert e[k][0] == e_cpu[k][0]
        assert math.isclose(e[k][1], e_cpu[k][1], rel_tol=1e-12)


@pytest.mark.parametrize("S", [2, 3, 4])
@pytest.mark.parametrize("N", [20, 45])
def test_tb_emulation_analytic_start(C, S, N):
    """The analytic-start pass (u0 = φ, u1 from the sin tables) == init_first + S CPU steps, bit for bit."""
    prob = C.Problem(N, 1e-3 * 40 / N, 20, 1.0)
    co = C.Coeffs.from_problem(prob)
    lay = C.make_layout(prob, C.rank_box(prob, C.Dims(1, 1, 1), 0))
    box = C.compute_box(lay)
    s = ops.sin_table_ext(prob)
    u0, u1 = ops.alloc_field(lay), ops.alloc_field(lay)
    ops.init_first(lay, co, s, u0, u1)
    ct = [math.cos(prob.a_t * (1 + k) * prob.tau) for k in range(1, S + 1)]
    a, b = u0.clone(), u1.clone()
    e_cpu = {}
    for k in range(1, S + 1):
        e_cpu[k] = ops.leapfrog(lay, co, b, a, [box], s, ct[k - 1], check=True)
        a, b = b, a
    o1 = np.zeros(int(lay.total))
    o2 = np.zeros(int(lay.total))
    e = tb_emulate.run_pass(lay, co, None, None, o1, o2, box, s.numpy(), S, (box.x0, box.x1), ct, (1 << S) - 1,
                            analytic_start=True)
    assert np.array_equal(ops.to_grid(lay, torch.from_numpy(o1)).numpy()[1:-1, 1:-1, 1:-1],
                          ops.to_grid(lay, a).numpy()[1:-1, 1:-1, 1:-1])
    assert np.array_equal(ops.to_grid(lay, torch.from_numpy(o2)).numpy()[1:-1, 1:-1, 1:-1],
                          ops.to_grid(lay, b).numpy()[1:-1, 1:-1, 1:-1])
    for k in range(1, S + 1):
        assert e[k][0] == e_cpu[k][0]
        assert math.isclose(e[k][1], e_cpu[k][1], rel_tol=1e-12)
