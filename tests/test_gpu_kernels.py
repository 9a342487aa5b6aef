"""HIP kernel numerics vs the native CPU path (bit-exact, same op order, -ffp-contract=off) and vs a plain PyTorch
fp64 reference of the same op."""
import math

import pytest
import torch

from mpi_cuda_amd.ops import stencil as ops

pytestmark = pytest.mark.gpu


def _setup(C, N, world=1, rank=0, decomp="slab", tau=1e-3):
    prob = C.Problem(N, tau, 20, 1.0)
    dims = C.parse_dims(decomp, world, N)
    lay = C.make_layout(prob, C.rank_box(prob, dims, rank))
    return prob, C.Coeffs.from_problem(prob), lay, dims


@pytest.mark.parametrize("N,world,rank,decomp", [(32, 1, 0, "slab"), (47, 1, 0, "slab"), (64, 2, 1, "slab"),
                                                 (50, 8, 5, "block"), (33, 4, 0, "1x2x2"), (129, 3, 2, "slab")])
def test_init_first_bitexact(gpu, N, world, rank, decomp):
    C = gpu
    prob, co, lay, _ = _setup(C, N, world, rank, decomp)
    s_cpu = ops.sin_table_ext(prob)
    a0, a1 = ops.alloc_field(lay), ops.alloc_field(lay)
    ops.init_first(lay, co, s_cpu, a0, a1)
    s_gpu = s_cpu.cuda()
    g0, g1 = ops.alloc_field(lay, "cuda"), ops.alloc_field(lay, "cuda")
    ops.init_first(lay, co, s_gpu, g0, g1)
    torch.cuda.synchronize()
    assert torch.equal(ops.to_grid(lay, g0).cpu(), ops.to_grid(lay, a0))
    assert torch.equal(ops.to_grid(lay, g1).cpu(), ops.to_grid(lay, a1))


TILINGS = [dict(variant=0, ty=8), dict(variant=0, ty=4), dict(variant=0, ty=16), dict(variant=0, ty=8, xcd_remap=False),
           dict(variant=0, ty=8, nt_store=True), dict(variant=0, ty=4, target_blocks=64),
           dict(variant=1, rows=1), dict(variant=1, rows=2), dict(variant=1, rows=4), dict(variant=1, rows=8),
           dict(variant=1, rows=4, xcd_remap=False, nt_store=True), dict(variant=1, rows=2, target_blocks=100)]


@pytest.mark.parametrize("tiling", TILINGS)
@pytest.mark.parametrize("N,world,rank,decomp", [(40, 1, 0, "slab"), (61, 2, 0, "slab"), (70, 8, 3, "block"),
                                                 (130, 1, 0, "slab")])
def test_leapfrog_bitexact_and_vs_torch(gpu, tiling, N, world, rank, decomp):
    C = gpu
    prob, co, lay, _ = _setup(C, N, world, rank, decomp)
    torch.manual_seed(N + rank)
    # random fields (ghosts included) so every neighbour access is exercised
    cur = torch.randn(int(lay.total), dtype=torch.float64)
    old = torch.randn(int(lay.total), dtype=torch.float64)
    box = C.compute_box(lay)
    s = ops.sin_table_ext(prob)
    ct = math.cos(prob.a_t * 5 * prob.tau)
    old_cpu = old.clone()
    e_cpu = ops.leapfrog(lay, co, cur, old_cpu, [box], s, ct, check=True)
    t = C.LeapfrogTiling()
    for k, v in tiling.items():
        setattr(t, k, v)
    cur_g, old_g = cur.cuda(), old.cuda()
    e_gpu = ops.leapfrog(lay, co, cur_g, old_g, [box], s.cuda(), ct, check=True, tiling=t)
    torch.cuda.synchronize()
    # whole padded array must match: updated nodes bit-exact, everything else untouched
    assert torch.equal(old_g.cpu(), old_cpu)
    assert e_gpu[0] == e_cpu[0]
    assert math.isclose(e_gpu[1], e_cpu[1], rel_tol=1e-12)
    # PyTorch fp64 reference of the same op
    ref = ops.ref_leapfrog_grid(ops.to_grid(lay, cur), ops.to_grid(lay, old), co.ihx2, co.ihy2, co.ihz2, co.tau2, box)
    torch.testing.assert_close(ops.to_grid(lay, old_g.cpu()), ref, rtol=0, atol=1e-9)


def test_leapfrog_subboxes(gpu):
    """Several disjoint boxes in one launch (the shell of a block-decomposed rank) == one launch per box == CPU."""
    C = gpu
    prob, co, lay, _ = _setup(C, 90, 8, 6, "2x2x2")
    torch.manual_seed(1)
    cur = torch.randn(int(lay.total), dtype=torch.float64)
    old = torch.randn(int(lay.total), dtype=torch.float64)
    s = ops.sin_table_ext(prob)
    full = C.compute_box(lay)
    boxes = [C.LBox(full.x0, full.x0 + 1, full.y0, full.y1, full.z0, full.z1),
             C.LBox(full.x0 + 1, full.x1, full.y0, full.y0 + 1, full.z0, full.z1),
             C.LBox(full.x0 + 1, full.x1, full.y0 + 1, full.y1, full.z1 - 1, full.z1),
             C.LBox(full.x0 + 3, full.x0 + 7, full.y0 + 5, full.y0 + 6, full.z0 + 3, full.z0 + 4)]
    o_cpu = old.clone()
    e_cpu = ops.leapfrog(lay, co, cur, o_cpu, boxes, s, 0.7, check=True)
    o_gpu = old.cuda()
    e_gpu = ops.leapfrog(lay, co, cur.cuda(), o_gpu, boxes, s.cuda(), 0.7, check=True)
    torch.cuda.synchronize()
    assert torch.equal(o_gpu.cpu(), o_cpu)
    assert e_gpu[0] == e_cpu[0] and math.isclose(e_gpu[1], e_cpu[1], rel_tol=1e-12)


def test_error_kernel(gpu):
    C = gpu
    prob, co, lay, _ = _setup(C, 77, 2, 1, "slab")
    torch.manual_seed(3)
    u = torch.randn(int(lay.total), dtype=torch.float64)
    s = ops.sin_table_ext(prob)
    box = C.compute_box(lay)
    a = ops.error(lay, u, box, s, 0.3)
    b = ops.error(lay, u.cuda(), box, s.cuda(), 0.3)
    assert a[0] == b[0] and math.isclose(a[1], b[1], rel_tol=1e-12)


@pytest.mark.parametrize("decomp,world,rank", [("2x2x2", 8, 3), ("1x2x3", 6, 4), ("block", 16, 9)])
def test_pack_unpack(gpu, decomp, world, rank):
    C = gpu
    prob, co, lay, dims = _setup(C, 45, world, rank, decomp)
    plan = C.make_halo_plan(lay, dims, rank)
    torch.manual_seed(rank)
    u = torch.randn(int(lay.total), dtype=torch.float64)
    n = max(int(plan.packed_doubles), 1)
    b_cpu = torch.zeros(n, dtype=torch.float64)
    ops.pack(lay, plan, u, b_cpu)
    b_gpu = torch.zeros(n, dtype=torch.float64, device="cuda")
    ops.pack(lay, plan, u.cuda(), b_gpu)
    torch.cuda.synchronize()
    assert torch.equal(b_gpu.cpu(), b_cpu)
    src = torch.randn(n, dtype=torch.float64)
    v_cpu = u.clone()
    ops.unpack(lay, plan, src, v_cpu)
    v_gpu = u.cuda()
    ops.unpack(lay, plan, src.cuda(), v_gpu)
    torch.cuda.synchronize()
    assert torch.equal(v_gpu.cpu(), v_cpu)


@pytest.mark.parametrize("rows", [1, 2, 4])
@pytest.mark.parametrize("N", [40, 77, 130])
@pytest.mark.parametrize("target_waves", [0, 50])
def test_leapfrog2_equals_two_single_steps(gpu, rows, N, target_waves):
    """Temporal blocking: one fused pass == two CPU steps, bit for bit (random interior, Dirichlet-zero boundary)."""
    C = gpu
    prob, co, lay, _ = _setup(C, N)
    box = C.compute_box(lay)
    torch.manual_seed(N * 7 + rows)

    def rand_field():
        g = torch.zeros((int(lay.nx) + 2, int(lay.ny) + 2, int(lay.nz) + 2), dtype=torch.float64)
        g[2:-2, 2:-2, 2:-2] = torch.randn(int(lay.nx) - 2, int(lay.ny) - 2, int(lay.nz) - 2, dtype=torch.float64)
        return ops.from_grid(lay, g)

    prev, cur = rand_field(), rand_field()
    s = ops.sin_table_ext(prob)
    ct2 = math.cos(prob.a_t * 6 * prob.tau)
    # CPU: u^{n+1} in place over prev, then u^{n+2} in place over cur
    a, b = prev.clone(), cur.clone()
    ops.leapfrog(lay, co, b, a, [box], s)          # a = u^{n+1}
    e_cpu = ops.leapfrog(lay, co, a, b, [box], s, ct2, check=True)  # b = u^{n+2}
    t = C.Leapfrog2Tiling()
    t.rows, t.target_waves = rows, target_waves
    o1 = torch.zeros(int(lay.total), dtype=torch.float64, device="cuda")
    o2 = torch.zeros_like(o1)
    e_gpu = ops.leapfrog2(lay, co, prev.cuda(), cur.cuda(), o1, o2, box, s.cuda(), ct2, check=True, tiling=t)
    torch.cuda.synchronize()
    # the fused kernel writes only the interior; boundary/ghost nodes of the outputs stay 0 like the inputs' boundary
    assert torch.equal(ops.to_grid(lay, o1.cpu()), ops.to_grid(lay, a))
    assert torch.equal(ops.to_grid(lay, o2.cpu()), ops.to_grid(lay, b))
    assert e_gpu[0] == e_cpu[0] and math.isclose(e_gpu[1], e_cpu[1], rel_tol=1e-12)


@pytest.mark.parametrize("stages", [2, 3, 4])
@pytest.mark.parametrize("N", [40, 77, 130])
@pytest.mark.parametrize("threads", [768, 1024])
def test_leapfrog_tb_equals_single_steps(gpu, stages, N, threads):
    """Deep temporal blocking: one LDS pass of S steps == S CPU steps, bit for bit, with every level checked."""
    C = gpu
    prob, co, lay, _ = _setup(C, N)
    box = C.compute_box(lay)
    torch.manual_seed(N * 11 + stages)

    def rand_field():
        g = torch.zeros((int(lay.nx) + 2, int(lay.ny) + 2, int(lay.nz) + 2), dtype=torch.float64)
        g[2:-2, 2:-2, 2:-2] = torch.randn(int(lay.nx) - 2, int(lay.ny) - 2, int(lay.nz) - 2, dtype=torch.float64)
        return ops.from_grid(lay, g)

    prev, cur = rand_field(), rand_field()
    s = ops.sin_table_ext(prob)
    ct = [math.cos(prob.a_t * (5 + k) * prob.tau) for k in range(1, stages + 1)]
    a, b = prev.clone(), cur.clone()
    e_cpu = {}
    for k in range(1, stages + 1):  # u^{n+k} in place over u^{n+k-2}
        e_cpu[k] = ops.leapfrog(lay, co, b, a, [box], s, ct[k - 1], check=True)
        a, b = b, a
    # now b = u^{n+S}, a = u^{n+S-1}
    o1 = torch.zeros(int(lay.total), dtype=torch.float64, device="cuda")
    o2 = torch.zeros_like(o1)
    mask = (1 << stages) - 1
    e_gpu = ops.leapfrog_tb(lay, co, prev.cuda(), cur.cuda(), o1, o2, box, s.cuda(), stages, ct, mask, threads, p2=False)
    torch.cuda.synchronize()
    assert torch.equal(ops.to_grid(lay, o1.cpu()), ops.to_grid(lay, a))
    assert torch.equal(ops.to_grid(lay, o2.cpu()), ops.to_grid(lay, b))
    for k in range(1, stages + 1):
        assert e_gpu[k][0] == e_cpu[k][0]
        assert math.isclose(e_gpu[k][1], e_cpu[k][1], rel_tol=1e-12)


@pytest.mark.parametrize("stages", [2, 3, 4])
@pytest.mark.parametrize("N", [40, 77, 130])
def test_leapfrog_tb_analytic_start(gpu, stages, N):
    """Analytic-start pass (u⁰ = φ, u¹ computed in the kernel) == init_first + S CPU steps on the interior."""
    C = gpu
    prob, co, lay, _ = _setup(C, N)
    box = C.compute_box(lay)
    s = ops.sin_table_ext(prob)
    u0, u1 = ops.alloc_field(lay), ops.alloc_field(lay)
    ops.init_first(lay, co, s, u0, u1)
    ct = [math.cos(prob.a_t * (1 + k) * prob.tau) for k in range(1, stages + 1)]
    a, b = u0.clone(), u1.clone()
    e_cpu = {}
    for k in range(1, stages + 1):
        e_cpu[k] = ops.leapfrog(lay, co, b, a, [box], s, ct[k - 1], check=True)
        a, b = b, a
    o1 = torch.zeros(int(lay.total), dtype=torch.float64, device="cuda")
    o2 = torch.zeros_like(o1)
    e_gpu = ops.leapfrog_tb(lay, co, None, None, o1, o2, box, s.cuda(), stages, ct, (1 << stages) - 1,
                            analytic_start=True, p2=False)
    torch.cuda.synchronize()
    inner = (slice(1, -1),) * 3  # u⁰ = φ also fills the ghosts of the CPU buffers; the pass writes the interior only
    assert torch.equal(ops.to_grid(lay, o1.cpu())[inner], ops.to_grid(lay, a)[inner])
    assert torch.equal(ops.to_grid(lay, o2.cpu())[inner], ops.to_grid(lay, b)[inner])
    for k in range(1, stages + 1):
        assert e_gpu[k][0] == e_cpu[k][0]
        assert math.isclose(e_gpu[k][1], e_cpu[k][1], rel_tol=1e-12)


def _rand_interior(C, lay, seed):
    torch.manual_seed(seed)
    g = torch.zeros((int(lay.nx) + 2, int(lay.ny) + 2, int(lay.nz) + 2), dtype=torch.float64)
    g[2:-2, 2:-2, 2:-2] = torch.randn(int(lay.nx) - 2, int(lay.ny) - 2, int(lay.nz) - 2, dtype=torch.float64)
    return ops.from_grid(lay, g)


P2_MASKS = {"all": lambda S: (1 << S) - 1, "odd": lambda S: 0b10101 & ((1 << S) - 1),
            "even": lambda S: 0b01010 & ((1 << S) - 1), "none": lambda S: 0}


@pytest.mark.parametrize("stages", [2, 3, 4, 5])
@pytest.mark.parametrize("N", [40, 77, 130])
@pytest.mark.parametrize("chunked", [False, True])
@pytest.mark.parametrize("mask", ["all", "odd", "even"])
def test_leapfrog_p2_equals_single_steps(gpu, stages, N, chunked, mask):
    """Pair-tiled pass (k_leapfrog_p2): one pass of S steps == S CPU steps, bit for bit, fields and checked levels.
    chunked: x split into chunks (the CH instantiations); N = 130 has interior tiles (no Dirichlet select needed)."""
    C = gpu
    prob, co, lay, _ = _setup(C, N)
    box = C.compute_box(lay)
    assert C.gpu_leapfrog_p2_supported(lay, box, stages)
    prev, cur = _rand_interior(C, lay, N * 13 + stages), _rand_interior(C, lay, N * 17 + stages)
    s = ops.sin_table_ext(prob)
    ct = [math.cos(prob.a_t * (5 + k) * prob.tau) for k in range(1, stages + 1)]
    a, b = prev.clone(), cur.clone()
    e_cpu = {}
    for k in range(1, stages + 1):
        e_cpu[k] = ops.leapfrog(lay, co, b, a, [box], s, ct[k - 1], check=True)
        a, b = b, a
    o1 = torch.zeros(int(lay.total), dtype=torch.float64, device="cuda")
    o2 = torch.zeros_like(o1)
    m = P2_MASKS[mask](stages)
    e_gpu = ops.leapfrog_tb(lay, co, prev.cuda(), cur.cuda(), o1, o2, box, s.cuda(), stages, ct, m,
                            p2=True, target_blocks=256 if chunked else 1)
    torch.cuda.synchronize()
    assert torch.equal(ops.to_grid(lay, o1.cpu()), ops.to_grid(lay, a))
    assert torch.equal(ops.to_grid(lay, o2.cpu()), ops.to_grid(lay, b))
    assert sorted(e_gpu) == [k for k in range(1, stages + 1) if m >> (k - 1) & 1]
    for k in e_gpu:
        assert e_gpu[k][0] == e_cpu[k][0]
        assert math.isclose(e_gpu[k][1], e_cpu[k][1], rel_tol=1e-12)
    # PyTorch fp64 reference of the last level (S plain leapfrog steps of the same op)
    pa, pb = ops.to_grid(lay, prev), ops.to_grid(lay, cur)
    for _ in range(stages):
        pa, pb = pb, ops.ref_leapfrog_grid(pb, pa, co.ihx2, co.ihy2, co.ihz2, co.tau2, box)
    torch.testing.assert_close(ops.to_grid(lay, o2.cpu()), pb, rtol=0, atol=1e-9)


@pytest.mark.parametrize("stages", [2, 3, 4])
@pytest.mark.parametrize("N", [40, 77, 130])
@pytest.mark.parametrize("chunked", [False, True])
def test_leapfrog_p2_analytic_start(gpu, stages, N, chunked):
    """Pair-tiled analytic-start pass == init_first + S CPU steps on the interior, bit for bit."""
    C = gpu
    prob, co, lay, _ = _setup(C, N)
    box = C.compute_box(lay)
    s = ops.sin_table_ext(prob)
    u0, u1 = ops.alloc_field(lay), ops.alloc_field(lay)
    ops.init_first(lay, co, s, u0, u1)
    ct = [math.cos(prob.a_t * (1 + k) * prob.tau) for k in range(1, stages + 1)]
    a, b = u0.clone(), u1.clone()
    e_cpu = {}
    for k in range(1, stages + 1):
        e_cpu[k] = ops.leapfrog(lay, co, b, a, [box], s, ct[k - 1], check=True)
        a, b = b, a
    o1 = torch.zeros(int(lay.total), dtype=torch.float64, device="cuda")
    o2 = torch.zeros_like(o1)
    e_gpu = ops.leapfrog_tb(lay, co, None, None, o1, o2, box, s.cuda(), stages, ct, (1 << stages) - 1,
                            analytic_start=True, p2=True, target_blocks=256 if chunked else 1)
    torch.cuda.synchronize()
    inner = (slice(1, -1),) * 3
    assert torch.equal(ops.to_grid(lay, o1.cpu())[inner], ops.to_grid(lay, a)[inner])
    assert torch.equal(ops.to_grid(lay, o2.cpu())[inner], ops.to_grid(lay, b)[inner])
    for k in range(1, stages + 1):
        assert e_gpu[k][0] == e_cpu[k][0]
        assert math.isclose(e_gpu[k][1], e_cpu[k][1], rel_tol=1e-12)


def test_leapfrog_p2_equals_tb(gpu):
    """The two LDS kernels agree bit for bit on a 4-step pass (same formulas and operation order)."""
    C = gpu
    prob, co, lay, _ = _setup(C, 96)
    box = C.compute_box(lay)
    prev, cur = _rand_interior(C, lay, 5), _rand_interior(C, lay, 6)
    s = ops.sin_table_ext(prob).cuda()
    ct = [0.5, 0.4, 0.3, 0.2]
    outs = []
    for p2 in (False, True):
        o1 = torch.zeros(int(lay.total), dtype=torch.float64, device="cuda")
        o2 = torch.zeros_like(o1)
        e = ops.leapfrog_tb(lay, co, prev.cuda(), cur.cuda(), o1, o2, box, s, 4, ct, 0b1111, p2=p2)
        outs.append((o1.cpu(), o2.cpu(), e))
    assert torch.equal(ops.to_grid(lay, outs[0][0]), ops.to_grid(lay, outs[1][0]))
    assert torch.equal(ops.to_grid(lay, outs[0][1]), ops.to_grid(lay, outs[1][1]))
    for k in range(1, 5):
        assert outs[0][2][k][0] == outs[1][2][k][0]
        assert math.isclose(outs[0][2][k][1], outs[1][2][k][1], rel_tol=1e-12)


@pytest.mark.parametrize("N,world,rank,decomp", [(36, 1, 0, "slab"), (53, 1, 0, "slab"), (40, 2, 1, "slab"),
                                                 (45, 8, 5, "2x2x2"), (38, 6, 2, "1x2x3")])
@pytest.mark.parametrize("check", [False, True])
def test_init_two_equals_init_plus_step(gpu, N, world, rank, decomp, check):
    """k_init_two (u¹, u² analytically) == init_first + one leapfrog step of the GLOBAL field, ghosts included."""
    C = gpu
    prob, co, lay, _ = _setup(C, N, world, rank, decomp)
    # global reference on the CPU
    g_prob, g_co, g_lay, _ = _setup(C, N)
    s = ops.sin_table_ext(prob)
    u0, u1 = ops.alloc_field(g_lay), ops.alloc_field(g_lay)
    ops.init_first(g_lay, g_co, s, u0, u1)
    u2 = u0.clone()
    ct2 = math.cos(prob.a_t * 2 * prob.tau)
    ops.leapfrog(g_lay, g_co, u1, u2, [C.compute_box(g_lay)], s)
    G1, G2 = ops.to_grid(g_lay, u1), ops.to_grid(g_lay, u2)
    a = ops.alloc_field(lay, "cuda")
    b = ops.alloc_field(lay, "cuda")
    nb = C.gpu_init_two_partials(lay)
    part = torch.zeros((nb, 2), dtype=torch.float64, device="cuda")
    C.gpu_init_two(lay, co, s.cuda().data_ptr(), a.data_ptr(), b.data_ptr(), ct2, part.data_ptr() if check else 0,
                   torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    A, B = ops.to_grid(lay, a.cpu()), ops.to_grid(lay, b.cpu())
    # local grid index i <-> global node gx0 - 1 + i; compare every allocated node inside the global grid
    n = N + 1
    xs = slice(max(0, 1 - int(lay.gx0)), min(int(lay.nx) + 2, n + 1 - int(lay.gx0)))
    ys = slice(max(0, 1 - int(lay.gy0)), min(int(lay.ny) + 2, n + 1 - int(lay.gy0)))
    zs = slice(max(0, 1 - int(lay.gz0)), min(int(lay.nz) + 2, n + 1 - int(lay.gz0)))

    def gsl(sl, g0):
        return slice(sl.start + g0, sl.stop + g0)  # +1 (ghost) -1 (local->global) cancel in the padded grids

    ref1 = G1[gsl(xs, int(lay.gx0)), gsl(ys, int(lay.gy0)), gsl(zs, int(lay.gz0))]
    ref2 = G2[gsl(xs, int(lay.gx0)), gsl(ys, int(lay.gy0)), gsl(zs, int(lay.gz0))]
    assert torch.equal(A[xs, ys, zs], ref1)
    assert torch.equal(B[xs, ys, zs], ref2)
    if check:
        out = torch.empty(2, dtype=torch.float64, device="cuda")
        C.gpu_reduce(part.data_ptr(), nb, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        e = ops.error(lay, b.cpu(), C.compute_box(lay), s, ct2)
        o = out.cpu()
        assert float(o[0]) == e[0] and math.isclose(float(o[1]), e[1], rel_tol=1e-12)


def test_reduce_batch_matches_single_reductions(gpu):
    """k_reduce_batch (one workgroup per job, the deferred reductions of the LDS passes) == k_reduce per job, bit for
    bit, for job counts across the 64-job launch split and lengths around the 1024-thread stride."""
    C = gpu
    torch.manual_seed(7)
    st = torch.cuda.current_stream().cuda_stream
    lens = [1, 5, 256, 1023, 1024, 1025, 3000] * 10  # 70 jobs: two launches
    parts = [torch.rand((n, 2), dtype=torch.float64, device="cuda") for n in lens]
    a = torch.zeros((len(lens), 2), dtype=torch.float64, device="cuda")
    b = torch.zeros_like(a)
    for j, p in enumerate(parts):
        C.gpu_reduce(p.data_ptr(), p.shape[0], a[j].data_ptr(), st)
    C.gpu_reduce_batch([(p.data_ptr(), p.shape[0], b[j].data_ptr()) for j, p in enumerate(parts)], st)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert torch.equal(b[:, 0], torch.stack([p[:, 0].max() for p in parts]))
