"""End-to-end native GPU solver: golden log, oracle, bit-exact vs CPU, graph == eager, native code actually loaded."""
import math
import os

import pytest
import torch

from mpi_cuda_amd import ProblemSpec
from mpi_cuda_amd.models.wave3d import REFERENCE_LOG_512, oracle_errors
from mpi_cuda_amd.solver import Solver

pytestmark = pytest.mark.gpu


def test_native_extension_is_the_gpu_path(gpu):
    assert gpu.__file__.endswith(".so")
    assert gpu.gpu_arch().startswith("gfx950"), gpu.gpu_arch()


@pytest.mark.parametrize("N,K", [(48, 10), (65, 7), (128, 20)])
def test_gpu_matches_cpu_bitexact(gpu, N, K):
    spec = ProblemSpec(N=N, tau=1e-3, K=K, check_every=1)
    g = Solver(spec, backend="hip", device=0)
    rg = g.run()
    c = Solver(spec, backend="cpu")
    rc = c.run()
    assert rg.steps == rc.steps
    assert rg.max_err == rc.max_err
    for a, b in zip(rg.rms_err, rc.rms_err):
        assert math.isclose(a, b, rel_tol=1e-12)
    assert torch.equal(g.owned_field(0), c.owned_field(0))
    assert torch.equal(g.owned_field(1), c.owned_field(1))


@pytest.mark.parametrize("graph", [True, False])
def test_graph_and_eager_identical_and_repeatable(gpu, graph):
    spec = ProblemSpec(N=96, tau=1e-3, K=12)
    s = Solver(spec, backend="hip", device=0, graph=graph)
    r1 = s.run()
    f1 = s.owned_field(0)
    r2 = s.run()
    assert r1.max_err == r2.max_err and r1.rms_err == r2.rms_err
    assert torch.equal(f1, s.owned_field(0))
    ref = oracle_errors(spec)
    for n, m, e in zip(r1.steps, r1.max_err, r1.rms_err):
        assert math.isclose(m, ref[n][0], rel_tol=1e-6) and math.isclose(e, ref[n][1], rel_tol=1e-6)


def test_golden_log_512(gpu):
    """The reference's printed 512³ log (report.pdf p.15-16) to its 7 printed digits (±1 in the last place)."""
    spec = ProblemSpec(N=512, tau=1e-3, K=20)
    r = Solver(spec, backend="hip", device=0).run()
    assert r.steps == [n for n, _, _ in REFERENCE_LOG_512]
    for (n, m, e), gm, ge in zip(REFERENCE_LOG_512, r.max_err, r.rms_err):
        assert abs(gm - m) <= 1.5e-6 * m + 2e-17, (n, gm, m)
        assert abs(ge - e) <= 1.5e-6 * e + 2e-17, (n, ge, e)
    lines = r.lines()
    assert lines[-1] == "Step 20, t = 0.020000, Max Error = 3.960129e-09, L2 Error = 1.404229e-09"


@pytest.mark.parametrize("tiling", [dict(variant=0, ty=4), dict(variant=0, ty=16, xcd_remap=False),
                                    dict(variant=0, ty=8, nt_store=True), dict(variant=1, rows=1),
                                    dict(variant=1, rows=8, nt_store=True)])
def test_tilings_agree(gpu, tiling):
    spec = ProblemSpec(N=100, tau=1e-3, K=8)
    a = Solver(spec, backend="hip", device=0, tiling=dict(variant=1, rows=4))
    b = Solver(spec, backend="hip", device=0, tiling=tiling)
    ra, rb = a.run(), b.run()
    assert ra.max_err == rb.max_err
    assert torch.equal(a.owned_field(0), b.owned_field(0))


@pytest.mark.parametrize("N,K,ce", [(64, 20, 2), (65, 9, 3), (50, 7, 0), (48, 6, 1), (70, 13, 1)])
@pytest.mark.parametrize("temporal,tb", [(2, False), (2, True), (3, True), (4, True)])
def test_temporal_blocking_identical(gpu, N, K, ce, temporal, tb):
    """Every temporal-blocking schedule (two-step register kernel, 2..4-step LDS kernel with checks at any level)
    reproduces the single-step solve bit for bit."""
    spec = ProblemSpec(N=N, tau=1e-3, K=K, check_every=ce)
    a = Solver(spec, backend="hip", device=0, temporal=1)
    b = Solver(spec, backend="hip", device=0, temporal=temporal, tb=tb)
    ra, rb = a.run(), b.run()
    assert ra.steps == rb.steps and ra.max_err == rb.max_err
    for x, y in zip(ra.rms_err, rb.rms_err):
        assert math.isclose(x, y, rel_tol=1e-12)
    assert torch.equal(a.owned_field(0), b.owned_field(0))
    assert torch.equal(a.owned_field(1), b.owned_field(1))
    rb2 = b.run()
    assert rb2.max_err == rb.max_err


@pytest.mark.parametrize("temporal", [1, 2, 4])
@pytest.mark.parametrize("N,K,ce", [(60, 12, 2), (45, 2, 1), (50, 5, 1), (33, 1, 2)])
def test_init2_identical(gpu, temporal, N, K, ce):
    spec = ProblemSpec(N=N, tau=1e-3, K=K, check_every=ce)
    a = Solver(spec, backend="hip", device=0, temporal=temporal, init2=False)
    b = Solver(spec, backend="hip", device=0, temporal=temporal, init2=True)
    ra, rb = a.run(), b.run()
    assert ra.steps == rb.steps and ra.max_err == rb.max_err
    for x, y in zip(ra.rms_err, rb.rms_err):
        assert math.isclose(x, y, rel_tol=1e-12)
    assert torch.equal(a.owned_field(0), b.owned_field(0))
    assert torch.equal(a.owned_field(1), b.owned_field(1))


@pytest.mark.parametrize("N,L,tau,K,ce,temporal", [(64, 1.0, 1e-3, 1, 1, 4), (65, 1.0, 1e-3, 7, 3, 4),
                                                   (100, math.pi, 1e-3, 20, 2, 4), (127, 1.0, 1e-3, 50, 2, 4),
                                                   (129, 1.0, 1e-3, 33, 5, 2), (300, math.pi, 2e-3, 41, 4, 4)])
def test_oracle_sweep(gpu, N, L, tau, K, ce, temporal):
    """Odd/even N, L ∈ {1, π}, K up to 50 (more LDS passes than reduction regions), several check cadences and pass
    depths: the printed errors match the closed-form oracle and the CPU solver's (tools/oracle_sweep.py
    runs the full list)."""
    from mpi_cuda_amd.models.wave3d import oracle_errors

    spec = ProblemSpec(N=N, tau=tau, K=K, L=L, check_every=ce)
    r = Solver(spec, backend="hip", device=0, temporal=temporal).run()
    cpu = Solver(spec, backend="cpu").run()
    ref = oracle_errors(spec)
    assert r.steps == cpu.steps == [n for n in range(1, K + 1) if (ce and n % ce == 0) or n == K]
    assert r.max_err == cpu.max_err
    for n, m, e, ec in zip(r.steps, r.max_err, r.rms_err, cpu.rms_err):
        om, oe = ref[n]
        assert abs(m - om) <= 1e-5 * om and abs(e - oe) <= 1e-5 * oe
        assert math.isclose(e, ec, rel_tol=1e-12)


def test_traffic_accounting(gpu):
    """GpuSolver::traffic (SURVEY.md §5.5 effective GB/s): K = 20 on one rank is the analytic-start pass (4 steps,
    writes two levels) plus three 5-step passes (read two, write two) over the 63³ updated nodes; no halo."""
    spec = ProblemSpec(N=64, tau=1e-3, K=20)
    s = Solver(spec, backend="hip", device=0)
    s.run()
    t = s.traffic()
    assert t["field_bytes"] == (2 + 3 * 4) * 63 ** 3 * 8
    assert t["halo_bytes"] == 0


def test_run_batch_pipelined_logs(gpu):
    """GpuSolver::run_batch (bench.py's timed block): n graph replays enqueued back to back, each solve's log copied
    into its own pinned slot, one sync — every solve returns the same log as a synchronised run(), and the field after
    the batch is the single run()'s field bit for bit (also for a batch larger than the previous pinned buffer)."""
    spec = ProblemSpec(N=96, tau=1e-3, K=20)
    s = Solver(spec, backend="hip", device=0)
    r1 = s.run()  # (captures the graph)
    h1 = s.field_hash(0)
    for n in (3, 7):
        rs = s.run_batch(n)
        assert len(rs) == n
        for r in rs:
            assert r.steps == r1.steps and r.max_err == r1.max_err
            assert r.rms_err == r1.rms_err and r.solve_s > 0 and r.finite
        assert s.field_hash(0) == h1


def test_capture_guard_refuses_the_round4_split(gpu):
    """HIP 7.2's hipStreamEndCapture crashes (SIGSEGV in the runtime) when a stream forked from a
    non-origin stream waits on its sibling's event inside a capture (tools/probes/capture_probe3.hip modes 2 and 5,
    profiles/r5/capture/). Every cross-stream wait of a captured schedule goes through wave3d::capture::wait, which
    refuses that wait before it enters the capture; the production topology captures and replays. Run in bin/wave3d
    (the system ROCm 7.2 runtime: the HIP 7.0 runtime PyTorch bundles does not capture multi-stream schedules at all)."""
    import subprocess

    cli = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bin", "wave3d")

    def run(m):
        return subprocess.run([cli, "64", "0.001", "20", "--capture-selftest", str(m)], check=True, timeout=60,
                              capture_output=True, text=True).stdout

    assert "mode 0: ok" in run(0)
    out = run(2)
    assert "capture topology refused" in out and "sibling" in out
