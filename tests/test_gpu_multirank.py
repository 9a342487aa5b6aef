"""Multi-rank native GPU path on ONE GPU.

RCCL refuses two ranks of one communicator on one device, so the production C++ multi-rank code (shell/interior split,
halo plans, pack/unpack kernels, side-stream overlap, event ordering) is exercised through the in-process GpuGroup:
every rank of the decomposition lives in this process. Two transports move the halos:
  * loopback  — device copies;
  * rccl-self — the production RCCL calls (ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd on the rank's
    high-priority side stream, ncclAllGather of the error log), each rank over its own one-rank communicator.
Both run eager (first solve) and captured in one hipGraph (later solves). The decomposed result must be BIT-identical
to the single-GPU solve (the reference's "1-GPU log == 2-GPU log" property, report.pdf p.15-16)."""
import math
import os
import subprocess
import sys

import pytest
import torch

from mpi_cuda_amd import ProblemSpec
from mpi_cuda_amd.solver import Solver

pytestmark = pytest.mark.gpu

CASES = [(2, "slab"), (3, "slab"), (8, "slab"), (4, "block"), (8, "2x2x2"), (6, "1x2x3"), (4, "1x1x4"), (12, "block")]


@pytest.fixture(scope="module")
def single():
    spec = ProblemSpec(N=70, tau=1e-3, K=9, check_every=2)  # K odd: single-step schedule
    s = Solver(spec, backend="hip", device=0)
    r = s.run()
    return spec, r, s.global_field(0), s.global_field(1)


TRANSPORTS = ["loopback", "rccl-self"]


def _same(r, r1):
    assert r.finite and r.steps == r1.steps
    assert r.max_err == r1.max_err
    for a, b in zip(r.rms_err, r1.rms_err):
        assert math.isclose(a, b, rel_tol=1e-12)


@pytest.mark.parametrize("transport", TRANSPORTS)
@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("world,decomp", CASES)
def test_group_bitexact(gpu, single, world, decomp, overlap, transport):
    """Single-step schedule (slab and block decompositions, packed y/z faces): eager, then graph-captured."""
    spec, r1, f0, f1 = single
    g = Solver(spec, backend="hip", transport=transport, world=world, rank=0, decomp=decomp, overlap=overlap,
               device=0)
    for it in range(3):  # run 0 eager (RCCL connects), run 1 captures the group graph, run 2 replays it
        r = g.run()
        _same(r, r1)
        assert torch.equal(g.global_field(0), f0)
        assert torch.equal(g.global_field(1), f1)
    # inside a torch process the HIP runtime is PyTorch's 7.0, which cannot capture these multi-stream graphs: the
    # group then runs eagerly (the captured variant is covered through the native CLI, test_gpu_rccl_cli.py)
    assert g.native.graph_enabled == gpu.runtime_versions()["multistream_capture_safe"]


def test_rccl_self_communicators(gpu):
    """Every in-process rank owns a one-rank RCCL communicator (ncclCommCount == 1) that passed the all-reduce
    self-test in its constructor; the group graph holds the RCCL kernels."""
    spec = ProblemSpec(N=40, tau=1e-3, K=6)
    g = Solver(spec, backend="hip", transport="rccl-self", world=4, rank=0, decomp="2x2x1", device=0)
    assert g.native.comm_counts() == [1, 1, 1, 1]
    assert g.native.transport == "rccl-self"
    r1 = g.run()
    r2 = g.run()
    assert r1.max_err == r2.max_err


def test_loopback_repeat_and_tilings(gpu, single):
    spec, r1, f0, _ = single
    for tiling in (dict(variant=0, ty=8), dict(variant=1, rows=4), dict(variant=1, rows=1)):
        g = Solver(spec, backend="hip", transport="loopback", world=8, rank=0, decomp="2x2x2", device=0,
                   tiling=tiling)
        g.run()
        r = g.run()
        assert r.max_err == r1.max_err
        assert torch.equal(g.global_field(0), f0)


_WORKER = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["ROOT"])
from mpi_cuda_amd import ProblemSpec
from mpi_cuda_amd.solver import Solver
dist.init_process_group("gloo")
spec = ProblemSpec(N=40, tau=1e-3, K=6)
s = Solver(spec, backend="hip", transport="torch", decomp=os.environ["DECOMP"], device=0, stage_via_host=True)
r = s.run()
f = s.owned_field(0)
torch.save({"err": (r.max_err, r.rms_err), "f": f, "rank": dist.get_rank()}, os.environ["OUT"] + f".{dist.get_rank()}.pt")
dist.destroy_process_group()
"""


@pytest.mark.parametrize("decomp", ["slab", "1x2x1"])
def test_torch_transport_two_processes_share_gpu(gpu, tmp_path, decomp):
    """Python step loop + HIP kernels + torch.distributed (gloo, host-staged) across 2 processes on one GPU."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "w.py"
    script.write_text(_WORKER)
    env = dict(os.environ, ROOT=root, OUT=str(tmp_path / "res"), DECOMP=decomp)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(29600 + (os.getpid() % 200)), str(script)]
    subprocess.run(cmd, env=env, check=True, timeout=300)
    spec = ProblemSpec(N=40, tau=1e-3, K=6)
    ref = Solver(spec, backend="hip", device=0)
    rr = ref.run()
    full = ref.global_field(0)
    for rank in range(2):
        d = torch.load(str(tmp_path / f"res.{rank}.pt"), weights_only=True)
        assert d["err"][0] == rr.max_err
        from mpi_cuda_amd.parallel.decomp import plan

        p = plan(40, 2, rank, decomp)
        x0, x1, y0, y1, z0, z1 = p.box
        assert torch.equal(d["f"], full[x0:x1, y0:y1, z0:z1])


@pytest.mark.parametrize("transport", TRANSPORTS)
@pytest.mark.parametrize("world,decomp,overlap", [(4, "2x2x1", True), (8, "2x2x2", False), (3, "slab", True)])
def test_poisoned_ghosts_still_bitexact(gpu, single, world, decomp, overlap, transport):
    """NaN-filled ghost layers before every exchange: any ghost node the stencil reads without it having been
    received would poison the error norms. Results stay bit-identical, so every read ghost is delivered."""
    spec, r1, f0, _ = single
    g = Solver(spec, backend="hip", transport=transport, world=world, rank=0, decomp=decomp, overlap=overlap,
               device=0, poison_ghosts=True, debug_sync=True)
    r = g.run()
    assert r.finite and r.max_err == r1.max_err
    assert torch.equal(g.global_field(0), f0)


@pytest.mark.parametrize("tb", [True, False])
def test_phase_timers(gpu, tb):
    spec = ProblemSpec(N=96, tau=1e-3, K=10)
    s = Solver(spec, backend="hip", device=0, timers=True, tb=tb)
    r = s.run()
    ph = r.extra["phases"]
    assert ph["compute_ms"] > 0 and ph["check_ms"] > 0
    # the LDS schedule's first pass computes u⁰, u¹ itself: no separate init kernel
    assert (ph["init_ms"] == 0) if tb else (ph["init_ms"] > 0)
    ref = Solver(spec, backend="hip", device=0, tb=tb).run()
    assert r.max_err == ref.max_err
    # per-unit trace: the units cover every step after the init, and their compute sums to the phase total
    tr = r.extra["trace"]
    assert tr and tr[-1]["n"] + tr[-1]["steps"] == spec.K
    assert all(a["n"] + a["steps"] == b["n"] for a, b in zip(tr, tr[1:]))
    assert math.isclose(sum(u["compute_ms"] for u in tr), ph["compute_ms"], rel_tol=1e-6)


def test_cli_trace_deep_tb(gpu, tmp_path):
    """--trace on a fake slab rank (deep-tb schedule): one JSON line per pass with shell, exchange and compute."""
    import json

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "trace.jsonl"
    subprocess.run([os.path.join(root, "bin", "wave3d"), "128", "0.001", "20", "1", "--fake-rank", "1/3",
                    "--trace", str(out), "--quiet"], check=True, timeout=120)
    rows = [json.loads(x) for x in (tmp_path / "trace.jsonl.rank1").read_text().splitlines()]  # per-rank file
    assert rows and all(r["schedule"] == "deep-tb" for r in rows)
    assert rows[0]["n"] == 1 and rows[-1]["n"] + rows[-1]["steps"] == 20
    assert all(r["shell_ms"] > 0 for r in rows[:-1]) and rows[-1]["shell_ms"] == 0  # no exchange after the last


@pytest.fixture(scope="module")
def single_even():
    spec = ProblemSpec(N=66, tau=1e-3, K=10, check_every=2)
    s = Solver(spec, backend="hip", device=0)
    r = s.run()
    return spec, r, s.global_field(0), s.global_field(1)


@pytest.mark.parametrize("transport", TRANSPORTS)
@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("world", [2, 3, 4, 8, 16])
def test_deep_halo_temporal_blocking_bitexact(gpu, single_even, world, overlap, transport):
    """Slab ranks with 2-deep x halos run the fused two-step kernel (one exchange of 3 planes per face per pass):
    bit-identical to one GPU, also with NaN-poisoned ghosts, eager and graph-captured."""
    spec, r1, f0, f1 = single_even
    g = Solver(spec, backend="hip", transport=transport, world=world, rank=0, decomp="slab", overlap=overlap,
               device=0, poison_ghosts=True, deep_min_planes=3, tb=False)
    assert g.native.mode() == "deep-halo"
    for _ in range(3):
        r = g.run()
        _same(r, r1)
        assert torch.equal(g.global_field(0), f0)
        assert torch.equal(g.global_field(1), f1)


@pytest.mark.parametrize("transport", TRANSPORTS)
@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("K,check_every,temporal", [(10, 2, 4), (20, 2, 4), (9, 1, 4), (12, 3, 3), (11, 2, 2)])
def test_deep_tb_bitexact(gpu, world, overlap, K, check_every, temporal, transport):
    """Slab ranks on the LDS S-step kernel with S-deep x halos: each pass computes the planes its neighbours need
    first (shells), sends S planes of u^{n+S} and S−1 of u^{n+S−1} per face on the side stream while the interior
    pass runs. Bit-identical to one GPU, with NaN-poisoned ghosts; odd-level checks and a checked step 1 (no
    analytic start) included."""
    spec = ProblemSpec(N=66, tau=1e-3, K=K, check_every=check_every)
    ref = Solver(spec, backend="hip", device=0, temporal=1)
    r1 = ref.run()
    f0, f1 = ref.global_field(0), ref.global_field(1)
    g = Solver(spec, backend="hip", transport=transport, world=world, rank=0, decomp="slab", overlap=overlap,
               device=0, poison_ghosts=True, tb_min_planes=2 * temporal, temporal=temporal)
    assert g.native.mode() == "deep-tb"
    for _ in range(3):  # eager, capture, replay
        r = g.run()
        _same(r, r1)
        assert torch.equal(g.global_field(0), f0)
        assert torch.equal(g.global_field(1), f1)


def test_schedule_modes(gpu):
    even = ProblemSpec(N=40, tau=1e-3, K=10)
    odd_check = ProblemSpec(N=40, tau=1e-3, K=10, check_every=1)
    assert Solver(even, backend="hip", device=0).native.mode == "fused-single"
    assert Solver(even, backend="hip", device=0, temporal=1).native.mode == "single-step"
    assert Solver(even, backend="hip", transport="loopback", world=4, rank=0, decomp="2x2x1",
                  device=0).native.mode() == "deep-tb-block"  # S-deep ghosts on x and y
    assert Solver(even, backend="hip", transport="loopback", world=4, rank=0, decomp="2x2x1", temporal=1,
                  device=0).native.mode() == "single-step"
    assert Solver(even, backend="hip", transport="loopback", world=16, rank=0, decomp="8x2x1",
                  device=0).native.mode() == "single-step"  # x boxes of 5 planes < 2·temporal
    assert Solver(odd_check, backend="hip", transport="loopback", world=2, rank=0, decomp="slab",
                  device=0, deep_min_planes=3, tb=False).native.mode() == "single-step"  # odd checks: no pairs
    assert Solver(odd_check, backend="hip", transport="loopback", world=2, rank=0, decomp="slab",
                  device=0).native.mode() == "deep-tb"  # the LDS passes check any level
    assert Solver(even, backend="hip", transport="loopback", world=2, rank=0, decomp="slab",
                  device=0, deep_min_planes=3, tb=False).native.mode() == "deep-halo"
    assert Solver(even, backend="hip", transport="loopback", world=2, rank=0, decomp="slab",
                  device=0, tb=False).native.mode() == "single-step"  # 20 planes per rank < default 96
    assert Solver(even, backend="hip", transport="loopback", world=2, rank=0, decomp="slab",
                  device=0).native.mode() == "deep-tb"  # 20 planes per rank >= default 16
    assert Solver(even, backend="hip", transport="loopback", world=4, rank=0, decomp="slab",
                  device=0).native.mode() == "single-step"  # 10 planes per rank < 16


@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("world,decomp", [(4, "2x2x1"), (4, "1x2x2"), (8, "2x2x2"), (6, "3x2x1"), (4, "2x1x2")])
@pytest.mark.parametrize("K,check_every,temporal", [(20, 2, 4), (9, 1, 4), (12, 3, 3), (11, 2, 2)])
def test_block_deep_tb_bitexact(gpu, world, decomp, overlap, K, check_every, temporal):
    """3-D block ranks on the LDS S-step kernel with S-deep ghosts on every split axis: one exchange of faces, edges and
    corners (packed per neighbour by k_box_copy) between passes, small boxes split into x chunks. Bit-identical to one
    GPU with NaN-poisoned ghost regions; odd-level checks and a checked step 1 (no analytic start) included."""
    spec = ProblemSpec(N=66, tau=1e-3, K=K, check_every=check_every)
    ref = Solver(spec, backend="hip", device=0, temporal=1)
    r1 = ref.run()
    f0, f1 = ref.global_field(0), ref.global_field(1)
    g = Solver(spec, backend="hip", transport="loopback", world=world, rank=0, decomp=decomp, overlap=overlap,
               device=0, poison_ghosts=True, temporal=temporal)
    assert g.native.mode() == "deep-tb-block"
    for _ in range(2):
        r = g.run()
        _same(r, r1)
        assert torch.equal(g.global_field(0), f0)
        assert torch.equal(g.global_field(1), f1)


@pytest.mark.parametrize("transport", ["loopback", "rccl-self", "sdma"])
@pytest.mark.parametrize("world,decomp,N", [(27, "3x3x3", 100), (9, "1x3x3", 100), (27, "3x3x3", 140),
                                            (8, "2x2x2", 70), (12, "3x2x2", 100)])
def test_block_overlap_geometries(gpu, world, decomp, N, transport):
    """Block ranks with overlap compute the regions their neighbours receive first (border tile rows/columns, the
    core's x-face slabs) on the side stream while the core runs on s0. Box sizes whose last tile row is a remainder
    narrower than the halo (N=100 over 3: 33 nodes = 32 + 1) put the border on the w rows next to the face instead."""
    spec = ProblemSpec(N=N, tau=1e-3, K=20)
    ref = Solver(spec, backend="hip", device=0, temporal=1)
    r1 = ref.run()
    f0 = ref.global_field(0)
    g = Solver(spec, backend="hip", transport=transport, world=world, rank=0, decomp=decomp, device=0,
               overlap=True, poison_ghosts=transport != "rccl-self")
    assert g.native.mode() == "deep-tb-block"
    for _ in range(2):
        r = g.run()
        _same(r, r1)
        assert torch.equal(g.global_field(0), f0)


@pytest.mark.parametrize("transport", ["loopback", "rccl-self", "sdma"])
@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("world,decomp,N,overlap", [(8, "2x2x2", 70, True), (4, "1x2x2", 66, False),
                                                    (12, "3x2x2", 100, True), (27, "3x3x3", 100, False)])
def test_block_fused_zface_pack(gpu, world, decomp, N, overlap, transport, fused):
    """The z-face message parts are written by the pass itself (TbPack) or, with fused_pack=False,
    gathered by the pack kernel like the x / y faces: both bit-identical to one GPU with NaN-poisoned ghosts (a z-face
    node the pass failed to store would arrive as a stale value of an earlier pass). The fused pack is k_leapfrog_tb's
    (S ≤ 4): with the pair-tiled pass on (the default) block ranks pack with the pack kernel, so fused=True runs the
    older kernel (tiling_tb p2 off)."""
    spec = ProblemSpec(N=N, tau=1e-3, K=20)
    ref = Solver(spec, backend="hip", device=0, temporal=1)
    r1 = ref.run()
    f0 = ref.global_field(0)
    g = Solver(spec, backend="hip", transport=transport, world=world, rank=0, decomp=decomp, device=0,
               overlap=overlap, poison_ghosts=transport != "rccl-self", fused_pack=fused,
               tiling_tb={"p2": False} if fused else None, temporal=4 if fused else 5)
    assert g.native.mode() == "deep-tb-block"
    for _ in range(2):
        r = g.run()
        _same(r, r1)
        assert torch.equal(g.global_field(0), f0)


@pytest.mark.parametrize("transport", ["loopback", "sdma"])
@pytest.mark.parametrize("world,decomp,K,temporal", [(2, "1x1x2", 10, 4), (8, "2x2x2", 10, 4), (2, "1x1x2", 20, 3),
                                                     (4, "1x2x2", 11, 4)])
def test_block_fused_zface_pack_mixed_depths(gpu, world, decomp, K, temporal, transport):
    """Schedules whose exchanges change depth (K = 10: passes of 2, 3, 4 steps, exchanges of depth 3 then 4): the
    fused z-face pack leaves the global-boundary entries of its message parts at their initial zero, so each depth
    needs its own send region — a shared one carried the previous depth's values into those entries (a regression:
    bit-identical before only for uniform-depth schedules)."""
    spec = ProblemSpec(N=70, tau=1e-3, K=K)
    ref = Solver(spec, backend="hip", device=0, temporal=1)
    r1 = ref.run()
    f0 = ref.global_field(0)
    g = Solver(spec, backend="hip", transport=transport, world=world, rank=0, decomp=decomp, device=0, overlap=False,
               poison_ghosts=True, fused_pack=True, temporal=temporal, tiling_tb={"p2": False})
    for _ in range(2):
        r = g.run()
        _same(r, r1)
        assert torch.equal(g.global_field(0), f0)


@pytest.mark.parametrize("transport", ["loopback", "sdma"])
@pytest.mark.parametrize("temporal", [2, 3, 4, 5])
@pytest.mark.parametrize("world,decomp,N", [(8, "2x2x2", 70), (4, "2x2x1", 66), (4, "1x2x2", 67), (27, "3x3x3", 100)])
def test_block_overlap_p2_bitexact(gpu, world, decomp, N, temporal, transport):
    """Round 6: overlapped 3-D block ranks run the pair-tiled pass (S = 2..5) on their shell and interior boxes, which
    are cut on whole 16-byte pairs (cpu.hpp deep_split), so no pass writes a node of another box. Bit-identical to one
    GPU with NaN-poisoned ghosts, eager and graph-replayed; N = 67 gives odd rank extents (remainder boxes widened to
    a whole pair), N = 100 over 3 a remainder tile row narrower than the halo. (K = 21: S = 2 needs an even number of
    steps after the analytic start.)"""
    spec = ProblemSpec(N=N, tau=1e-3, K=21)
    ref = Solver(spec, backend="hip", device=0, temporal=1)
    r1 = ref.run()
    f0, f1 = ref.global_field(0), ref.global_field(1)
    g = Solver(spec, backend="hip", transport=transport, world=world, rank=0, decomp=decomp, device=0,
               overlap=True, poison_ghosts=True, temporal=temporal)
    assert g.native.mode() == "deep-tb-block" and g.native.temporal() == temporal and g.native.overlapped()
    for _ in range(2):
        r = g.run()
        _same(r, r1)
        assert torch.equal(g.global_field(0), f0)
        assert torch.equal(g.global_field(1), f1)


@pytest.mark.parametrize("transport", ["loopback", "rccl-self", "sdma"])
@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("world,temporal,K", [(2, 5, 20), (3, 5, 21), (3, 4, 21), (4, 3, 21), (8, 2, 21)])
def test_slab_ghost_store_bitexact(gpu, world, temporal, K, overlap, transport):
    """Round 6: slab passes store u^{n+S−1} on the first ghost plane beyond each neighbour face themselves (they compute
    it anyway; SolverOptions.ghost_store), and the exchange sends S − 2 planes of that level instead of S − 1 (the 5-step
    passes' split stores reach the upper ghost plane with one more march iteration). Bit-identical to one GPU with
    NaN-poisoned ghosts, eager and replayed, on RCCL, loopback and copy-engine transports; with the option off the same
    result, and exactly one plane per face per exchange more."""
    spec = ProblemSpec(N=66, tau=1e-3, K=K)
    ref = Solver(spec, backend="hip", device=0, temporal=1)
    r1 = ref.run()
    f0, f1 = ref.global_field(0), ref.global_field(1)
    halo = {}
    for ghost in (True, False):
        g = Solver(spec, backend="hip", transport=transport, world=world, rank=0, decomp="slab", device=0,
                   overlap=overlap, poison_ghosts=True, temporal=temporal, tb_min_planes=2 * temporal,
                   ghost_store=ghost)
        assert g.native.mode() == "deep-tb" and g.native.temporal() == temporal
        for _ in range(2):
            r = g.run()
            _same(r, r1)
            assert torch.equal(g.global_field(0), f0)
            assert torch.equal(g.global_field(1), f1)
        halo[ghost] = g.native.traffic(1)["halo_bytes"]  # (rank 1: neighbours on both sides unless world = 2)
        plane_bytes = 8 * g.native.layout(1).plane
    # one plane per face per exchange (one after every pass but the last) fewer
    faces = 1 if world == 2 else 2
    exchanges = (halo[False] - halo[True]) / (faces * plane_bytes)
    assert exchanges == int(exchanges) and 2 <= exchanges <= K // 2
