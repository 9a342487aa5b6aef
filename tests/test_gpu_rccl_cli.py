"""The production RCCL calls on one GPU, captured in a hipGraph, through the native runtime (bin/wave3d).

``bin/wave3d ... --group P`` runs all P ranks of a decomposition in one process on one GPU with the rccl-self
transport: every rank owns a one-rank RCCL communicator and moves each halo message with ncclGroupStart / ncclSend /
ncclRecv / ncclGroupEnd on its high-priority side stream, joined to the compute stream with the same events as the
multi-process path; the error logs go through ncclAllGather. The binary runs on the system ROCm 7.2 runtime (HIP +
RCCL), which captures these multi-stream schedules, so solve 1 runs eagerly (RCCL connects), solve 2 is captured and the
later ones replay the graph. The dumped fields must be BIT-identical to the single-GPU solve and the printed error lines
identical (the reference's 1-GPU log == 2-GPU log property, report.pdf p.15-16).
"""
import json
import os
import subprocess

import numpy as np
import pytest

from mpi_cuda_amd import ProblemSpec
from mpi_cuda_amd.solver import Solver

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "bin", "wave3d")


def _single(N, K, check_every=2):
    s = Solver(ProblemSpec(N=N, tau=1e-3, K=K, check_every=check_every), backend="hip", device=0)
    r = s.run()
    return r, s.global_field(0).numpy()


def _group(tmp_path, N, K, world, decomp, transport="rccl-self", extra=()):
    prefix = str(tmp_path / "f")
    js = str(tmp_path / "g.json")
    cmd = [CLI, str(N), "0.001", str(K), "1", "--group", str(world), "--group-transport", transport, "--decomp",
           decomp, "--warmup", "2", "--repeat", "2", "--dump", prefix, "--json", js, "--quiet", *extra]
    out = subprocess.run(cmd, check=True, timeout=120, capture_output=True, text=True).stdout
    meta = json.loads(open(js).read())
    field = np.zeros((N + 1,) * 3)
    for r in range(world):
        m = json.loads(open(f"{prefix}.rank{r}.json").read())
        nx, ny, nz = m["shape"]
        x0, y0, z0 = m["offset"]
        field[x0:x0 + nx, y0:y0 + ny, z0:z0 + nz] = np.fromfile(f"{prefix}.rank{r}.bin").reshape(nx, ny, nz)
    return meta, field, out


@pytest.mark.parametrize("world,decomp,K", [(2, "slab", 20), (4, "slab", 20), (8, "slab", 9), (3, "slab", 11),
                                            (4, "2x2x1", 9), (8, "2x2x2", 10), (6, "1x2x3", 9)])
def test_rccl_self_graph_bitexact(gpu, tmp_path, world, decomp, K):
    N = 70
    r1, f1 = _single(N, K)
    meta, f, _ = _group(tmp_path, N, K, world, decomp)
    assert meta["transport"] == "rccl-self" and meta["rccl_comms"] == world
    assert meta["graph"] is True  # captured (ROCm 7.2 runtime), RCCL kernels inside the graph
    assert np.array_equal(f, f1)
    assert [s[0] for s in meta["steps"]] == r1.steps
    for (n, m, e), m1, e1 in zip(meta["steps"], r1.max_err, r1.rms_err):
        assert m == pytest.approx(m1, rel=1e-9) and e == pytest.approx(e1, rel=1e-9)


@pytest.mark.parametrize("extra", [("--no-overlap",), ("--poison-ghosts",), ("--temporal", "1"),
                                   ("--no-tb", "--deep-min-planes", "3")])
def test_rccl_self_graph_schedules(gpu, tmp_path, extra):
    """Late-exchange deep-tb (no overlap), NaN-poisoned ghosts, single steps and two-step deep halos, captured."""
    N, K = 66, 10
    _, f1 = _single(N, K)
    meta, f, _ = _group(tmp_path, N, K, 3, "slab", extra=extra)
    assert meta["graph"] is True and np.array_equal(f, f1)


def test_loopback_graph_bitexact(gpu, tmp_path):
    _, f1 = _single(70, 9)
    meta, f, _ = _group(tmp_path, 70, 9, 4, "2x2x1", transport="loopback")
    assert meta["graph"] is True and meta["rccl_comms"] == 0 and np.array_equal(f, f1)


@pytest.mark.parametrize("world,decomp,K", [(4, "2x2x1", 20), (8, "2x2x2", 20), (4, "1x2x2", 9), (6, "3x2x1", 12)])
def test_rccl_self_block_deep_tb_graph(gpu, tmp_path, world, decomp, K):
    """3-D block deep-tb ranks (S-deep ghosts, faces + edges + corners to up to 26 neighbours in one RCCL group),
    captured with RCCL inside the graph: bit-identical to one GPU, also with poisoned ghost regions."""
    N = 66
    _, f1 = _single(N, K)
    for extra in ((), ("--poison-ghosts",)):
        meta, f, _ = _group(tmp_path, N, K, world, decomp, extra=extra)
        assert meta["schedule"] == "deep-tb-block" and meta["graph"] is True
        assert np.array_equal(f, f1)


def test_cli_traffic_line_and_json(gpu, tmp_path):
    """Effective GB/s: the CLI prints the schedule's compulsory field traffic and halo volume per
    solve and puts both (and the GB/s) into --json; a fake slab rank of 2 sends 5 + 3 planes after each pass (5 + 4
    with --no-ghost-store)."""
    js = str(tmp_path / "one.json")
    out = subprocess.run([CLI, "128", "0.001", "20", "1", "--repeat", "2", "--warmup", "1", "--json", js, "--quiet"],
                         check=True, timeout=120, capture_output=True, text=True).stdout
    m = json.loads(open(js).read())
    # (analytic 4-step start writes 2 fields, three 5-step passes read 2 and write 2)
    assert m["field_bytes"] == (2 + 3 * 4) * 127 ** 3 * 8 and m["halo_bytes"] == 0
    assert m["effective_gbs"] == pytest.approx(m["field_bytes"] / m["solve_s"] / 1e9, rel=1e-6)
    assert "Traffic: " in out and "GB/s effective" in out
    js = str(tmp_path / "fake.json")
    out = subprocess.run([CLI, "128", "0.001", "20", "1", "--fake-rank", "0/2", "--repeat", "2", "--warmup", "1",
                          "--json", js, "--quiet"], check=True, timeout=120, capture_output=True, text=True).stdout
    m = json.loads(open(js).read())
    # three exchanges on the one face: 5 planes of u^{n+5} and 3 of u^{n+4} (the pass stores the 4th itself: ghost_store)
    plane_bytes = m["halo_bytes"] / (3 * 8)
    assert m["halo_bytes"] > 0 and plane_bytes == int(plane_bytes) and plane_bytes >= 129 * 129 * 8
    assert "Traffic (this rank): " in out
    subprocess.run([CLI, "128", "0.001", "20", "1", "--fake-rank", "0/2", "--repeat", "2", "--warmup", "1",
                    "--json", js, "--quiet", "--no-ghost-store"], check=True, timeout=120, capture_output=True)
    assert json.loads(open(js).read())["halo_bytes"] == m["halo_bytes"] * 9 / 8  # 5 + 4 planes per exchange


@pytest.mark.parametrize("world,decomp,N", [(4, "2x2x1", 66), (8, "2x2x2", 77), (6, "1x2x3", 71), (8, "2x2x2", 128)])
def test_rccl_self_block_p2_five_step_passes(gpu, tmp_path, world, decomp, N):
    """3-D block ranks with the exchange after each pass run the pair-tiled 5-step passes over their whole box (y/z
    ghosts 5 deep, the z-face pack by the pack kernel): bit-identical to one GPU, also with NaN-poisoned ghosts. Odd
    extents put a pair across a block's last z node (its second node lands in the ghost the next exchange rewrites)."""
    K = 20
    _, f1 = _single(N, K)
    for extra in (("--no-overlap",), ("--no-overlap", "--poison-ghosts")):
        meta, f, _ = _group(tmp_path, N, K, world, decomp, extra=extra)
        assert meta["schedule"] == "deep-tb-block" and meta["temporal"] == 5 and meta["graph"] is True
        assert np.array_equal(f, f1)


@pytest.mark.parametrize("extra", [[], ["--fake-traffic"]])
def test_fake_rank_bench_block_is_pipelined(gpu, tmp_path, extra):
    """Round 6: run_batch enqueues the timed block's graph replays back to back for fake ranks (and RCCL ranks, whose
    error-log all-gather follows each replay on the same stream) instead of one host round trip per solve; the block
    completes, reports itself pipelined, and takes about the device time of the synchronised solves (whose own times
    leave the host gaps between solves out)."""
    js = str(tmp_path / "fb.json")
    subprocess.run([CLI, "256", "0.001", "20", "1", "--fake-rank", "1/4", "--decomp", "slab", "--no-overlap",
                    "--repeat", "5", "--warmup", "2", "--bench-steps", "10", "--json", js, "--quiet"] + extra,
                   check=True, timeout=120, capture_output=True)
    m = json.loads(open(js).read())
    assert m["bench_steps"] == 10 and m["bench_s"] > 0
    assert m["bench_pipelined"] is True
    assert m["bench_s"] / 10 < 1.5 * m["mean_s"]
    env = dict(os.environ, W3D_BENCH_SYNC_EACH="1")
    subprocess.run([CLI, "256", "0.001", "20", "1", "--fake-rank", "1/4", "--decomp", "slab", "--no-overlap",
                    "--repeat", "2", "--warmup", "1", "--bench-steps", "3", "--json", js, "--quiet"] + extra,
                   check=True, timeout=120, capture_output=True, env=env)
    assert json.loads(open(js).read())["bench_pipelined"] is False
