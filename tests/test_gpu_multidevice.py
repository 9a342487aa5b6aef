"""Multi-GPU execution across REAL devices: skipped below 2 visible GPUs, run on a node.

Everything multi-rank elsewhere in tests/ runs on one GPU (in-process groups, or processes sharing the card). Here every
rank owns its own device, so these are the tests that exercise what one GPU cannot:
  * ncclCommInitRank with world > 1 (unique id through the rendezvous file) and RCCL P2P between devices;
  * hipIpcOpenMemHandle of another GPU's buffers + hipDeviceCanAccessPeer (the copy-engine transport over xGMI);
  * bench.py's multi-GPU contract line (one rank per GPU under torch.distributed.run).
Each solve must be BIT-identical to the one-GPU solve (the reference's 1-GPU log == 2-GPU log, report.pdf p.15-16
§4.3.2) and must say which communicator / transport it used.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "bin", "wave3d")


def _ndev() -> int:
    import torch

    return torch.cuda.device_count()  # (does not initialise the GPU on this image)


NDEV = _ndev()
needs2 = pytest.mark.skipif(NDEV < 2, reason=f"needs >= 2 visible GPUs ({NDEV} visible)")
WORLDS = sorted({2, min(8, NDEV)}) if NDEV >= 2 else [2]
# (a lost peer ends a solve within W3D_TIMEOUT_S / 2 on the device, the host gives up at W3D_TIMEOUT_S)
ENV = dict(os.environ, W3D_TIMEOUT_S="30", W3D_SPAWN_GRACE_S="10")

# The whole file runs within BUDGET_S of wall time even if every test hangs once: each subprocess
# gets min(its own limit, what is left), and once less than MIN_S is left the remaining tests skip, so a first contact
# that goes wrong cannot eat the round's GPU test budget and hide the other files' results.
BUDGET_S, MIN_S = 300.0, 20.0
_T0 = []


def _limit(own: float) -> float:
    import time

    if not _T0:
        _T0.append(time.monotonic())
    left = BUDGET_S - (time.monotonic() - _T0[0])
    if left < MIN_S:
        pytest.skip(f"test_gpu_multidevice.py wall budget ({BUDGET_S:.0f} s) spent")
    return min(own, left)


def _read_dump(prefix, world, N):
    field = np.zeros((N + 1,) * 3)
    for r in range(world):
        path = f"{prefix}.rank{r}" if world > 1 else prefix
        m = json.loads(open(f"{path}.json").read())
        nx, ny, nz = m["shape"]
        x0, y0, z0 = m["offset"]
        field[x0:x0 + nx, y0:y0 + ny, z0:z0 + nz] = np.fromfile(f"{path}.bin").reshape(nx, ny, nz)
    return field


@pytest.fixture(scope="module")
def one_gpu(tmp_path_factory):
    if NDEV < 2:
        pytest.skip(f"needs >= 2 visible GPUs ({NDEV} visible)")
    d = tmp_path_factory.mktemp("one")
    N, K = 192, 20
    js = str(d / "one.json")
    subprocess.run([CLI, str(N), "0.001", str(K), "1", "--dump", str(d / "one"), "--json", js, "--quiet"], check=True,
                   timeout=_limit(60), env=ENV)
    return N, K, _read_dump(str(d / "one"), 1, N), json.loads(open(js).read())


@needs2
@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("decomp,transport,extra", [
    ("slab", "rccl", ()), ("slab", "rccl", ("--no-overlap",)), ("slab", "sdma", ()),
    ("block", "rccl", ()), ("block", "sdma", ()), ("slab", "push", ("--no-overlap",))])
def test_ranks_on_distinct_gpus_bitexact(one_gpu, tmp_path, world, decomp, transport, extra):
    """`bin/wave3d --np P`: P processes, one GPU each, an RCCL communicator of P ranks; the halos go by RCCL P2P, by
    the copy engines over xGMI (IPC-mapped peer memory) or by the push transport. Dumped u^K identical to one GPU."""
    N, K, f1, m1 = one_gpu
    if decomp == "block" and world < 4:
        pytest.skip("2 ranks: the block decomposition is the slab")
    prefix, js = str(tmp_path / "p"), str(tmp_path / "p.json")
    cmd = [CLI, str(N), "0.001", str(K), "1", "--np", str(world), "--decomp", decomp, "--transport", transport,
           "--warmup", "1", "--repeat", "3", "--dump", prefix, "--json", js, "--quiet", *extra]
    subprocess.run(cmd, check=True, timeout=_limit(60), env=ENV)
    meta = json.loads(open(js).read())
    assert meta["ranks"] == world and meta["rccl_nranks"] == world
    assert meta["transport"] == transport
    assert np.array_equal(_read_dump(prefix, world, N), f1)
    assert [s[1] for s in meta["steps"]] == [s[1] for s in m1["steps"]]


@needs2
@pytest.mark.parametrize("world", WORLDS)
def test_autotune_across_gpus(one_gpu, tmp_path, world):
    """The autotune on real devices: every candidate that survives reproduces the one-GPU log, RCCL reports P ranks."""
    N, K, f1, m1 = one_gpu
    prefix, js = str(tmp_path / "a"), str(tmp_path / "a.json")
    subprocess.run([CLI, str(N), "0.001", str(K), "1", "--np", str(world), "--autotune", "--dump", prefix, "--json", js,
                    "--quiet"], check=True, timeout=_limit(120), env=ENV)
    meta = json.loads(open(js).read())
    assert meta["rccl_nranks"] == world and len(meta["autotune_s"]) >= 3
    assert np.array_equal(_read_dump(prefix, world, N), f1)


@needs2
def test_bench_two_gpus_contract(tmp_path):
    """bench.py at 2 GPUs under torch.distributed.run: one JSON line, correct (oracle + reference digits), two distinct
    GPUs, an RCCL communicator of 2 ranks, and no rehearsal marker."""
    out = tmp_path / "b.jsonl"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(29900 + os.getpid() % 90), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
           "5", "--warmup", "2", "--out", str(out)]
    subprocess.run(cmd, check=True, timeout=_limit(120), env=ENV)
    line = json.loads(out.read_text().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["distinct_gpus"] == 2 and line["rccl_nranks"] == 2
    assert "rehearsal" not in line and line["correct"] is True
    assert line["final_max_err"] == pytest.approx(3.960129e-09, rel=1e-6)
    assert "fallback_schedule" not in line  # (the main run, not the conservative retry)


@needs2
@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("extra", [(), ("--no-overlap",), ("--no-ghost-store",)])
def test_pipelined_bench_block_across_gpus(one_gpu, tmp_path, world, extra):
    """Round 6: the timed block of P RCCL ranks on P GPUs enqueues its graph replays back to back, each followed by the
    error-log all-gather, and synchronises once (run_batch); its last solve's log and u^K equal one GPU's."""
    N, K, f1, m1 = one_gpu
    prefix, js = str(tmp_path / "b"), str(tmp_path / "b.json")
    subprocess.run([CLI, str(N), "0.001", str(K), "1", "--np", str(world), "--decomp", "slab", "--warmup", "2",
                    "--repeat", "1", "--bench-steps", "10", "--dump", prefix, "--json", js, "--quiet", *extra],
                   check=True, timeout=_limit(90), env=ENV)
    meta = json.loads(open(js).read())
    assert meta["rccl_nranks"] == world and meta["bench_pipelined"] is True and meta["bench_s"] > 0
    assert [s[1] for s in meta["steps"]] == [s[1] for s in m1["steps"]]
    assert np.array_equal(_read_dump(prefix, world, N), f1)


@needs2
def test_peer_access_between_all_visible_gpus(gpu):
    """xGMI peer access, which the copy-engine and push transports need between every pair of ranks' devices."""
    import torch

    n = torch.cuda.device_count()
    for a in range(n):
        for b in range(n):
            if a != b:
                assert torch.cuda.can_device_access_peer(a, b), (a, b)


@needs2
def test_multidevice_group_bitexact(gpu):
    """One process, one host thread per GPU (GpuGroup 'multi-device': an RCCL communicator over every visible device
    from ncclCommInitAll): the production schedules across real devices without a launcher."""
    from mpi_cuda_amd import ProblemSpec
    from mpi_cuda_amd.solver import Solver
    import torch

    _limit(MIN_S)  # (in-process: bounded by pytest's per-test timeout; skipped once the file's budget is spent)
    spec = ProblemSpec(N=128, tau=1e-3, K=20)
    ref = Solver(spec, backend="hip", device=0)
    r1 = ref.run()
    f0 = ref.global_field(0)
    world = min(8, torch.cuda.device_count())
    for decomp in ("slab", "block"):
        for ce in (False, True):
            g = Solver(spec, backend="hip", transport="multi-device", world=world, rank=0, decomp=decomp,
                       copy_engines=ce)
            for _ in range(3):
                r = g.run()
                assert r.max_err == r1.max_err
                assert torch.equal(g.global_field(0), f0)


def test_multidevice_group_one_gpu(gpu):
    """The multi-device group's plumbing on whatever is visible (one GPU: ncclCommInitAll over one device, one
    thread): the path runs everywhere, not only on a node."""
    from mpi_cuda_amd import ProblemSpec
    from mpi_cuda_amd.solver import Solver
    import torch

    spec = ProblemSpec(N=64, tau=1e-3, K=10)
    ref = Solver(spec, backend="hip", device=0)
    r1 = ref.run()
    g = Solver(spec, backend="hip", transport="multi-device", world=1, rank=0)
    for _ in range(3):
        r = g.run()
        assert r.max_err == r1.max_err
    assert torch.equal(g.global_field(0), ref.global_field(0))
