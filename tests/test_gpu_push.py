"""The push halo transport of the slab LDS passes (SolverOptions::push, TbPush in kernels.hpp).

Each pass stores the face planes its neighbours read as ghosts a second time, straight into their fine-grained staging
(over xGMI on a node), reads its own ghosts from its staging, and orders itself against its neighbours with flags in
uncached memory: it waits for both neighbours' previous pass, then raises its slot in their flags once all its stores
are visible. No exchange phase, no RCCL kernels, no shell launches; with overlap the pass produces both face regions
first so the remote stores drain while it marches on.

On one GPU this runs as
  * an in-process GpuGroup (every rank's passes on one stream in schedule order; the data path, flags, epochs and
    flag resets are the multi-process ones) — eager in the torch process, captured in a hipGraph by the native CLI;
  * two processes sharing the GPU (``--np 2 --no-rccl``): IPC-mapped staging and flags of the other process, the
    waits done by the command processor (``--push-cp-wait``) so the two processes' passes never hold CUs while waiting.
Every variant must be BIT-identical to the single-GPU solve (the reference's 1-GPU log == 2-GPU log property,
report.pdf p.15-16).
"""
import json
import math
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from mpi_cuda_amd import ProblemSpec
from mpi_cuda_amd.solver import Solver

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "bin", "wave3d")


def _same(r, r1):
    assert r.finite and r.steps == r1.steps
    assert r.max_err == r1.max_err
    for a, b in zip(r.rms_err, r1.rms_err):
        assert math.isclose(a, b, rel_tol=1e-12)


@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("K,check_every,temporal", [(20, 2, 4), (9, 1, 4), (12, 3, 3), (11, 2, 2)])
def test_push_group_bitexact(gpu, world, overlap, K, check_every, temporal):
    spec = ProblemSpec(N=66, tau=1e-3, K=K, check_every=check_every)
    ref = Solver(spec, backend="hip", device=0, temporal=1)
    r1 = ref.run()
    f0, f1 = ref.global_field(0), ref.global_field(1)
    g = Solver(spec, backend="hip", transport="push", world=world, rank=0, decomp="slab", overlap=overlap,
               device=0, poison_ghosts=True, tb_min_planes=2 * temporal, temporal=temporal)
    assert g.native.mode() == "deep-tb"
    for _ in range(3):  # repeated solves: flags reset and counters re-zeroed per solve
        r = g.run()
        _same(r, r1)
        assert torch.equal(g.global_field(0), f0)
        assert torch.equal(g.global_field(1), f1)


def test_push_group_needs_slab_passes(gpu):
    spec = ProblemSpec(N=40, tau=1e-3, K=10)
    with pytest.raises(Exception, match="push transport"):
        Solver(spec, backend="hip", transport="push", world=4, rank=0, decomp="2x2x1", device=0)


def _single(N, K, check_every=2):
    s = Solver(ProblemSpec(N=N, tau=1e-3, K=K, check_every=check_every), backend="hip", device=0)
    r = s.run()
    return r, s.global_field(0).numpy()


def _read_dump(prefix, world, N):
    field = np.zeros((N + 1,) * 3)
    for r in range(world):
        m = json.loads(open(f"{prefix}.rank{r}.json").read())
        nx, ny, nz = m["shape"]
        x0, y0, z0 = m["offset"]
        field[x0:x0 + nx, y0:y0 + ny, z0:z0 + nz] = np.fromfile(f"{prefix}.rank{r}.bin").reshape(nx, ny, nz)
    return field


@pytest.mark.parametrize("world,K,extra", [(2, 20, ()), (4, 20, ()), (3, 11, ("--no-overlap",)),
                                           (4, 10, ("--poison-ghosts",)),
                                           (8, 20, ("--temporal", "3", "--tb-min-planes", "6"))])
def test_push_group_cli_graph(gpu, tmp_path, world, K, extra):
    """The native CLI captures the push group's solve into one hipGraph (in-kernel waits, signals and flag resets
    replayed), bit-identical to one GPU."""
    N = 70
    r1, f1 = _single(N, K)
    prefix, js = str(tmp_path / "f"), str(tmp_path / "g.json")
    cmd = [CLI, str(N), "0.001", str(K), "1", "--group", str(world), "--group-transport", "push", "--warmup", "2",
           "--repeat", "3", "--dump", prefix, "--json", js, "--quiet", *extra]
    subprocess.run(cmd, check=True, timeout=120, capture_output=True, text=True)
    meta = json.loads(open(js).read())
    assert meta["transport"] == "push" and meta["schedule"] == "deep-tb" and meta["graph"] is True
    assert np.array_equal(_read_dump(prefix, world, N), f1)
    for (n, m, e), m1, e1 in zip(meta["steps"], r1.max_err, r1.rms_err):
        assert m == pytest.approx(m1, rel=1e-9) and e == pytest.approx(e1, rel=1e-9)  # (JSON: 10 digits)


@pytest.mark.parametrize("overlap", [True, False])
def test_push_two_processes_share_gpu(gpu, tmp_path, overlap):
    """Two processes (fork before any GPU call) on one GPU, no RCCL: each maps the other's staging and flags through
    hipIpcOpenMemHandle (handles exchanged through files), forwards its faces into the other's staging and waits for
    its flags with hipStreamWaitValue32. The dumped fields are bit-identical to one GPU."""
    N, K = 96, 20
    _, f1 = _single(N, K)
    prefix = str(tmp_path / "p")
    env = dict(os.environ, W3D_SHARE_GPUS="1", W3D_TIMEOUT_S="60")
    env.pop("W3D_RDZV_FILE", None)
    cmd = [CLI, str(N), "0.001", str(K), "1", "--np", "2", "--transport", "push", "--no-rccl", "--push-cp-wait",
           "--repeat", "3", "--dump", prefix, "--quiet"] + ([] if overlap else ["--no-overlap"])
    subprocess.run(cmd, check=True, timeout=120, env=env, capture_output=True, text=True)
    assert np.array_equal(_read_dump(prefix, 2, N), f1)


def test_push_two_processes_in_kernel_waits(gpu, tmp_path):
    """As above, but the passes wait for each other IN THE KERNEL (the production wait), truly concurrently: each
    process's compute stream owns half of the CUs (W3D_CU_SPLIT=auto), so a waiting pass never holds the CUs its peer
    needs. A lost signal would end the wait at its bound with an error, not hang."""
    N, K = 96, 20
    _, f1 = _single(N, K)
    prefix = str(tmp_path / "q")
    env = dict(os.environ, W3D_SHARE_GPUS="1", W3D_TIMEOUT_S="30", W3D_CU_SPLIT="auto")
    env.pop("W3D_RDZV_FILE", None)
    cmd = [CLI, str(N), "0.001", str(K), "1", "--np", "2", "--transport", "push", "--no-rccl", "--repeat", "3",
           "--dump", prefix, "--quiet"]
    subprocess.run(cmd, check=True, timeout=150, env=env, capture_output=True, text=True)
    assert np.array_equal(_read_dump(prefix, 2, N), f1)


def test_bench_two_ranks_rehearsal(gpu, tmp_path):
    """bench.py end to end with 2 ranks on one GPU: torch.distributed.run → bench.py ranks (gloo nonce) → native runtime
    children (IPC push transport, in-kernel waits on disjoint CU halves, host collectives through files) → one JSON
    line whose log is the reference's (combined over both ranks) and which says it is a rehearsal, not a scaling point."""
    out = tmp_path / "b.jsonl"
    env = dict(os.environ, W3D_TIMEOUT_S="60")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(29700 + os.getpid() % 200), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--share-gpus", "--no-rccl", "--native-transport", "push", "--steps", "5", "--warmup", "2",
           "--out", str(out)]
    subprocess.run(cmd, check=True, timeout=240, env=env, capture_output=True, text=True)
    line = json.loads(out.read_text().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["distinct_gpus"] == 1 and "rehearsal" in line
    assert line["config"]["transport"] == "push" and line["config"]["schedule"].endswith("-push")
    assert line["correct"] is True and line["final_max_err"] == pytest.approx(3.960129e-09, rel=1e-6)


def test_bench_setup_failure_stops_every_rank(gpu, tmp_path):
    """Fault injection on the GPU path: rank 1's native runtime fails right after setup. Its bench.py
    process raises the abort flag, rank 0's process kills its own child (which would otherwise wait for rank 1's flags
    or files), both agree on the failure over gloo, and the job exits non-zero quickly with no JSON line."""
    import time

    out = tmp_path / "b.jsonl"
    env = dict(os.environ, W3D_TIMEOUT_S="60", W3D_BENCH_FAIL_SETUP_RANK="1", W3D_BENCH_FAIL_FALLBACK="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(29300 + os.getpid() % 200), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--share-gpus", "--no-rccl", "--native-transport", "push", "--steps", "3", "--warmup", "2",
           "--out", str(out)]
    t0 = time.perf_counter()
    p = subprocess.run(cmd, timeout=240, env=env, capture_output=True, text=True)
    assert p.returncode != 0
    assert "injected fault" in p.stderr
    assert not out.exists() or not out.read_text().strip()
    assert time.perf_counter() - t0 < 120


def test_push_fake_rank_runs(gpu, tmp_path):
    """Perf-study mode: one slab rank of 4 timed alone, forwarding into its own staging and waiting for its own
    signals (the cost of the push without peers)."""
    js = str(tmp_path / "f.json")
    subprocess.run([CLI, "128", "0.001", "20", "1", "--fake-rank", "1/4", "--transport", "push", "--repeat", "3",
                    "--json", js, "--quiet"], check=True, timeout=120)
    meta = json.loads(open(js).read())
    assert meta["transport"] == "push" and meta["mode"] == "deep-tb" and meta["finite"]


_PUSH_WORKER = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["ROOT"])
from mpi_cuda_amd import ProblemSpec
from mpi_cuda_amd.solver import Solver
dist.init_process_group("gloo")
spec = ProblemSpec(N=66, tau=1e-3, K=20)
s = Solver(spec, backend="hip", transport="push-ipc", decomp="slab", device=0, graph=False, rccl=False)
rs = [s.run() for _ in range(3)]
torch.save({"err": [r.max_err for r in rs], "f": s.owned_field(0), "rank": dist.get_rank()},
           os.environ["OUT"] + f".{dist.get_rank()}.pt")
dist.destroy_process_group()
"""


def test_push_ipc_python_two_processes(gpu, tmp_path):
    """Python Solver(transport="push-ipc") under torch.distributed.run: one GpuSolver per process with the push
    transport, IPC handles all-gathered over gloo. Two processes on one GPU cannot hold an RCCL communicator, so each
    rank's error log here is its own (push_no_collective); the owned fields must equal the single-GPU field."""
    import sys

    root = ROOT
    script = tmp_path / "w.py"
    script.write_text(_PUSH_WORKER)
    env = dict(os.environ, ROOT=root, OUT=str(tmp_path / "res"), W3D_TIMEOUT_S="30", W3D_CU_SPLIT="auto")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(29500 + os.getpid() % 200), str(script)]
    subprocess.run(cmd, env=env, check=True, timeout=240, capture_output=True, text=True)
    spec = ProblemSpec(N=66, tau=1e-3, K=20)
    ref = Solver(spec, backend="hip", device=0)
    ref.run()
    full = ref.global_field(0)
    from mpi_cuda_amd.parallel.decomp import plan

    for rank in range(2):
        d = torch.load(str(tmp_path / f"res.{rank}.pt"), weights_only=True)
        x0, x1, y0, y1, z0, z1 = plan(66, 2, rank, "slab").box
        assert torch.equal(d["f"], full[x0:x1, y0:y1, z0:z1])
        assert d["err"][0] == d["err"][2]  # repeated solves agree
