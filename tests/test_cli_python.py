"""Python CLI (python -m mpi_cuda_amd), dump reader and checkpoint/resume."""
import os
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pycli(*args, env=None):
    return subprocess.run([sys.executable, "-m", "mpi_cuda_amd", *map(str, args)], cwd=ROOT, capture_output=True,
                          text=True, timeout=300, env=env)


def test_python_cli_cpu_matches_reference_digits():
    r = pycli(128, 0.001, 20, "--backend", "cpu")
    assert r.returncode == 0, r.stderr
    assert "Step 20, t = 0.020000, Max Error = 2.820954e-07, L2 Error = 1.009161e-07" in r.stdout


def test_python_cli_cfl_guard():
    r = pycli(1024, 0.001, 20, "--backend", "cpu")
    assert r.returncode == 2 and "CFL" in r.stderr


def test_dump_roundtrip_and_checkpoint_resume(tmp_path):
    from mpi_cuda_amd import ProblemSpec
    from mpi_cuda_amd.models.wave3d import torch_reference_solve
    from mpi_cuda_amd.utils import dump as dumpio

    ck = str(tmp_path / "ck")
    r = pycli(30, 0.001, 6, "--backend", "cpu", "--checkpoint", ck, "--dump", str(tmp_path / "u6"))
    assert r.returncode == 0, r.stderr
    u6, meta = dumpio.load(str(tmp_path / "u6"))
    assert meta["step"] == 6 and u6.shape == (31, 31, 31)
    _, ref6, _ = torch_reference_solve(ProblemSpec(N=30, tau=1e-3, K=6), return_fields=True)
    assert np.array_equal(u6, ref6.numpy())
    # continue 6 -> 10 from the checkpoint; must equal a straight 10-step run bit for bit
    r2 = pycli(30, 0.001, 10, "--backend", "cpu", "--resume", ck, "--dump", str(tmp_path / "u10"))
    assert r2.returncode == 0, r2.stderr
    u10, m10 = dumpio.load(str(tmp_path / "u10"))
    errs, ref10, _ = torch_reference_solve(ProblemSpec(N=30, tau=1e-3, K=10), return_fields=True)
    assert np.array_equal(u10, ref10.numpy())
    assert "Step 10, t = 0.010000" in r2.stdout and "Step 6," not in r2.stdout


def test_multirank_dump_assembles(tmp_path):
    from mpi_cuda_amd.utils import dump as dumpio

    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "3", "--master-addr", "127.0.0.1",
           "--master-port", str(29350 + os.getpid() % 40), "-m", "mpi_cuda_amd", "26", "0.001", "5", "--backend",
           "cpu", "--decomp", "1x3x1", "--dump", str(tmp_path / "d")]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    u, meta = dumpio.load(str(tmp_path / "d"))
    assert meta["world"] == 3
    from mpi_cuda_amd import ProblemSpec
    from mpi_cuda_amd.models.wave3d import torch_reference_solve

    _, ref, _ = torch_reference_solve(ProblemSpec(N=26, tau=1e-3, K=5), return_fields=True)
    assert np.array_equal(u, ref.numpy())


def test_process_runtime_rejects_options_it_cannot_honour():
    """Solver(runtime='process') forwards the options its rank process honours as CLI flags and raises for
    the others instead of dropping them silently (checked before any process or GPU is touched)."""
    import pytest

    from mpi_cuda_amd import ProblemSpec
    from mpi_cuda_amd.solver import Solver

    spec = ProblemSpec(N=16, tau=1e-3, K=4)
    for kw in (dict(tiling={"rows": 4}), dict(tiling2={"rows": 2}), dict(tiling_tb={"xcd_blocks": True}),
               dict(copy_engines=True)):
        with pytest.raises(ValueError):
            Solver(spec, backend="hip", transport="rccl", runtime="process", **kw)
