"""The standalone CLI keeps the reference's interface: positional `N tau K [L]`, the per-step error lines of
report.pdf p.15-16, a CFL guard, JSON output and the field dump format."""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "bin", "wave3d")


@pytest.fixture(scope="module", autouse=True)
def cli_built():
    if not os.path.exists(CLI):
        from mpi_cuda_amd._native import load

        load()
        subprocess.run(["python", os.path.join(ROOT, "tools", "build.py")], check=True)
    assert os.path.exists(CLI)


def run(*args, check=True):
    return subprocess.run([CLI, *map(str, args)], capture_output=True, text=True, check=check, timeout=120)


def test_cpu_sequential_config_output_format():
    out = run(128, 0.001, 20, "--cpu", "--threads", 1).stdout.splitlines()
    steps = [l for l in out if l.startswith("Step ")]
    assert len(steps) == 10
    assert steps[0].startswith("Step 2, t = 0.002000, Max Error = ")
    assert steps[-1] == "Step 20, t = 0.020000, Max Error = 2.820954e-07, L2 Error = 1.009161e-07"
    assert any(l.startswith("Total time:") for l in out)


def test_fourth_positional_is_L():
    import math

    out = run(128, 0.001, 20, math.pi, "--cpu").stdout
    assert "Max Error = 2.996306e-08, L2 Error = 1.071891e-08" in out


def test_cfl_guard():
    r = run(1024, 0.001, 20, "--cpu", check=False)
    assert r.returncode == 2 and "CFL" in r.stderr


def test_bad_args():
    assert run(12, check=False).returncode == 2
    assert run(12, 0.001, 2, "--bogus", check=False).returncode == 2


def test_json_and_dump(tmp_path):
    j = tmp_path / "o.json"
    d = tmp_path / "field"
    run(24, 0.001, 4, "--cpu", "--json", j, "--dump", d, "--check-every", 1)
    rec = json.loads(j.read_text())
    assert rec["N"] == 24 and rec["K"] == 4 and rec["backend"] == "cpu"
    meta = json.loads((tmp_path / "field.json").read_text())
    assert meta["shape"] == [25, 25, 25] and meta["dtype"] == "float64"
    u = np.fromfile(tmp_path / "field.bin", dtype=np.float64).reshape(meta["shape"])
    from mpi_cuda_amd import ProblemSpec
    from mpi_cuda_amd.models.wave3d import torch_reference_solve

    _, uk, _ = torch_reference_solve(ProblemSpec(N=24, tau=1e-3, K=4), return_fields=True)
    assert np.array_equal(u, uk.numpy())
