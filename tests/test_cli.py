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
    if not os.path.exists(CLI) or not os.path.lexists(os.path.join(ROOT, "bin", "mpiomp")):
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


@pytest.mark.parametrize("np_,decomp", [(2, "slab"), (3, "slab"), (4, "block"), (6, "1x2x3"), (8, "2x2x2")])
def test_cpu_multiprocess_bitexact(tmp_path, np_, decomp):
    """`--cpu --np P`: the reference's MPI / MPI+OpenMP programs (one process per rank, OpenMP inside, halos through a
    shared-memory segment). Same log as the sequential program and, assembled from the per-rank dumps, the same field
    bit for bit (the reference's rank-count invariance, report.pdf p.7-11)."""
    seq = run(30, 0.001, 8, "--cpu", "--threads", 1, "--dump", tmp_path / "seq")
    par = run(30, 0.001, 8, "--cpu", "--np", np_, "--decomp", decomp, "--threads", 1, "--dump", tmp_path / "par")
    lines = lambda o: [l for l in o.stdout.splitlines() if l.startswith("Step ")]  # noqa: E731
    assert lines(par) == lines(seq) and len(lines(seq)) == 4
    assert f"max over {np_} ranks" in par.stdout
    meta = json.loads((tmp_path / "seq.json").read_text())
    full = np.fromfile(tmp_path / "seq.bin", dtype=np.float64).reshape(meta["shape"])
    got = np.full_like(full, np.nan)
    for r in range(np_):
        m = json.loads((tmp_path / f"par.rank{r}.json").read_text())
        (x0, y0, z0), (nx, ny, nz) = m["offset"], m["shape"]
        got[x0:x0 + nx, y0:y0 + ny, z0:z0 + nz] = np.fromfile(tmp_path / f"par.rank{r}.bin",
                                                              dtype=np.float64).reshape(nx, ny, nz)
    assert np.array_equal(got, full)


@pytest.mark.parametrize("np_", [1, 2, 4])
def test_cpu_phase_columns(tmp_path, np_):
    """The reference's CPU phase columns (report.pdf p.16): init / compute / boundary / exchange, each
    the max over ranks, printed and in --json, plus the slowest rank's own four, which account for its solve (sum
    within 5 % of the total; maxima of different ranks overlap in time, so their sum may exceed it)."""
    j = tmp_path / "p.json"
    args = [64, 0.001, 10, "--cpu", "--threads", 1, "--repeat", 3, "--json", j]
    if np_ > 1:
        args += ["--np", np_, "--decomp", "slab"]
    out = run(*args).stdout
    assert any(l.startswith("Phases (s") and "boundary" in l and "exchange" in l for l in out.splitlines())
    rec = json.loads(j.read_text())
    ph, sl = rec["phases_s"], rec["phases_slowest_rank_s"]
    assert set(ph) == set(sl) == {"init", "compute", "boundary", "exchange"}
    assert all(ph[k] >= sl[k] for k in ph)
    total = sum(sl.values())
    assert abs(total - rec["solve_s"]) <= 0.05 * rec["solve_s"], (sl, rec["solve_s"])
    if np_ == 1:
        assert ph["boundary"] == 0.0 and ph["exchange"] == 0.0
    else:
        assert ph["boundary"] > 0.0 and ph["exchange"] > 0.0


def test_cpu_multiprocess_rank_failure_is_an_error():
    """Fault injection: one rank fails before its first exchange; the others leave their barriers with an error at
    once (shared failure flag) instead of waiting for the barrier timeout, and the run exits non-zero."""
    import time

    t0 = time.time()
    r = subprocess.run([CLI, "40", "0.001", "6", "--cpu", "--np", "4", "--threads", "1"], capture_output=True,
                       text=True, timeout=120, env=dict(os.environ, W3D_FAULT_RANK="2"))
    assert r.returncode != 0
    assert "injected fault" in r.stderr and "another rank failed" in r.stderr
    assert time.time() - t0 < 30


def _children(pid):
    try:
        with open(f"/proc/{pid}/task/{pid}/children") as f:
            return [int(c) for c in f.read().split()]
    except OSError:
        return []


def _alive(pid):
    """A process that exists and is not a zombie (an orphan's zombie waits for a reaper; it runs nothing)."""
    try:
        with open(f"/proc/{pid}/status") as f:
            state = next(l for l in f if l.startswith("State:"))
        return "Z" not in state.split()[1]
    except (OSError, StopIteration):
        return False


def test_spawned_ranks_die_with_the_spawner():
    """`--np P` ranks are forked children of the spawner; when the spawner is killed (a test or
    bench timeout sends SIGKILL to the process it started, not to its children) the ranks must not keep running — each
    child holds PR_SET_PDEATHSIG = SIGKILL."""
    import signal
    import time

    p = subprocess.Popen([CLI, "96", "0.001", "20", "--cpu", "--np", "2", "--threads", "1", "--repeat", "100000",
                          "--quiet"], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        t0 = time.time()
        kids = []
        while len(kids) < 2 and time.time() - t0 < 30:
            kids = _children(p.pid)
            time.sleep(0.05)
        assert len(kids) == 2, kids
        time.sleep(0.5)  # (mid-solve)
        assert all(_alive(k) for k in kids)
        os.kill(p.pid, signal.SIGKILL)
        p.wait(timeout=10)
        t1 = time.time()
        while any(_alive(k) for k in kids) and time.time() - t1 < 10:
            time.sleep(0.05)
        assert not any(_alive(k) for k in kids), [k for k in kids if _alive(k)]
    finally:
        if p.poll() is None:
            p.kill()


def test_reference_program_personalities():
    """The build links the reference's program names to the CLI (tools/build.py); argv[0] picks the behaviour:
    `wave N tau K` sequential, `wave3dOMP N tau K T` / `mpiomp N tau K T` take OpenMP threads as the 4th argument,
    `mpigpu-1 N tau K L` takes L (report.pdf p.12-15, p.20-24)."""
    seq = run(40, 0.001, 6, "--cpu", "--threads", 1)
    b = os.path.join(ROOT, "bin")
    for prog, extra, threads in (("wave", [], 1), ("wave3dOMP", [3], 3), ("openmpwave", [2], 2), ("mpiomp", [2], 2)):
        out = subprocess.run([os.path.join(b, prog), "40", "0.001", "6", *map(str, extra)], capture_output=True,
                             text=True, check=True, timeout=120).stdout
        assert [l for l in out.splitlines() if l.startswith("Step ")] == \
            [l for l in seq.stdout.splitlines() if l.startswith("Step ")]
        assert f"threads {threads}" in out, (prog, out)


def test_mpi_program_under_external_launcher():
    """`mpirun -np P ./onlyMPI N tau K` semantics: P independently started processes with the launcher's rank env find
    each other through a named shared-memory segment (keyed by the job id) and print the sequential program's log."""
    import uuid

    seq = run(36, 0.001, 6, "--cpu", "--threads", 1)
    job = uuid.uuid4().hex[:12]
    prog = os.path.join(ROOT, "bin", "onlyMPI")
    procs = []
    for r in range(3):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="3", LOCAL_RANK=str(r), W3D_JOB_ID=job)
        procs.append(subprocess.Popen([prog, "36", "0.001", "6"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True, env=env))
    outs = [p.communicate(timeout=120) for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    lines = [l for l in outs[0][0].splitlines() if l.startswith("Step ")]
    assert lines == [l for l in seq.stdout.splitlines() if l.startswith("Step ")] and len(lines) == 3
    assert "max over 3 ranks" in outs[0][0]
    assert not os.path.exists(f"/dev/shm/wave3d-cpu-{job}")  # rank 0 unlinked the segment


def test_cli_cpu_checkpoint_resume_bitexact(tmp_path):
    """bin/wave3d --cpu: K=10 → --checkpoint → --resume to K=20 equals a direct K=20 run bit for bit (field dump) and
    prints the same error lines for steps 12..20."""
    import numpy as np

    cli = os.path.join(ROOT, "bin", "wave3d")
    run = lambda *a: subprocess.run([cli, *map(str, a)], check=True, capture_output=True, text=True,  # noqa: E731
                                    cwd=tmp_path).stdout
    run(40, 0.001, 10, 1, "--cpu", "--checkpoint", "c10")
    resumed = run(40, 0.001, 20, 1, "--cpu", "--resume", "c10", "--dump", "r20")
    direct = run(40, 0.001, 20, 1, "--cpu", "--dump", "d20")
    assert np.array_equal(np.fromfile(tmp_path / "r20.bin"), np.fromfile(tmp_path / "d20.bin"))
    steps = lambda out: [l for l in out.splitlines() if l.startswith("Step")]  # noqa: E731
    assert steps(resumed) == [l for l in steps(direct) if int(l.split()[1].rstrip(",")) > 10]
    meta = json.loads((tmp_path / "c10.prev.json").read_text())
    assert meta["step"] == 9 and json.loads((tmp_path / "c10.cur.json").read_text())["step"] == 10


def test_native_rank_process_protocol_cpu(tmp_path):
    """The rank-process protocol behind Solver(runtime="process") (bin/wave3d --serve, parallel/native_proc.py), on
    the CPU solver: greeting, repeated solves with the exact log, dump, error replies, clean quit, and a child that
    dies mid-session turning into a Python error instead of a hang."""
    from mpi_cuda_amd import ProblemSpec
    from mpi_cuda_amd.parallel.native_proc import NativeRankProcess
    from mpi_cuda_amd.solver import Solver
    from mpi_cuda_amd.utils.dump import load

    spec = ProblemSpec(N=32, tau=1e-3, K=10, check_every=1)
    ref = Solver(spec, backend="cpu")
    r = ref.run()
    p = NativeRankProcess(spec, 0, 1, 0, extra_args=("--cpu", "--threads", "2"), timeout_s=60)
    try:
        assert p.info["ready"] and p.info["backend"] == "cpu" and p.info["dims"] == [1, 1, 1]
        for _ in range(2):
            a = p.run()
            assert a["steps"] == r.steps and a["max_err"] == r.max_err and a["rms_err"] == r.rms_err
            assert a["finite"] is True and a["graph"] is False and a["solve_s"] > 0
        prefix = str(tmp_path / "d")
        p.dump(prefix)
        field, meta = load(prefix)
        assert np.array_equal(field, ref.owned_field(0).numpy())
        with pytest.raises(RuntimeError, match="unknown command"):
            p.command("bogus")
        assert p.run()["max_err"] == r.max_err  # (still serving after an error reply)
    finally:
        p.close()
    assert p._p.returncode == 0
    q = NativeRankProcess(spec, 0, 1, 0, extra_args=("--cpu",), timeout_s=60)
    q._p.kill()
    q._p.wait()
    with pytest.raises(RuntimeError, match="exited"):
        q.run()
    q.close()


def test_native_rank_process_banner_in_one_chunk(tmp_path, monkeypatch):
    """A library banner written to the child's stdout in the same pipe chunk as the greeting (RCCL prints one while an
    rccl-self group initialises, before the serve loop takes stdout over): the client skips the banner lines and
    still finds the greeting and every reply, and a silent child times out instead of hanging."""
    from mpi_cuda_amd import ProblemSpec
    from mpi_cuda_amd.parallel import native_proc

    fake = tmp_path / "wave3d"
    fake.write_text("#!/bin/sh\n"
                    "printf 'RCCL version : x\\nHIP version : y\\n{\"ready\": true, \"dims\": [2, 1, 1]}\\n'\n"
                    "while read l; do case \"$l\" in\n"
                    "  run) printf 'noise\\n{\"steps\": [[2, 0.5, 0.25]], \"solve_s\": 0.1}\\n';;\n"
                    "  hang) sleep 30;;\n"
                    "  quit) echo '{\"bye\": true}'; exit 0;;\n"
                    "esac; done\n")
    fake.chmod(0o755)
    monkeypatch.setattr(native_proc, "CLI", str(fake))
    spec = ProblemSpec(N=16, tau=1e-3, K=2)
    p = native_proc.NativeRankProcess(spec, 0, 1, 0, timeout_s=5)
    try:
        assert p.info == {"ready": True, "dims": [2, 1, 1]}
        r = p.run()
        assert r["steps"] == [2] and r["max_err"] == [0.5] and r["rms_err"] == [0.25]
    finally:
        p.close()
    assert p._p.returncode == 0
    q = native_proc.NativeRankProcess(spec, 0, 1, 0, timeout_s=1)
    with pytest.raises(TimeoutError, match="no reply"):
        q.command("hang")
    q.close()
