"""The multi-rank schedule autotune of the native runtime (csrc/src/runtime_autotune.cpp): ``bin/wave3d --autotune``
(what bench.py runs on every rank) and the Python ``Solver(autotune=True)`` run the same code.

Every candidate is built, clones of an earlier candidate (same mode, transport, overlap, depth, decomposition) are
dropped, each survivor is run, checked against the first accepted candidate's error log (all schedules compute
bit-identical fields, so a transport that delivers wrong ghosts is rejected), timed in interleaved rounds, and the
simplest candidate within 2 % of the fastest is kept. One GPU exercises the single-rank candidates and, through a fake
rank, the multi-rank candidate list (slab / block × RCCL / copy engines × overlap).
"""
import json
import os
import subprocess

import pytest

from mpi_cuda_amd import ProblemSpec
from mpi_cuda_amd.solver import Solver

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "bin", "wave3d")


def _run(tmp_path, *args):
    js = str(tmp_path / "a.json")
    p = subprocess.run([CLI, *args, "--autotune", "--json", js, "--quiet"], check=True, timeout=240,
                       capture_output=True, text=True)
    return json.loads(open(js).read()), p.stderr


def _chosen_ok(meta):
    tuned = meta["autotune_s"]
    best = min(tuned.values())
    assert tuned[meta["schedule"]] <= best * 1.02 + 1e-12
    # the simplest (first listed) candidate within the tie margin
    first = next(k for k, v in tuned.items() if v <= best * 1.02 + 1e-12)
    assert meta["schedule"] == first


def test_autotune_one_rank(gpu, tmp_path):
    meta, err = _run(tmp_path, "128", "0.001", "20", "1", "--repeat", "2")
    tuned = meta["autotune_s"]
    assert set(tuned) == {"slab-S5", "slab-S4", "slab-S3", "slab-S2", "slab-S1"}  # (no neighbours: nothing else differs)
    _chosen_ok(meta)
    assert "rejected" not in err  # every one-rank schedule reproduces the reference log bit for bit
    assert meta["steps"][-1][0] == 20 and meta["finite"] and meta["autotune_rounds"] == 5


def test_autotune_fake_rank_candidates(gpu, tmp_path):
    meta, _ = _run(tmp_path, "128", "0.001", "20", "1", "--fake-rank", "1/4", "--repeat", "2")
    tuned = meta["autotune_s"]
    assert {"slab-S4-seq", "slab-S4", "slab-S4-sdma", "block-S4-seq", "block-S4", "block-S4-sdma"} <= set(tuned)
    # (round 6: the 5-step pair-tiled pass beside the copy engines, and on overlapped 3-D blocks)
    assert {"slab-S5-sdma", "slab-S5-sdma-seq", "block-S5", "block-S5-sdma", "block-S5-sdma-seq"} <= set(tuned)
    assert not any("push" in k for k in tuned)  # push only on request
    _chosen_ok(meta)


def test_autotune_push_on_request(gpu, tmp_path):
    meta, _ = _run(tmp_path, "128", "0.001", "20", "1", "--fake-rank", "1/4", "--transport", "push")
    assert {"slab-S4-push", "slab-S4-push-seq"} <= set(meta["autotune_s"])


def test_autotune_drops_clones(gpu, tmp_path):
    """Two candidates that run the same schedule are one candidate: 2 ranks have no block decomposition, and a rank of
    a slab job whose passes are too thin for the LDS schedule runs single steps whatever the pass depth asks."""
    meta, _ = _run(tmp_path, "64", "0.001", "20", "1", "--fake-rank", "0/8", "--repeat", "1")
    rej = meta["autotune_rejected"]
    assert any("same schedule" in v for v in rej.values())
    assert len(set(meta["autotune_s"])) == len(meta["autotune_s"])


def test_autotune_repeatable(gpu, tmp_path):
    """Two autotune runs on the same box pick the same schedule (interleaved rounds, 2 % tie margin)."""
    a, _ = _run(tmp_path, "128", "0.001", "20", "1")
    b, _ = _run(tmp_path, "128", "0.001", "20", "1")
    assert a["schedule"] == b["schedule"]


def test_autotune_python_entry_point(gpu, tmp_path):
    """Solver(autotune=True) runs the CLI's autotune: same candidates, same choice on one rank."""
    spec = ProblemSpec(N=128, tau=1e-3, K=20)
    s = Solver(spec, backend="hip", device=0, autotune=True)
    assert set(s.autotune_times) == {"slab-S5", "slab-S4", "slab-S3", "slab-S2", "slab-S1"}
    cli, _ = _run(tmp_path, "128", "0.001", "20", "1")
    assert s.schedule == cli["schedule"]
    r = s.run()
    ref = Solver(spec, backend="hip", device=0).run()
    assert r.max_err == ref.max_err


def test_block_overlap_label_is_honest(gpu, tmp_path):
    """The JSON reports the overlap that ran: block ranks with --no-overlap exchange after the pass (false); with
    overlap their border tiles and x-face slabs run first on the side stream (true)."""
    js = str(tmp_path / "o.json")
    for extra, want in ((["--no-overlap"], False), ([], True)):
        subprocess.run([CLI, "128", "0.001", "20", "1", "--fake-rank", "3/8", "--decomp", "2x2x2", "--json", js,
                        "--quiet", *extra], check=True, timeout=120)
        meta = json.loads(open(js).read())
        assert meta["mode"] == "deep-tb-block" and meta["overlap"] is want


def test_autotune_times_medians_of_back_to_back_solves(gpu, tmp_path):
    """each candidate is timed in rounds of back-to-back solves (the bench's pattern) and
    chosen on the MEDIAN round, not the best one; the JSON carries both, the rounds x reps and the autotune's wall
    time."""
    meta, _ = _run(tmp_path, "128", "0.001", "20", "1", "--fake-rank", "1/4", "--autotune-rounds", "3",
                   "--autotune-reps", "4")
    med, best = meta["autotune_s"], meta["autotune_best_s"]
    assert set(med) == set(best) and meta["autotune_rounds"] == 3 and meta["autotune_reps"] == 4
    assert all(best[k] <= med[k] for k in med)
    assert 0 < meta["autotune_wall_s"] < 120
    _chosen_ok(meta)


def test_autotune_wall_budget(gpu, tmp_path):
    """once the wall-time budget is spent no further candidate is built (rejected with the
    reason) and at least one round still times what was accepted."""
    meta, _ = _run(tmp_path, "128", "0.001", "20", "1", "--fake-rank", "1/4", "--autotune-budget", "0.001")
    rej = meta["autotune_rejected"]
    assert any("budget" in v for v in rej.values())
    assert len(meta["autotune_s"]) >= 1 and meta["autotune_rounds"] >= 1
    assert meta["schedule"] in meta["autotune_s"]


def test_field_hash_is_decomposition_free(gpu):
    """The autotune's field check: the hash of u^K and u^{K-1} summed over the ranks equals the one-rank hash for slab
    and block groups (bit-identical fields), and a different field (one step fewer) hashes differently."""
    spec = ProblemSpec(N=66, tau=1e-3, K=20)
    ref = Solver(spec, backend="hip", device=0)
    ref.run()
    h0, h1 = ref.field_hash(0), ref.field_hash(1)
    assert h0 != h1
    for decomp, world in (("slab", 3), ("2x2x2", 8)):
        g = Solver(spec, backend="hip", transport="loopback", world=world, rank=0, decomp=decomp, device=0)
        g.run()
        assert g.field_hash(0) == h0 and g.field_hash(1) == h1
    other = Solver(ProblemSpec(N=66, tau=1e-3, K=19), backend="hip", device=0)
    other.run()
    assert other.field_hash(0) != h0 and other.field_hash(0) == h1
