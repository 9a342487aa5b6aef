"""The multi-rank schedule autotune of the native runtime (``bin/wave3d --autotune``, what bench.py runs on every rank).

Every candidate is built, run, checked against the first accepted candidate's error log (all schedules compute
bit-identical fields, so a transport that delivers wrong ghosts is rejected), timed, and the fastest is kept. One GPU
exercises the single-rank candidates and, through a fake rank, the multi-rank candidate list (slab RCCL / push, blocks).
"""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "bin", "wave3d")


def _run(tmp_path, *args):
    js = str(tmp_path / "a.json")
    p = subprocess.run([CLI, *args, "--autotune", "--json", js, "--quiet"], check=True, timeout=240,
                       capture_output=True, text=True)
    return json.loads(open(js).read()), p.stderr


def test_autotune_one_rank(gpu, tmp_path):
    meta, err = _run(tmp_path, "128", "0.001", "20", "1", "--repeat", "2")
    tuned = meta["autotune_s"]
    assert {"slab-S4", "slab-S3", "slab-S2", "slab-S1"} <= set(tuned)  # (push / block need neighbours)
    assert meta["schedule"] == min(tuned, key=tuned.get)
    assert "rejected" not in err  # every one-rank schedule reproduces the reference log bit for bit
    assert meta["steps"][-1][0] == 20 and meta["finite"]


def test_autotune_fake_rank_candidates(gpu, tmp_path):
    meta, _ = _run(tmp_path, "128", "0.001", "20", "1", "--fake-rank", "1/4", "--repeat", "2")
    tuned = meta["autotune_s"]
    assert {"slab-S4", "slab-S4-seq", "slab-S4-push", "slab-S4-push-seq", "block-S4"} <= set(tuned)
    assert meta["schedule"] == min(tuned, key=tuned.get)
