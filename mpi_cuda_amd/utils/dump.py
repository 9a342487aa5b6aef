"""Field dump format (the reference defines none, so this is the framework's own, documented here).

A dump of u at step n is ``<prefix>.bin`` + ``<prefix>.json`` for one rank, or ``<prefix>.rank<r>.bin/.json`` per rank
of a decomposed run:

* ``.bin``  raw little-endian float64, C order [x][y][z], the rank's OWNED nodes only (shape = json "shape");
* ``.json`` {"format": "wave3d-dump-v1", "dtype": "float64", "order": "C", "N", "L", "tau", "step", "t", "shape",
  "offset" (global index of the first node), "global_shape" [(N+1)]*3, "rank", "world", "dims"}.

A single-rank dump is the whole (N+1)³ field: ``numpy.fromfile(p + ".bin").reshape(N+1, N+1, N+1)``.
``load()`` assembles either kind; ``save()`` writes the same format from Python (used for checkpoints).
"""
from __future__ import annotations

import glob
import json
import os

import numpy as np

FORMAT = "wave3d-dump-v1"


def save(prefix: str, field: np.ndarray, *, N: int, L: float, tau: float, step: int, offset=(0, 0, 0), rank: int = 0,
         world: int = 1, dims=(1, 1, 1), extra: dict | None = None) -> None:
    field = np.ascontiguousarray(field, dtype="<f8")
    base = prefix if world == 1 else f"{prefix}.rank{rank}"
    field.tofile(base + ".bin")
    meta = {"format": FORMAT, "dtype": "float64", "order": "C", "N": int(N), "L": float(L), "tau": float(tau),
            "step": int(step), "t": float(step * tau), "shape": list(field.shape), "offset": [int(o) for o in offset],
            "global_shape": [N + 1] * 3, "rank": int(rank), "world": int(world), "dims": [int(d) for d in dims]}
    if extra:
        meta.update(extra)
    with open(base + ".json", "w") as f:
        json.dump(meta, f)


def read_meta(prefix: str) -> list[dict]:
    if os.path.exists(prefix + ".json"):
        paths = [prefix + ".json"]
    else:
        paths = sorted(glob.glob(prefix + ".rank*.json"), key=lambda p: int(p.rsplit(".rank", 1)[1][:-5]))
    if not paths:
        raise FileNotFoundError(f"no dump at {prefix}(.rank*).json")
    metas = []
    for p in paths:
        with open(p) as f:
            m = json.load(f)
        if m.get("format") != FORMAT:
            raise ValueError(f"{p}: not a {FORMAT} dump")
        m["_bin"] = p[:-5] + ".bin"
        metas.append(m)
    return metas


def load(prefix: str) -> tuple[np.ndarray, dict]:
    """Assemble the global field from a single- or multi-rank dump. Returns (array (N+1)³, metadata of rank 0)."""
    metas = read_meta(prefix)
    g = metas[0]["global_shape"]
    out = np.zeros(g, dtype=np.float64)
    covered = 0
    for m in metas:
        a = np.fromfile(m["_bin"], dtype="<f8")
        shape = m["shape"]
        if a.size != int(np.prod(shape)):
            raise ValueError(f"{m['_bin']}: size {a.size} does not match shape {shape}")
        a = a.reshape(shape)
        x, y, z = m["offset"]
        out[x:x + shape[0], y:y + shape[1], z:z + shape[2]] = a
        covered += a.size
    if covered != out.size:
        raise ValueError(f"dump covers {covered} of {out.size} nodes (missing ranks?)")
    return out, metas[0]
