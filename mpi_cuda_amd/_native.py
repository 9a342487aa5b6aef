"""Loader for the in-tree native extension ``mpi_cuda_amd._C`` (HIP kernels, RCCL runtime, CPU/OpenMP path).

The extension is built by ``tools/build.py`` (or ``__graft_entry__.build()``) and lives next to this file, so it travels
with the repository snapshot. There is deliberately no silent fallback: on a machine with a GPU every GPU op goes
through the HIP kernels, and a missing or stale extension is an error, not a slower path.
"""
from __future__ import annotations

import importlib
import os
import sys
from pathlib import Path

import torch  # noqa: F401  (load torch's HIP runtime first: the extension binds to the same libamdhip64.so.7)

_ROOT = Path(__file__).resolve().parents[1]
_C = None


def _build_if_requested() -> None:
    if os.environ.get("WAVE3D_AUTOBUILD", "1") != "1":
        return
    sys.path.insert(0, str(_ROOT / "tools"))
    try:
        import build as _b  # type: ignore

        _b.build(cli=False)
    finally:
        sys.path.pop(0)


def load():
    """Return the native module, building it in-tree on first use if it is missing."""
    global _C
    if _C is not None:
        return _C
    try:
        _C = importlib.import_module("mpi_cuda_amd._C")
    except ImportError:
        _build_if_requested()
        _C = importlib.import_module("mpi_cuda_amd._C")
    return _C


def native_path() -> str:
    return load().__file__


def gpu_available() -> bool:
    return torch.cuda.is_available()


def require_gpu():
    """The native module, after checking that a GPU is present (GPU ops never fall back to PyTorch)."""
    C = load()
    if not torch.cuda.is_available():
        raise RuntimeError("wave3d: a GPU op was requested but no GPU is visible")
    return C
