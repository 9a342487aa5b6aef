#!/usr/bin/env python3
"""Native build driver: compiles the HIP/C++ runtime for gfx950 IN-TREE.

Outputs
  mpi_cuda_amd/_C<ext-suffix>   Python extension (pybind11): HIP kernels + RCCL GpuSolver + CPU/OpenMP path
  bin/wave3d                    standalone CLI, reference-compatible ``wave3d N tau K [L]`` (see csrc/app/wave3d_main.cpp)

Every translation unit is compiled with -ffp-contract=off so host and device evaluate the stencil with identical
rounding (bit-exact CPU == GPU == any decomposition). HIP sources go through hipcc --offload-arch=gfx950, host-only
C++ through g++ (-fopenmp -> libgomp, the same OpenMP runtime PyTorch loads). Objects are cached by content hash
under build/ so re-running is cheap.

Usage: python tools/build.py [--jobs N] [--force] [--no-cli] [--verbose]
"""
from __future__ import annotations

import argparse
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "csrc"
BUILD = ROOT / "build"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("WAVE3D_ARCH", "gfx950")

HIPCC = str(ROCM / "bin" / "hipcc")
CXX = os.environ.get("CXX", "g++")

COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
          f"-I{CSRC / 'include'}"]
HIP_FLAGS = COMMON + [f"--offload-arch={ARCH}", "-fno-gpu-rdc", "-munsafe-fp-atomics"]
# (perf-attribution experiments only: e.g. W3D_EXTRA_DEFS=-DW3D_EXPERIMENT_NOLOAD builds a variant whose results are wrong)
HIP_FLAGS += os.environ.get("W3D_EXTRA_DEFS", "").split()
# (... and W3D_EXTRA_DEFS_P2 for the pair-tiled pass's translation units only: a variant rebuilds 5 objects, not all)
P2_EXTRA = os.environ.get("W3D_EXTRA_DEFS_P2", "").split()
# x86-64-v3: std::fma (stencil.hpp) is one vfmadd instruction, not a libm call
CPU_FLAGS = COMMON + ["-fopenmp", "-march=x86-64-v3"]

# (source, compiler kind). 'hip' = device code or HIP runtime host code, 'cpu' = plain C++ with OpenMP.
LIB_SOURCES = [
    ("src/kernels_stencil.hip", "hip"),
    ("src/kernels_halo.hip", "hip"),
    ("src/kernels_leapfrog2.hip", "hip"),
    ("src/kernels_init2.hip", "hip"),
    ("src/kernels_leapfrog_tb.hip", "hip"),
    ("src/kernels_leapfrog_tb_push.hip", "hip"),
    ("src/kernels_leapfrog_p2.hip", "hip"),
    ("src/kernels_leapfrog_p2_s2.hip", "hip"),
    ("src/kernels_leapfrog_p2_s3.hip", "hip"),
    ("src/kernels_leapfrog_p2_s4.hip", "hip"),
    ("src/kernels_leapfrog_p2_s5.hip", "hip"),
    ("src/solver_gpu.cpp", "hip"),
    ("src/capture_guard.cpp", "hip"),
    ("src/transport_sdma.cpp", "hip"),
    ("src/runtime_launch.cpp", "hip"),
    ("src/runtime_io.cpp", "hip"),
    ("src/runtime_autotune.cpp", "hip"),
    ("src/cpu_kernels.cpp", "cpu"),
    ("src/cpu_solver.cpp", "cpu"),
    ("src/cpu_dist.cpp", "cpu"),
]
EXT_SOURCES = [("src/bindings.cpp", "hip")]
CLI_SOURCES = [("app/wave3d_main.cpp", "hip"), ("app/cli_args.cpp", "hip"), ("app/cli_cpu.cpp", "hip")]
PERSONALITIES = ["wave", "openmpwave", "wave3dOMP", "onlyMPI", "mpi", "mpiomp", "mpigpu-1"]


def _pybind_includes() -> list[str]:
    import pybind11

    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _hash_inputs(src: Path, flags: list[str]) -> str:
    h = hashlib.sha256()
    h.update(" ".join(flags).encode())
    h.update(src.read_bytes())
    for hdr in sorted([*(CSRC / "include").rglob("*.hpp"), *(CSRC / "app").glob("*.hpp")]):
        h.update(hdr.read_bytes())
    return h.hexdigest()[:16]


def _compile(src_rel: str, kind: str, extra: list[str], force: bool, verbose: bool) -> Path:
    src = CSRC / src_rel
    flags = (HIP_FLAGS if kind == "hip" else CPU_FLAGS) + extra
    if src_rel.startswith("src/kernels_leapfrog_p2"):
        flags = flags + P2_EXTRA
    if kind == "hip" and src.suffix == ".cpp":
        flags = flags + ["-x", "hip"]
    tag = _hash_inputs(src, flags)
    obj = BUILD / "obj" / f"{src.stem}.{tag}.o"
    if obj.exists() and not force:
        return obj
    obj.parent.mkdir(parents=True, exist_ok=True)
    cc = HIPCC if kind == "hip" else CXX
    cmd = [cc, *flags, "-c", str(src), "-o", str(obj) + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"compile failed: {src_rel}")
    os.replace(str(obj) + ".tmp", obj)
    return obj


def _link(objs: list[Path], out: Path, shared: bool, verbose: bool) -> None:
    out.parent.mkdir(parents=True, exist_ok=True)
    rocm_lib = ROCM / "lib"
    cmd = [HIPCC, f"--offload-arch={ARCH}", *map(str, objs), "-o", str(out) + ".tmp",
           f"-L{rocm_lib}", "-lrccl", "-lrocprofiler-sdk-roctx", "-lamdhip64", "-lgomp", "-lpthread", f"-Wl,-rpath,{rocm_lib}"]
    if shared:
        cmd.insert(1, "-shared")
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"link failed: {out}")
    os.replace(str(out) + ".tmp", out)


def ext_path() -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return ROOT / "mpi_cuda_amd" / f"_C{suffix}"


def cli_path() -> Path:
    return ROOT / "bin" / "wave3d"


def build(jobs: int = 8, force: bool = False, cli: bool = True, verbose: bool = False, cli_out: str = "") -> dict:
    if not Path(HIPCC).exists():
        raise RuntimeError(f"hipcc not found at {HIPCC}")
    py_inc = _pybind_includes()
    units = [(s, k, []) for s, k in LIB_SOURCES] + ([] if cli_out else [(s, k, py_inc) for s, k in EXT_SOURCES])
    if cli or cli_out:
        units += [(s, k, []) for s, k in CLI_SOURCES]
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = {s: ex.submit(_compile, s, k, e, force, verbose) for s, k, e in units}
        objs = {s: f.result() for s, f in futs.items()}
    lib_objs = [objs[s] for s, _ in LIB_SOURCES]
    if cli_out:  # (an experiment build: the CLI alone, at its own path; bin/ and the extension stay as they are)
        Path(cli_out).parent.mkdir(parents=True, exist_ok=True)
        _link(lib_objs + [objs[s] for s, _ in CLI_SOURCES], Path(cli_out), shared=False, verbose=verbose)
        return {"cli": cli_out}
    ext = ext_path()
    _link(lib_objs + [objs[s] for s, _ in EXT_SOURCES], ext, shared=True, verbose=verbose)
    out = {"extension": str(ext)}
    if cli:
        _link(lib_objs + [objs[s] for s, _ in CLI_SOURCES], cli_path(), shared=False, verbose=verbose)
        out["cli"] = str(cli_path())
        # the reference's program names (the CLI picks its personality from argv[0]; csrc/app/wave3d_main.cpp)
        for name in PERSONALITIES:
            link = cli_path().parent / name
            if link.is_symlink() or link.exists():
                link.unlink()
            link.symlink_to(cli_path().name)
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--no-cli", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--cli-out", default="", help="experiment builds: link only the CLI, to this path")
    a = ap.parse_args()
    if a.clean and BUILD.exists():
        shutil.rmtree(BUILD)
    res = build(jobs=a.jobs, force=a.force, cli=not a.no_cli, verbose=a.verbose, cli_out=a.cli_out)
    for k, v in res.items():
        print(f"built {k}: {v}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
