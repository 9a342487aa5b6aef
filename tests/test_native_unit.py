"""Native C++ unit tests (csrc/tests/test_core.cpp) built with host AddressSanitizer + UBSan and run on the CPU.

SURVEY.md §4.2 (unit, C++) and §5.2(c) (host sanitizers on the CPU path and tools): decomposition and halo-plan
invariants, 64-bit layout arithmetic, exactness of Δ_h on quadratics, CFL guard, pack/unpack, and the 128³ golden
errors of the OpenMP solver, all under ASan/UBSan (any memory error or UB aborts the binary)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = ["csrc/tests/test_core.cpp", "csrc/src/cpu_kernels.cpp", "csrc/src/cpu_solver.cpp"]


@pytest.fixture(scope="module")
def sanitized_binary(tmp_path_factory):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    out = tmp_path_factory.mktemp("native") / "test_core_asan"
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fopenmp", "-ffp-contract=off", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", f"-I{ROOT}/csrc/include",
           *[os.path.join(ROOT, s) for s in SOURCES], "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300)
    return out


def test_core_under_asan_ubsan(sanitized_binary):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1", OMP_NUM_THREADS="4")
    r = subprocess.run([str(sanitized_binary)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "checks, 0 failed" in r.stdout
    assert "runtime error" not in r.stderr  # UBSan report


def test_fma_array_rounds_once():
    """The emulators' rounding primitive (bindings: fma_array) is the IEEE fused multiply-add of stencil.hpp: a·b + c
    rounded once — it differs from the twice-rounded numpy a * b + c exactly where the product's rounding error
    matters (here (1 + 2⁻³⁰)² − 1 keeps the 2⁻⁶⁰ term the plain product loses)."""
    import numpy as np

    from mpi_cuda_amd._native import load

    e = 2.0 ** -30
    a = np.array([1.0 + e, 3.0, 0.1])
    b = np.array([1.0 + e, 7.0, 0.3])
    c = np.array([-1.0, 1.0, -0.03])
    r = np.asarray(load().fma_array(a, b, c))
    assert r[0] == 2 * e + e * e and (a[0] * b[0] + c[0]) == 2 * e
    assert r[1] == 22.0
    assert abs(r[2] - (0.1 * 0.3 - 0.03)) <= 2 * np.spacing(0.03)
