"""The CMake build (CMakeLists.txt) and the build driver __graft_entry__.build() uses (tools/build.py) compile the same
translation units: a source added to one and not the other would leave the CMake build linking without it."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_cmake_lists_every_build_py_source():
    import build

    cmake = open(os.path.join(ROOT, "CMakeLists.txt")).read()
    listed = set(re.findall(r"csrc/((?:src|app)/[A-Za-z0-9_]+\.(?:hip|cpp))", cmake))
    wanted = {s for s, _ in build.LIB_SOURCES + build.CLI_SOURCES}
    assert wanted <= listed, sorted(wanted - listed)
    for s in wanted | listed:
        assert os.path.exists(os.path.join(ROOT, "csrc", s)), s
