"""The overlapped deep-tb split (cpu.hpp deep_split, GpuSolver::tb_split), checked on the CPU: the shell boxes and the
interior tile the rank's compute box exactly once, the shells hold every node a neighbour receives (w deep towards
each face with a neighbour), and every z cut lies a whole 16-byte pair from the box start — the pair-tiled pass stores
whole pairs, so a box that ended mid-pair would also write the first node of the next box (round 6: this is what lets
the overlapped 3-D block schedule run the 5-step pass on its sub-boxes)."""
import itertools

import pytest

C = pytest.importorskip("mpi_cuda_amd._C")


def _nodes(b):
    x0, x1, y0, y1, z0, z1 = b.as_tuple()
    return {(x, y, z) for x in range(x0, x1) for y in range(y0, y1) for z in range(z0, z1)}


@pytest.mark.parametrize("w", [2, 3, 4, 5])
@pytest.mark.parametrize("ext", [(9, 33, 33), (7, 66, 67), (11, 40, 71), (6, 100, 35)])
@pytest.mark.parametrize("nb", [
    [[True, True], [True, True], [True, True]],
    [[False, True], [True, False], [False, True]],
    [[True, True], [False, False], [False, False]],
    [[False, False], [True, True], [False, False]],
    [[False, False], [False, False], [True, True]],
])
def test_deep_split_tiles_box_on_whole_pairs(w, ext, nb):
    nx, ny, nz = ext
    full = C.LBox(0, nx, 0, ny, 0, nz)
    shells, interior = C.deep_split(full, nb, w, 32)
    boxes = list(shells) + ([interior] if not interior.empty() else [])
    seen = {}
    for i, b in enumerate(boxes):
        assert not b.empty()
        for n in _nodes(b):
            assert n not in seen, (n, i, seen.get(n))
            seen[n] = i
    assert set(seen) == _nodes(full)  # exactly once
    inner = set(_nodes(interior)) if not interior.empty() else set()
    # every node within w of a face with a neighbour is in a shell (the exchange may start once the shells are done)
    lim = (nx, ny, nz)
    for n in _nodes(full):
        near = any((nb[a][0] and n[a] < w) or (nb[a][1] and n[a] >= lim[a] - w) for a in range(3))
        if near:
            assert n not in inner, n
    for b in boxes:
        _, _, _, _, z0, z1 = b.as_tuple()
        assert z0 % 2 == 0  # (full.z0 = 0: pairs start on even offsets)
        assert z1 == nz or (z1 - z0) % 2 == 0
    assert len(shells) < 8  # kTbSlots


def test_deep_split_no_neighbours_is_the_box():
    full = C.LBox(0, 10, 0, 20, 0, 30)
    shells, interior = C.deep_split(full, [[False, False]] * 3, 5, 32)
    assert list(shells) == [] and interior.as_tuple() == full.as_tuple()
