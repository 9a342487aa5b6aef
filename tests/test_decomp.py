"""Decomposition / layout / halo-plan invariants (SURVEY.md §4.2 unit row): every node owned exactly once for many P,
uneven splits, balanced interior work, aligned pairs, symmetric neighbour and face plans, 64-bit sizes."""

import numpy as np
import pytest


@pytest.mark.parametrize("P", [1, 2, 3, 4, 7, 8, 10, 16, 20, 32])
@pytest.mark.parametrize("decomp", ["slab", "block"])
@pytest.mark.parametrize("N", [16, 63, 512])
def test_partition_covers_every_node_once(C, P, decomp, N):
    if decomp == "slab" and P > N - 1:
        pytest.skip("more slabs than interior planes")
    prob = C.Problem(N, 1e-3, 20, 1.0)
    dims = C.parse_dims(decomp, P, N)
    assert dims.size() == P
    n = N + 1
    count = np.zeros((n, n, n), dtype=np.int8) if n <= 64 else None
    total = 0
    for r in range(P):
        b = C.rank_box(prob, dims, r)
        assert b.x1 > b.x0 and b.y1 > b.y0 and b.z1 > b.z0
        total += b.count()
        if count is not None:
            count[b.x0:b.x1, b.y0:b.y1, b.z0:b.z1] += 1
    assert total == n ** 3
    if count is not None:
        assert (count == 1).all()


def test_split_balances_interior(C):
    # 511 interior planes over 8 ranks: 63 or 64 updated planes each, boundary nodes on the end ranks
    sizes = []
    for c in range(8):
        b, e = C.split_axis(512, 8, c)
        sizes.append((b, e))
    assert sizes[0][0] == 0 and sizes[-1][1] == 513
    upd = [min(e, 512) - max(b, 1) for b, e in sizes]
    assert max(upd) - min(upd) <= 1 and sum(upd) == 511


def test_block_dims_prefers_cubes(C):
    assert C.block_dims(8, 512).as_tuple() == (2, 2, 2)
    assert C.block_dims(2, 512).as_tuple() == (2, 1, 1)
    assert C.block_dims(4, 512).as_tuple() == (2, 2, 1)
    assert C.block_dims(1, 512).as_tuple() == (1, 1, 1)
    assert C.parse_dims("1x2x4", 8, 512).as_tuple() == (1, 2, 4)
    with pytest.raises(RuntimeError):
        C.parse_dims("3x3x1", 8, 512)
    with pytest.raises(RuntimeError):
        C.parse_dims("nonsense", 8, 512)


@pytest.mark.parametrize("P,decomp", [(2, "slab"), (8, "block"), (12, "block"), (6, "1x2x3"), (27, "3x3x3")])
def test_neighbors_and_faces_are_symmetric(C, P, decomp):
    prob = C.Problem(64, 1e-3, 20, 1.0)
    dims = C.parse_dims(decomp, P, 64)
    plans = {}
    lays = {}
    for r in range(P):
        lays[r] = C.make_layout(prob, C.rank_box(prob, dims, r))
        plans[r] = C.make_halo_plan(lays[r], dims, r)
    for r in range(P):
        for f in plans[r].faces:
            peer_faces = [g for g in plans[f.peer].faces if g.peer == r]
            assert len(peer_faces) == 1
            g = peer_faces[0]
            assert g.axis == f.axis and g.side == 1 - f.side and g.count == f.count
            if f.contiguous:
                # x-face neighbours share the (y,z) box, hence the row layout
                assert lays[r].pitch == lays[f.peer].pitch and lays[r].zs == lays[f.peer].zs


@pytest.mark.parametrize("N,P,decomp", [(512, 1, "slab"), (512, 8, "block"), (100, 3, "1x1x3"), (37, 5, "1x5x1")])
def test_layout_alignment(C, N, P, decomp):
    prob = C.Problem(N, 1e-3, 20, 1.0)
    dims = C.parse_dims(decomp, P, N)
    for r in range(P):
        lay = C.make_layout(prob, C.rank_box(prob, dims, r))
        assert lay.pitch % 16 == 0
        assert lay.off(lay.cx0, 0, lay.cz0) % 2 == 0 or lay.cz1 <= lay.cz0  # first updated node pair-aligned
        assert lay.pitch >= lay.nz + 2 + lay.zs + 2
        assert lay.total == (lay.nx + 2) * (lay.ny + 2) * lay.pitch


def test_64bit_sizes(C):
    prob = C.Problem(2048, 2.5e-4, 20, 1.0)
    lay = C.make_layout(prob, C.rank_box(prob, C.Dims(1, 1, 1), 0))
    assert lay.total > 2 ** 31
    assert lay.total * 8 * 2 < 288e9  # both leapfrog levels of 2049³ fit one MI355X
    lay8 = C.make_layout(prob, C.rank_box(prob, C.block_dims(8, 2048), 7))
    assert lay8.off(lay8.nx, lay8.ny, lay8.nz) < lay8.total


def test_python_split_boxes_match_native(C):
    """The Python shell/interior split partitions the compute box (same rule as the native GpuSolver)."""
    from mpi_cuda_amd.parallel.decomp import plan, split_boxes

    for P, d in [(8, "2x2x2"), (4, "slab"), (6, "1x2x3")]:
        for r in range(P):
            p = plan(40, P, r, d)
            shell, inner = split_boxes(p.layout, p.neighbors)
            full = C.compute_box(p.layout)
            mark = np.zeros((p.layout.nx, p.layout.ny, p.layout.nz), dtype=np.int8)
            for b in shell + [inner]:
                mark[b.x0:b.x1, b.y0:b.y1, b.z0:b.z1] += 1
            sub = mark[full.x0:full.x1, full.y0:full.y1, full.z0:full.z1]
            assert (sub == 1).all() and mark.sum() == full.count()
