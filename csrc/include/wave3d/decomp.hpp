// Domain decomposition, local memory layout and halo (ghost-layer) plan.
//
// The reference splits the (N+1)^3 node grid into blocks, one per MPI rank, and exchanges one ghost layer per face
// every step (report.pdf p.4 §1 "block decomposition of the computational domain between processes"; p.16 §4.4
// exchange-time column). Here the same capability is laid out for one GPU per rank:
//   * 1-D slab (P×1×1): x-planes are contiguous in memory, so faces go to RCCL with no packing.
//   * 3-D block (px×py×pz): y/z faces are strided and go through the HIP pack/unpack kernels.
// Work is balanced over the N−1 interior nodes of each axis (the boundary nodes 0 and N are never updated), splits may
// be uneven (513 nodes over 8 ranks), and every extent/offset is 64-bit (2049³ > 2³¹).
#pragma once

#include <array>
#include <cmath>
#include <string>
#include <vector>

#include "wave3d/common.hpp"
#include "wave3d/problem.hpp"

namespace wave3d {

struct Dims {
  int px = 1, py = 1, pz = 1;
  int size() const { return px * py * pz; }
};

// Global node ranges [x0,x1) × [y0,y1) × [z0,z1).
struct Box {
  i64 x0 = 0, x1 = 0, y0 = 0, y1 = 0, z0 = 0, z1 = 0;
  i64 nx() const { return x1 - x0; }
  i64 ny() const { return y1 - y0; }
  i64 nz() const { return z1 - z0; }
  i64 count() const { return nx() * ny() * nz(); }
};

// Part c of p of the interior nodes 1..N-1, with node 0 attached to part 0 and node N to part p-1.
inline void split_axis(i64 N, int p, int c, i64* b, i64* e) {
  const i64 n_int = N - 1;
  const i64 lo = 1 + (n_int * c) / p;
  const i64 hi = 1 + (n_int * (c + 1)) / p;
  *b = (c == 0) ? 0 : lo;
  *e = (c == p - 1) ? N + 1 : hi;
}

// Factor P into px·py·pz minimising the halo surface of the local box (MPI_Dims_create analogue). Ties prefer more
// splits along x, whose faces are contiguous.
inline Dims block_dims(int P, i64 N) {
  Dims best{P, 1, 1};
  double best_cost = -1.0;
  const double n = static_cast<double>(N + 1);
  for (int px = 1; px <= P; ++px) {
    if (P % px) continue;
    for (int py = 1; py <= P / px; ++py) {
      if ((P / px) % py) continue;
      const int pz = P / px / py;
      const double ax = n / px, ay = n / py, az = n / pz;
      // faces of the busiest rank: one per axis split in two, two per axis split further
      const double fx = px > 2 ? 2.0 : px - 1.0, fy = py > 2 ? 2.0 : py - 1.0, fz = pz > 2 ? 2.0 : pz - 1.0;
      double cost = fx * ay * az + fy * ax * az + fz * ax * ay;
      // strided (y/z) faces cost more than contiguous x faces: packing + non-contiguous access
      cost += 0.125 * fy * ax * az + 0.25 * fz * ax * ay;
      const bool better = best_cost < 0.0 || cost < best_cost - 1e-9 ||
                          (std::abs(cost - best_cost) <= 1e-9 && (px > best.px || (px == best.px && py > best.py)));
      if (better) {
        best_cost = cost;
        best = Dims{px, py, pz};
      }
    }
  }
  return best;
}

// Parse "slab" | "block" | "PxQxR".
inline Dims parse_dims(const std::string& spec, int P, i64 N) {
  if (spec.empty() || spec == "slab") return Dims{P, 1, 1};
  if (spec == "block" || spec == "auto") return block_dims(P, N);
  int a = 0, b = 0, c = 0;
  char x1 = 0, x2 = 0;
  if (std::sscanf(spec.c_str(), "%d%c%d%c%d", &a, &x1, &b, &x2, &c) == 5 && (x1 == 'x' || x1 == 'X') &&
      (x2 == 'x' || x2 == 'X')) {
    W3D_REQUIRE(a >= 1 && b >= 1 && c >= 1, "decomposition factors must be >= 1");
    W3D_REQUIRE(a * b * c == P, "decomposition " + spec + " does not match world size " + std::to_string(P));
    return Dims{a, b, c};
  }
  fail("unknown decomposition '" + spec + "' (use slab, block or PxQxR)");
}

// rank = (cx·py + cy)·pz + cz
inline std::array<int, 3> rank_coords(const Dims& d, int rank) {
  return {rank / (d.py * d.pz), (rank / d.pz) % d.py, rank % d.pz};
}
inline int coords_rank(const Dims& d, int cx, int cy, int cz) { return (cx * d.py + cy) * d.pz + cz; }

inline Box rank_box(const Problem& p, const Dims& d, int rank) {
  const auto c = rank_coords(d, rank);
  Box b;
  split_axis(p.N, d.px, c[0], &b.x0, &b.x1);
  split_axis(p.N, d.py, c[1], &b.y0, &b.y1);
  split_axis(p.N, d.pz, c[2], &b.z0, &b.z1);
  return b;
}

// Neighbour across face (axis 0/1/2, side 0 = low, 1 = high), or -1 at the physical boundary (non-periodic).
inline int neighbor_rank(const Dims& d, int rank, int axis, int side) {
  auto c = rank_coords(d, rank);
  const int lim[3] = {d.px, d.py, d.pz};
  c[axis] += side ? 1 : -1;
  if (c[axis] < 0 || c[axis] >= lim[axis]) return -1;
  return coords_rank(d, c[0], c[1], c[2]);
}

// Local storage of one rank's box with xg / yg / zg ghost layers on the two sides of each axis (1 for single steps; S
// on the split axes of ranks that run S-step passes with S-deep halos):
//   offset(ix,iy,iz) = (ix+xg)·plane + (iy+yg)·pitch + (iz+zg+zs),  ix ∈ [-xg,nx+xg), iy ∈ [-yg,ny+yg), iz ∈ [-zg,nz+zg)
// zs ∈ [0,15] shifts the row so that the first updated z node sits on a 128-byte line boundary: kernels move nodes
// in 16-byte pairs (dwordx4) and a wave's 64 pairs then cover exactly eight whole 128-B lines. pitch is a multiple of
// 16 doubles (128 B, so every row starts on a line) and keeps at least two spare doubles after the last ghost node so
// the pair holding a row's right neighbour never straddles into the next row. The last of them in the last row of every
// plane is never written by anything but zeros (zero_off): kernels load it for positions outside the global interior.
struct Layout {
  i64 N = 0;
  i64 xg = 1, yg = 1, zg = 1;     // ghost layers on each side of x / y / z
  i64 nx = 0, ny = 0, nz = 0;     // owned nodes
  i64 gx0 = 0, gy0 = 0, gz0 = 0;  // global index of local node 0
  i64 zs = 0, pitch = 0, plane = 0, total = 0;
  // Local index range of the nodes this rank updates: owned ∩ global interior [1, N-1].
  i64 cx0 = 0, cx1 = 0, cy0 = 0, cy1 = 0, cz0 = 0, cz1 = 0;

  W3D_HD i64 off(i64 ix, i64 iy, i64 iz) const { return (ix + xg) * plane + (iy + yg) * pitch + (iz + zg + zs); }
  // Kernels address local node (x,y,z) at (x+1)·plane + (y+1)·pitch + (z+1+zs) from their base pointer;
  // base = field + kbase() accounts for the ghost depths.
  W3D_HD i64 kbase() const { return (xg - 1) * plane + (yg - 1) * pitch + (zg - 1); }
  // first element of plane ix (its ghost rows and row padding included)
  W3D_HD i64 plane_off(i64 ix) const { return (ix + xg) * plane; }
  // offset from a plane's first element of a slot that always holds 0 (the last padding double of its last row)
  W3D_HD i64 zero_off() const { return plane - 1; }
  W3D_HD i64 bytes() const { return total * static_cast<i64>(sizeof(double)); }
  W3D_HD bool has_work() const { return cx1 > cx0 && cy1 > cy0 && cz1 > cz0; }
};

inline Layout make_layout(const Problem& p, const Box& b, i64 pitch_align = 16, i64 xg = 1, i64 yg = 1, i64 zg = 1) {
  Layout l;
  l.N = p.N;
  l.xg = xg;
  l.yg = yg;
  l.zg = zg;
  l.nx = b.nx();
  l.ny = b.ny();
  l.nz = b.nz();
  l.gx0 = b.x0;
  l.gy0 = b.y0;
  l.gz0 = b.z0;
  auto lo = [&](i64 g0) { return imax(g0, 1) - g0; };
  auto hi = [&](i64 g0, i64 n) { return imin(g0 + n, p.N) - g0; };
  l.cx0 = lo(b.x0);
  l.cx1 = imax(l.cx0, hi(b.x0, l.nx));
  l.cy0 = lo(b.y0);
  l.cy1 = imax(l.cy0, hi(b.y0, l.ny));
  l.cz0 = lo(b.z0);
  l.cz1 = imax(l.cz0, hi(b.z0, l.nz));
  l.zs = (16 - (l.cz0 + l.zg) % 16) % 16;
  l.pitch = round_up(l.nz + 2 * l.zg + l.zs + 2, pitch_align);
  l.plane = (l.ny + 2 * l.yg) * l.pitch;
  l.total = (l.nx + 2 * l.xg) * l.plane;
  return l;
}

// One face of the halo exchange. The send region is the owned layer touching the face, the receive region is the
// ghost layer beyond it. x faces are whole contiguous planes (no packing); y/z faces are packed.
struct Face {
  int axis = 0, side = 0;
  int peer = -1;
  i64 count = 0;         // doubles per message
  bool contiguous = false;
  i64 send_off = 0;      // contiguous: offset of the first sent double in the field
  i64 recv_off = 0;      // contiguous: offset of the first received double in the field
  i64 send_layer = 0;    // local index of the sent layer along `axis`
  i64 recv_layer = 0;    // local index of the ghost layer along `axis`
  i64 pack_off = 0;      // packed: offset (doubles) of this face in the send/recv staging buffers
};

struct HaloPlan {
  std::vector<Face> faces;
  i64 packed_doubles = 0;  // total staging size per direction
  bool any() const { return !faces.empty(); }
};

inline HaloPlan make_halo_plan(const Layout& l, const Dims& d, int rank) {
  HaloPlan h;
  for (int axis = 0; axis < 3; ++axis) {
    for (int side = 0; side < 2; ++side) {
      const int peer = neighbor_rank(d, rank, axis, side);
      if (peer < 0) continue;
      Face f;
      f.axis = axis;
      f.side = side;
      f.peer = peer;
      const i64 n_along = axis == 0 ? l.nx : (axis == 1 ? l.ny : l.nz);
      f.send_layer = side ? n_along - 1 : 0;
      f.recv_layer = side ? n_along : -1;
      if (axis == 0) {
        f.contiguous = true;
        f.count = l.plane;
        f.send_off = l.plane_off(f.send_layer);
        f.recv_off = l.plane_off(f.recv_layer);
      } else {
        f.contiguous = false;
        f.count = axis == 1 ? l.nx * l.nz : l.nx * l.ny;
        f.pack_off = h.packed_doubles;
        h.packed_doubles += round_up(f.count, 32);  // keep every face 256-B aligned in the staging buffer
      }
      h.faces.push_back(f);
    }
  }
  return h;
}

}  // namespace wave3d
