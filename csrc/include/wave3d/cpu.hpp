// CPU path: sequential / OpenMP solver kernels on the same local layout as the GPU path.
//
// Covers the reference's sequential (wave.cpp) and OpenMP (openmpwave.cpp) programs (readme.md:33-36, report.pdf
// p.20-21 §5.1-5.2) and is the bit-exact baseline the HIP kernels are tested against.
#pragma once

#include "wave3d/decomp.hpp"
#include "wave3d/problem.hpp"

namespace wave3d {

// Local compute sub-box (local node indices, half-open).
struct LBox {
  i64 x0 = 0, x1 = 0, y0 = 0, y1 = 0, z0 = 0, z1 = 0;
  bool empty() const { return x1 <= x0 || y1 <= y0 || z1 <= z0; }
  i64 count() const { return empty() ? 0 : (x1 - x0) * (y1 - y0) * (z1 - z0); }
};

inline LBox compute_box(const Layout& l) { return LBox{l.cx0, l.cx1, l.cy0, l.cy1, l.cz0, l.cz1}; }

// Shell / interior split of a rank's compute box for the overlapped single-step schedule: the interior is the box minus
// one layer on every side that has a neighbour (nb[axis][side]); the shell is the rest, in ≤ 6 disjoint boxes (x faces
// whole, y faces inside the x range, z faces inside x and y). The one definition: GpuSolver and the Python side
// (mpi_cuda_amd.parallel.decomp.split_boxes, through the binding) both call it.
inline void shell_split(const LBox& full, const bool nb[3][2], std::vector<LBox>& shell, LBox& interior) {
  shell.clear();
  interior = full;
  if (nb[0][0]) interior.x0 += 1;
  if (nb[0][1]) interior.x1 -= 1;
  if (nb[1][0]) interior.y0 += 1;
  if (nb[1][1]) interior.y1 -= 1;
  if (nb[2][0]) interior.z0 += 1;
  if (nb[2][1]) interior.z1 -= 1;
  auto push = [&](LBox b) {
    if (!b.empty()) shell.push_back(b);
  };
  if (!full.empty()) {
    const i64 ix0 = imin(imax(interior.x0, full.x0), full.x1), ix1 = imax(interior.x1, ix0);
    const i64 iy0 = imin(imax(interior.y0, full.y0), full.y1), iy1 = imax(interior.y1, iy0);
    if (nb[0][0]) push(LBox{full.x0, full.x0 + 1, full.y0, full.y1, full.z0, full.z1});
    if (nb[0][1]) push(LBox{imax(full.x1 - 1, full.x0 + (nb[0][0] ? 1 : 0)), full.x1, full.y0, full.y1, full.z0, full.z1});
    if (nb[1][0]) push(LBox{ix0, ix1, full.y0, full.y0 + 1, full.z0, full.z1});
    if (nb[1][1]) push(LBox{ix0, ix1, imax(full.y1 - 1, full.y0 + (nb[1][0] ? 1 : 0)), full.y1, full.z0, full.z1});
    if (nb[2][0]) push(LBox{ix0, ix1, iy0, iy1, full.z0, full.z0 + 1});
    if (nb[2][1]) push(LBox{ix0, ix1, iy0, iy1, imax(full.z1 - 1, full.z0 + (nb[2][0] ? 1 : 0)), full.z1});
  }
  if (interior.x1 < interior.x0 || interior.y1 < interior.y0 || interior.z1 < interior.z0) interior = LBox{};
}

// Shell / interior split of a deep-tb unit whose exchange overlaps the rest of the pass (GpuSolver::tb_split). The
// neighbours need the w = (next pass depth) nodes next to each face with a neighbour (edges and corners included). In
// y and z the shell is made of whole rows / columns of the pass's tile grid (tile edge T ≥ w), so the shell boxes
// recompute nothing the interior also computes; a remainder row narrower than w is replaced by the w rows next to
// the face (its own one-row box: the core ends a row earlier). In z every cut lies an EVEN number of nodes from the
// box's first node (the remainder box is widened to keep it so), so every sub-box starts and — unless it ends at the
// rank's last node — ends on a whole 16-byte pair: the pair-tiled pass stores whole pairs and never writes a node of
// another box. In x the shell is w planes of the remaining (y, z) core (recomputing S − 1 planes at the seam).
// Boxes: the y border rows (whole x, whole z), the z border columns of the rows between (whole x), then the core's
// x-face slabs; the interior is the core between the x slabs. Slab ranks (neighbours in x only): the two x slabs.
inline void deep_split(const LBox& full, const bool nb[3][2], i64 w, i64 T, std::vector<LBox>& shells,
                       LBox& interior) {
  shells.clear();
  interior = full;
  // core range along a tiled axis: the border is the first / last tile row of the box, or — when the last row is a
  // remainder narrower than w — the w (z: w rounded to a whole pair from the box start) rows next to the face
  auto grid = [&](i64 b0, i64 b1, bool lo, bool hi, bool pair, i64& c0, i64& c1) {
    const i64 nt = ceil_div(b1 - b0, T), rem = (b1 - b0) - (nt - 1) * T;
    c0 = lo ? imin(b0 + T, b1) : b0;
    i64 cut = rem >= w ? b0 + (nt - 1) * T : b1 - w;
    if (pair) cut = b0 + ((cut - b0) & ~i64{1});
    c1 = hi ? imax(cut, c0) : b1;
  };
  i64 ya, yb, za, zb;
  grid(full.y0, full.y1, nb[1][0], nb[1][1], false, ya, yb);
  grid(full.z0, full.z1, nb[2][0], nb[2][1], true, za, zb);
  auto add = [&](const LBox& b) {
    if (!b.empty()) shells.push_back(b);
  };
  add(LBox{full.x0, full.x1, full.y0, ya, full.z0, full.z1});
  add(LBox{full.x0, full.x1, yb, full.y1, full.z0, full.z1});
  add(LBox{full.x0, full.x1, ya, yb, full.z0, za});
  add(LBox{full.x0, full.x1, ya, yb, zb, full.z1});
  interior = LBox{full.x0, full.x1, ya, yb, za, zb};
  if (interior.empty()) {
    interior = LBox{};
    return;
  }
  if (nb[0][0]) {
    add(LBox{full.x0, imin(full.x0 + w, full.x1), ya, yb, za, zb});
    interior.x0 = imin(full.x0 + w, full.x1);
  }
  if (nb[0][1]) {
    const i64 x = imax(full.x1 - w, interior.x0);
    add(LBox{x, full.x1, ya, yb, za, zb});
    interior.x1 = x;
  }
}

// Resume / loaded-field start: the rank's padded local array (owned nodes and every ghost layer that lies inside the
// domain; ghosts beyond the global boundary and the row padding 0) from a GLOBAL (N+1)³ C-order field. With ghosts
// of any depth filled from the global field, the first pass after a resume needs no halo exchange.
void global_to_local(const Layout& l, const double* global, double* local);


// Error accumulator: L∞ and Σe² over the updated (interior) nodes.
struct ErrAcc {
  double max = 0.0;
  double sum = 0.0;
};

// Set the OpenMP thread count (<=0 keeps the runtime default). Returns the effective count.
int cpu_set_threads(int n);
int cpu_max_threads();

// u0 = φ and u1 = u0 + τ²/2 Δ_h u0 over the whole local allocation, ghosts included (they are analytic, so no halo
// exchange is needed before the first leapfrog step). `s` = &sin_table_ext[1].
void cpu_init_first(const Layout& l, const Coeffs& c, const double* s, double* u0, double* u1);

// u^{n+1} = 2u^n − u^{n−1} + τ²Δ_h u^n on `box`, written in place over u^{n−1} (`old_out`).
// If acc != nullptr also accumulates the error vs the analytic solution φ·ct over the box.
void cpu_leapfrog(const Layout& l, const Coeffs& c, const double* cur, double* old_out, const LBox& box,
                  const double* s, double ct, ErrAcc* acc);

// Error of a stored field vs φ·ct over `box` (used for step 1 and for the standalone error check).
void cpu_error(const Layout& l, const double* u, const LBox& box, const double* s, double ct, ErrAcc* acc);

// Pack / unpack one y or z face between the field and a contiguous buffer (x faces are contiguous already).
void cpu_pack_face(const Layout& l, const Face& f, const double* u, double* buf);
void cpu_unpack_face(const Layout& l, const Face& f, const double* buf, double* u);

}  // namespace wave3d

// ------------------------------------------------------------------------------------------------------------------
// Whole-domain CPU solver (the reference's sequential `wave` / OpenMP `wave3dOMP` programs).
// ------------------------------------------------------------------------------------------------------------------
#include <vector>

namespace wave3d {

struct CpuResult {
  std::vector<int> steps;
  std::vector<double> max_err, rms_err;
  double solve_s = 0.0, init_s = 0.0, compute_s = 0.0, check_s = 0.0;
  // the reference's CPU phase columns (report.pdf p.16): boundary = halo faces packed / unpacked,
  // exchange = waiting for the neighbours (and the final error reduction); ranks: each the max over ranks
  double boundary_s = 0.0, exchange_s = 0.0;
  // the slowest rank's own init / compute / boundary / exchange (they add up to its solve time; the per-phase maxima
  // above come from different ranks and overlap in time)
  double slow_phases[4] = {0.0, 0.0, 0.0, 0.0};
  bool finite = true;
};

class CpuSolver {
 public:
  CpuSolver(const Problem& p, int check_every = 2, int threads = 0);
  CpuResult run();
  // Start every following run() at step n0 from u^{n0−1} = prev and u^{n0} = cur (global (N+1)³ fields) instead of
  // the analytic initial condition: the leapfrog continues to K and checks the steps after n0.
  void set_state(const double* prev_global, const double* cur_global, int n0);
  // u^K (which = 0) or u^{K-1} (which = 1), padded local layout (single rank = whole domain).
  const std::vector<double>& field(int which) const { return which == 0 ? u_[final_] : u_[1 - final_]; }
  const Layout& layout() const { return lay_; }
  std::vector<int> check_steps() const;

 private:
  Problem prob_;
  int check_every_;
  Layout lay_;
  std::vector<double> u_[2];
  std::vector<double> s_;
  int final_ = 1;
  int resume_n_ = 0;                     // > 0: start step of a resumed run
  std::vector<double> resume_[2];        // local u^{n0−1}, u^{n0}
};

}  // namespace wave3d
