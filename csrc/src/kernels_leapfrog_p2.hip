// Pair-tiled deep temporal blocking (k_leapfrog_p2, leapfrog_p2_kernel.hpp): S = 2..5 leapfrog steps per HBM pass.
//
// Why a second LDS S-step kernel. The 4-step pass of k_leapfrog_tb (one node per thread and position set) ran at
// 1.0–1.06 ms against ≈0.8 ms for its bytes, and its compute alone took 684 µs (profiles/r4/lds_read2.md): per bulk
// iteration a wave issued ≈570 instructions for 8 node-stages — 240 of them scalar (exec-mask branches per stage and
// position set, 64-bit plane pointers), 13 LDS reads + a write per node-stage, and 9 of 16 waves carried a second,
// partly empty position set that the others waited for at every barrier. S = 5 (one HBM pass fewer per 20-step
// solve) did not fit its registers. This kernel is laid out for CDNA4 from the instruction stream up:
//   * TWO z-adjacent nodes per thread (a 16-byte pair): the y neighbours of both are one ds_read_b128 each, the z
//     neighbours one ds_read_b64 each, the new values one ds_write_b128 — 5 LDS instructions per pair-stage instead of
//     10 — and the loads and stores of a pair are one buffer dwordx4 each;
//   * the tile's own 32 × 32 nodes are exactly waves 0–7 (the lane groups of ds_read_b128 each hold one tile row, so
//     every y-neighbour read is conflict-free); the halo pairs follow in "onion" order, so a wave computes only the
//     stages its deepest pair needs (stage k's region shrinks by one node per side), and the halo waves are dealt to
//     the four SIMDs by stage work (leapfrog_p2_kernel.hpp make_tab): per plane ≈54 pair-stage wave-instructions
//     where position sets × stages would be 62.5, spread within one stage over the SIMDs;
//   * stores and the check run only in waves 0–7 (wave-uniform), Dirichlet zeros are selects on SGPR lane masks
//     (all-true in interior tiles), the x tests of the general planes are scalar: the bulk iteration has no exec-mask
//     branches at all;
//   * planes are addressed through buffer resources (a 32-bit per-thread offset, the plane base in SGPRs; an offset
//     past the plane returns 0 / drops a store), and every wave issues the same vector-memory sequence, so the
//     in-order vmcnt wait of the u^n commit covers exactly its load, not the previous stores;
//   * S = 5 at 128 VGPRs: u^{n−1} and u^n are loaded late (after stages 1 and 2, into registers those stages free),
//     three per-thread LDS bases replace per-plane address registers, and the loop-invariant address folding that
//     LLVM would otherwise hoist is blocked per iteration.
// One pass is bit-identical to S single steps (stencil.hpp formulas and operation order), the analytic-start pass to
// k_init_first + S steps. Tests: tests/test_gpu_kernels.py (test_leapfrog_p2_*).
#include "wave3d/leapfrog_p2_launch.hpp"

#ifdef W3D_EXPERIMENT_WGTIME
#include <array>
#include <cstdio>
#include <cstdlib>
#include <vector>
#endif

namespace wave3d {

using namespace p2k;

namespace {

struct P2Plan {
  P2Params prm{};
  int nblocks = 0;
};

// LDS budget of a pass: the largest x chunk whose sin table still fits next to the planes (the analytic start uses
// the same planes: its φ values are table products)
int p2_max_xlen(int S) {
  const size_t cap = 160 * 1024 - 2 * 16 * sizeof(double) - 256;  // minus the reduction arrays (+ alignment slack)
  size_t base = 0;
  switch (S) {
    case 2: base = p2_lds_bytes<2>(0); break;
    case 3: base = p2_lds_bytes<3>(0); break;
    case 4: base = p2_lds_bytes<4>(0); break;
    default: base = p2_lds_bytes<5>(0); break;
  }
  if (base >= cap) return 0;
  return static_cast<int>((cap - base) / sizeof(double)) - (2 * S + 4);
}

// workgroup grid of a pass over box b: the (y, z) tile grid times the x chunks; returns the launch's block count
int p2_grid(const LBox& b, const LeapfrogTbTiling& t, int S, int* nty, int* ntz, int* xlen, int* nxc) {
  *nty = static_cast<int>(ceil_div(b.y1 - b.y0, kT));
  *ntz = static_cast<int>(ceil_div(b.z1 - b.z0, kT));
  const int tiles = *nty * *ntz;
  const i64 nxb = b.x1 - b.x0;
  i64 want = 1;
  // x chunks when the tile grid alone leaves CUs idle (at least min_chunk planes each), or when the x sin table of
  // the whole range would not fit the LDS. (At most target_blocks workgroups: one CU each. Rounding the chunk count up
  // instead put e.g. a 7 × 7-tile interior box on 294 workgroups — 256 and then a second round of 38.)
  if (t.target_blocks > tiles) want = imin(imax(1, t.target_blocks / tiles), imax(1, nxb / imax(1, t.min_chunk)));
  const int maxlen = p2_max_xlen(S);
  W3D_REQUIRE(maxlen >= 1, "leapfrog_p2: the tile does not fit in LDS");
  want = imax(want, ceil_div(nxb, maxlen));
  *xlen = static_cast<int>(ceil_div(nxb, want));
  *nxc = static_cast<int>(ceil_div(nxb, *xlen));
  return tiles * *nxc;  // (unrounded: the launch grid rounds the sum of its boxes up to whole XCD shares)
}

int p2_round(int blocks, const LeapfrogTbTiling& t) { return t.xcd_remap ? static_cast<int>(round_up(blocks, 8)) : blocks; }

// the checks a box must pass, and its grid (tiles × x chunks) as box k of a launch whose boxes before it take blk0
// workgroups
void p2_box(const Layout& l, const LBox& b, const LeapfrogTbTiling& t, const LBox& real, int blk0, P2Box& bx) {
  const int S = t.stages;
  W3D_REQUIRE(leapfrog_p2_supported(l, b, S), "leapfrog_p2: the box must lie in the rank's y/z range on whole pairs");
  // x: u^{n+k} (k < S) is read up to S−k planes beyond the box (real there, or beyond the global boundary); u^n is
  // read S planes beyond, within the allocation unless beyond the global boundary
  const bool lo_ok = real.x0 <= b.x0 - (S - 1) || l.gx0 + real.x0 <= 1;
  const bool hi_ok = real.x1 >= b.x1 + (S - 1) || l.gx0 + real.x1 >= l.N;
  W3D_REQUIRE(lo_ok && hi_ok, "leapfrog_p2: stage-1 range does not cover the box halo in x");
  W3D_REQUIRE(l.gx0 + b.x0 - S <= 0 || b.x0 - S >= -l.xg, "leapfrog_p2: halo deeper than the ghosts in x");
  W3D_REQUIRE(l.gx0 + b.x1 + S - 1 >= l.N || b.x1 + S - 1 < l.nx + l.xg, "leapfrog_p2: halo deeper than the ghosts in x");
  // y / z (3-D block ranks): u^n is read S nodes beyond the box, within the ghosts unless beyond the global boundary
  W3D_REQUIRE(l.gy0 + b.y0 - S <= 0 || b.y0 - S >= -l.yg, "leapfrog_p2: halo deeper than the ghosts in y");
  W3D_REQUIRE(l.gy0 + b.y1 + S - 1 >= l.N || b.y1 + S - 1 < l.ny + l.yg, "leapfrog_p2: halo deeper than the ghosts in y");
  W3D_REQUIRE(l.gz0 + b.z0 - S <= 0 || b.z0 - S >= -l.zg, "leapfrog_p2: halo deeper than the ghosts in z");
  W3D_REQUIRE(l.gz0 + b.z1 + S - 1 >= l.N || b.z1 + S - 1 < l.nz + l.zg, "leapfrog_p2: halo deeper than the ghosts in z");
  bx.x0 = static_cast<int>(b.x0);
  bx.x1 = static_cast<int>(b.x1);
  bx.y0 = static_cast<int>(b.y0);
  bx.z0 = static_cast<int>(b.z0);
  bx.y1 = static_cast<int>(b.y1);
  bx.z1 = static_cast<int>(b.z1);
  bx.blk0 = blk0;
  // ghost-plane stores of u^{n+S−1}: only on a side at the rank's face, within the real (computed) range
  const LBox full = compute_box(l);
  bx.gxl = (t.ghost_x1 & 1) && b.x0 == full.x0 ? 1 : 0;
  bx.gxh = (t.ghost_x1 & 2) && b.x1 == full.x1 ? 1 : 0;
  W3D_REQUIRE(!bx.gxl || (real.x0 <= b.x0 - 1 && b.x0 - 1 >= -l.xg), "leapfrog_p2: ghost plane x0 − 1 not computed");
  W3D_REQUIRE(!bx.gxh || (real.x1 >= b.x1 + 1 && b.x1 < l.nx + l.xg), "leapfrog_p2: ghost plane x1 not computed");
  bx.nty = bx.ntz = bx.nxc = 0;
  bx.xlen = 1;
  if (b.x1 > b.x0 && b.y1 > b.y0 && b.z1 > b.z0) p2_grid(b, t, S, &bx.nty, &bx.ntz, &bx.xlen, &bx.nxc);
}

// A launch over n boxes (n ≤ kP2Boxes): one grid, box k from workgroup blk0_k on. With several boxes each one's
// x-chunk target is its share of t.target_blocks by work (tiles × planes), so together they fill the GPU once.
P2Plan make_plan_p2(const Layout& l, const LBox* boxes, int n, const LeapfrogTbTiling& t, LBox real, bool init) {
  const int S = t.stages;
  W3D_REQUIRE(S >= 2 && S <= 5, "leapfrog_p2: stages must be 2..5");
  W3D_REQUIRE(!init || S <= 4, "leapfrog_p2: the analytic-start pass takes at most 4 steps");
  W3D_REQUIRE(n >= 1 && n <= kP2Boxes, "leapfrog_p2: too many boxes for one launch");
  W3D_REQUIRE(l.plane < (i64{1} << 27), "leapfrog_p2: plane too large for 32-bit buffer offsets");
  const LBox full = compute_box(l);
  if (real.x0 > real.x1) {
    real.x0 = full.x0;
    real.x1 = full.x1;
  }
  W3D_REQUIRE(real.x0 >= -l.xg && real.x1 <= l.nx + l.xg, "leapfrog_p2: real range outside the allocation in x");
  P2Plan pl;
  P2Params& p = pl.prm;
  p.plane = l.plane;
  p.pitch = static_cast<int>(l.pitch);
  p.ya = static_cast<int>(l.yg);
  p.za = static_cast<int>(l.zg + l.zs);
  p.ay0 = static_cast<int>(-l.yg);
  p.ay1 = static_cast<int>(l.ny + l.yg);
  p.sx0 = static_cast<int>(real.x0);
  p.sx1 = static_cast<int>(real.x1);
  p.ax0 = static_cast<int>(-l.xg);
  p.ax1 = static_cast<int>(l.nx + l.xg);
  p.N = static_cast<int>(l.N);
  p.gx0 = static_cast<int>(l.gx0);
  p.gy0 = static_cast<int>(l.gy0);
  p.gz0 = static_cast<int>(l.gz0);
  double work = 0.0;
  for (int k = 0; k < n; ++k)
    work += static_cast<double>(ceil_div(imax(0, boxes[k].y1 - boxes[k].y0), kT) *
                                ceil_div(imax(0, boxes[k].z1 - boxes[k].z0), kT) * imax(0, boxes[k].x1 - boxes[k].x0));
  int blk = 0;
  p.nbox = n;
  p.chunked = 0;
  p.xlen_max = 1;
  for (int k = 0; k < n; ++k) {
    LeapfrogTbTiling tk = t;
    if (n > 1 && work > 0.0) {
      const double wk = static_cast<double>(ceil_div(imax(0, boxes[k].y1 - boxes[k].y0), kT) *
                                            ceil_div(imax(0, boxes[k].z1 - boxes[k].z0), kT) *
                                            imax(0, boxes[k].x1 - boxes[k].x0));
      tk.target_blocks = imax(1, static_cast<int>(t.target_blocks * wk / work));
    }
    p2_box(l, boxes[k], tk, real, blk, p.box[k]);
    blk += p.box[k].nty * p.box[k].ntz * p.box[k].nxc;
    if (p.box[k].nxc > 1) p.chunked = 1;
    p.xlen_max = imax(p.xlen_max, p.box[k].xlen);
  }
  p.nactive = blk;
  if (blk == 0) return pl;
  pl.nblocks = p2_round(blk, t);
  p.nblocks = pl.nblocks;
  p.xcd_remap = t.xcd_remap ? 1 : 0;
  p.xper = pl.nblocks / 8;
  return pl;
}

#ifdef W3D_EXPERIMENT_WGTIME
// (perf study) every launch gets its own slot of 4 stamps per workgroup in pinned host memory (a captured launch keeps
// its slot: each replay overwrites it, so the file holds the last replay); written to $W3D_WGTIME_OUT at exit as text
// lines "launch S init nblocks" followed by one line of 4 stamps (100 MHz wall clock) per workgroup
struct WgTimeLog {
  unsigned long long* buf = nullptr;
  size_t cap = size_t{1} << 22, used = 0;
  std::vector<std::array<int, 4>> launches;  // S, init, nblocks, offset / 4
};
WgTimeLog& wgtime_log() {
  static WgTimeLog g;
  return g;
}
void wgtime_dump() {
  WgTimeLog& g = wgtime_log();
  const char* path = std::getenv("W3D_WGTIME_OUT");
  if (!path || !g.buf) return;
  FILE* f = std::fopen(path, "w");
  if (!f) return;
  for (size_t l = 0; l < g.launches.size(); ++l) {
    const auto& L = g.launches[l];
    std::fprintf(f, "launch %zu %d %d %d\n", l, L[0], L[1], L[2]);
    for (int b = 0; b < L[2]; ++b) {
      const unsigned long long* q = g.buf + (static_cast<size_t>(L[3]) + b) * 4;
      std::fprintf(f, "%llu %llu %llu %llu\n", q[0], q[1], q[2], q[3]);
    }
  }
  std::fclose(f);
}
unsigned long long* wgtime_slot(int nblocks, int S, bool init) {
  WgTimeLog& g = wgtime_log();
  if (!g.buf) {
    W3D_REQUIRE(hipHostMalloc(reinterpret_cast<void**>(&g.buf), g.cap * sizeof(unsigned long long),
                              hipHostMallocDefault) == hipSuccess,
                "wgtime: pinned buffer");
    std::atexit(wgtime_dump);
  }
  if (nblocks == 0) return g.buf;
  W3D_REQUIRE(g.used + static_cast<size_t>(nblocks) * 4 <= g.cap, "wgtime: log full");
  unsigned long long* q = g.buf + g.used;
  g.launches.push_back({S, init ? 1 : 0, nblocks, static_cast<int>(g.used / 4)});
  g.used += static_cast<size_t>(nblocks) * 4;
  return q;
}
#endif

}  // namespace

bool leapfrog_p2_supported(const Layout& l, const LBox& box, int stages) {
  // any box inside the rank's compute range in y/z (the whole range: one rank, x slabs, a 3-D block's whole box; or a
  // sub-box: the overlapped block schedule's shells and interior, cpu.hpp deep_split) whose pairs start on 16-byte
  // nodes and which ends on a whole pair unless it ends at the rank's last node: the pass stores whole pairs, so a box
  // ending in the middle of a pair would also write the first node of the next box (beyond the rank's last node the
  // second node of a pair is a ghost, which the next exchange rewrites)
  const LBox full = compute_box(l);
  return stages >= 2 && stages <= 5 && l.yg >= 1 && l.zg >= 1 && box.y0 >= full.y0 && box.y1 <= full.y1 &&
         box.z0 >= full.z0 && box.z1 <= full.z1 && (box.z0 + l.zg + l.zs) % 2 == 0 &&
         (box.z1 == full.z1 || (box.z1 - box.z0) % 2 == 0);
}

int leapfrog_p2_partials(const Layout& l, const LBox& box, const LeapfrogTbTiling& t) {
  // (the largest block count over S = 2..5: the chunk length shrinks with S, whose levels share the LDS with the
  // chunk's x sin table — ADVICE r5: S = 2 alone undercounted boxes longer than the S = 5 chunk)
  (void)l;
  if (box.x1 <= box.x0 || box.y1 <= box.y0 || box.z1 <= box.z0) return 0;
  int n = 0, nty = 0, ntz = 0, xlen = 0, nxc = 0;
  for (int S = 2; S <= 5; ++S) n = imax(n, p2_round(p2_grid(box, t, S, &nty, &ntz, &xlen, &nxc), t));
  return n;
}

std::vector<int> leapfrog_p2_table(int stages, std::vector<long>* geometry) {
  auto one = [&](auto sc) {
    constexpr int S = decltype(sc)::value;
    using G = p2k::Geo<S>;
    constexpr p2k::TabBuild<S> t = p2k::make_tab<S>();
    if (geometry)
      *geometry = {G::E, G::HY, G::HZ, G::PZ, p2k::kT,
                   static_cast<long>(p2k::p2_lds_bytes<S>(p2k::p2_nxt<S>(512))),
                   S <= 4 ? static_cast<long>(p2k::p2_lds_bytes<S>(p2k::p2_nxt<S>(512))) : 0L,
                   static_cast<long>(p2_max_xlen(S)), S <= 4 ? static_cast<long>(p2_max_xlen(S)) : 0L};
    return std::vector<int>(t.t.d, t.t.d + p2k::kNT);
  };
  switch (stages) {
    case 2: return one(std::integral_constant<int, 2>{});
    case 3: return one(std::integral_constant<int, 3>{});
    case 4: return one(std::integral_constant<int, 4>{});
    case 5: return one(std::integral_constant<int, 5>{});
    default: fail("leapfrog_p2_table: stages must be 2..5");
  }
  return {};
}

void leapfrog_p2_prepare() {
#ifdef W3D_EXPERIMENT_WGTIME
  wgtime_slot(0, 0, false);  // (the pinned buffer, before any capture)
#endif
  prepare_p2_s2();
  prepare_p2_s3();
  prepare_p2_s4();
  prepare_p2_s5();
}

void launch_leapfrog_p2_boxes(const Layout& l, const Coeffs& c, const double* prev, const double* cur, double* out1,
                              double* out2, const LBox* boxes, int nbox, const double* d_s, const double* ct,
                              int check_mask, Partial* partials, const LeapfrogTbTiling& t, hipStream_t stream,
                              const LBox& real, bool analytic_start, int level_stride, int grid_blocks) {
  W3D_REQUIRE(out1 != out2 && (analytic_start || (prev != out1 && prev != out2 && cur != out1 && cur != out2)),
              "leapfrog_p2 needs four distinct buffers");
  P2Plan pl = make_plan_p2(l, boxes, nbox, t, real, analytic_start);
  if (pl.nblocks == 0) return;
  P2Params& p = pl.prm;
  if (grid_blocks > 0) {
    W3D_REQUIRE(grid_blocks >= pl.nblocks && (!t.xcd_remap || grid_blocks % 8 == 0), "leapfrog_p2: bad grid_blocks");
    // (the padded grid's extra blocks get no tile: xper stays the active blocks' per-XCD share, else the remap would
    // hand every tile to the first XCDs — measured: a slab rank's 256 tiles on 4 of 8 XCDs, passes 2.2x slower)
    pl.nblocks = p.nblocks = grid_blocks;
  }
  const i64 kb = (l.xg - 1) * l.plane;  // x base only: in-plane offsets are plane-relative
  p.prev = analytic_start ? out1 + kb : prev + kb;  // (the analytic start reads neither: any valid buffer)
  p.cur = analytic_start ? out2 + kb : cur + kb;
  p.out1 = out1 + kb;
  p.out2 = out2 + kb;
  p.s = d_s;
  p.tau2 = c.lam;
  p.half_tau2 = c.half_lam;
  p.check_mask = partials != nullptr ? (check_mask & ((1 << t.stages) - 1)) : 0;
  p.partials = p.check_mask != 0 ? partials : nullptr;
  W3D_REQUIRE(level_stride == 0 || level_stride >= pl.nblocks, "leapfrog_p2: level stride below the block count");
  p.lstride = level_stride > 0 ? level_stride : pl.nblocks;
  for (int k = 0; k < 5; ++k) p.ct[k] = (ct != nullptr && k < t.stages) ? ct[k] : 0.0;
#ifdef W3D_EXPERIMENT_WGTIME
  p.wgtime = wgtime_slot(pl.nblocks, t.stages, analytic_start);
#endif
  switch (t.stages) {
    case 2: launch_p2_s2(p, pl.nblocks, analytic_start, stream); break;
    case 3: launch_p2_s3(p, pl.nblocks, analytic_start, stream); break;
    case 4: launch_p2_s4(p, pl.nblocks, analytic_start, stream); break;
    default: launch_p2_s5(p, pl.nblocks, analytic_start, stream); break;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) fail(std::string("leapfrog_p2 launch: ") + hipGetErrorString(e));
}

void launch_leapfrog_p2(const Layout& l, const Coeffs& c, const double* prev, const double* cur, double* out1,
                        double* out2, const LBox& box, const double* d_s, const double* ct, int check_mask,
                        Partial* partials, const LeapfrogTbTiling& t, hipStream_t stream, const LBox& real,
                        bool analytic_start, int level_stride, int grid_blocks) {
  launch_leapfrog_p2_boxes(l, c, prev, cur, out1, out2, &box, 1, d_s, ct, check_mask, partials, t, stream, real,
                           analytic_start, level_stride, grid_blocks);
}

}  // namespace wave3d
