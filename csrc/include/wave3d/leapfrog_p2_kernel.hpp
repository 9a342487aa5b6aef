// The pair-tiled S-step LDS pass (k_leapfrog_p2): S = 2..5 leapfrog steps per HBM pass, every thread holding TWO
// z-adjacent nodes (a 16-byte pair) of a 32 × 32 (y,z) tile marching along x. Instantiated in kernels_leapfrog_p2*.hip;
// design notes and measurements: kernels_leapfrog_p2.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <string>
#include <type_traits>

#include "wave3d/kernels.hpp"
#include "wave3d/stencil.hpp"

namespace wave3d {
namespace p2k {

constexpr int kT = 32;      // output tile edge (y and z)
constexpr int kNT = 1024;   // threads per workgroup: 16 waves, 4 per SIMD (128 VGPRs each)
constexpr int kTabWave = 15;  // the wave that holds no positions
constexpr unsigned kOob = 0xFFFFFFF0u;  // buffer offset beyond every plane: loads return 0, stores are dropped

// Geometry of an S-step tile (region coordinates: row a = y − (ty0 − (S−1)), z_r = z − (tz0 − E)).
//   stage-1 region: rows [0, HY), z_r ∈ [0, HZ); its z extent is rounded out to whole 16-byte pairs (E ≥ S − 1, even)
//   level-0 (u^n) planes add a one-pair ring: rows −1..HY, pair columns −1..PZ (row stride R0 pairs)
//   levels 1..S−1 live in compact planes of HY rows × R1 pairs
// R0, R1 ≡ 4 (mod 8) pairs: a ds_write_b128 serves 8 lanes per LDS cycle (8 × 16 B = 128 B, banks (addr/4) mod 32),
// and the inner waves' lanes 0–7 hold pair columns 0–3 of two rows: R ≡ 4 (mod 8) puts the second row's four pairs on
// the other half of the 128 B (MI355X_MICROARCH.md §LDS).
template <int S>
struct Geo {
  static_assert(S >= 2 && S <= 5, "p2: S must be 2..5");
  static constexpr int E = (S / 2) * 2;
  static constexpr int HY = kT + 2 * (S - 1);
  static constexpr int HZ = kT + 2 * E;
  static constexpr int PZ = HZ / 2;
  static constexpr int NP = HY * PZ;
  static constexpr int pad4(int v) { return v + ((4 - v % 8) + 8) % 8; }
  static constexpr int R0 = pad4(PZ + 2);
  static constexpr int P0 = (HY + 2) * R0;
  static constexpr int R1 = pad4(PZ);
  static constexpr int P1 = HY * R1;
  static constexpr int G1 = R1 + 1;   // guard pairs before / after the compact block (edge reads stay inside LDS)
  static constexpr int NY = HY + 4;   // y sin table: a ∈ [−2, HY + 2)
  static constexpr int NZ = HZ + 8;   // z sin table: z_r ∈ [−4, HZ + 4)
  // (in pairs) level-0 slots [0, 2·P0), then the compact levels (the analytic start needs no more: φ and its
  // neighbours are table products)
  static constexpr int lk0() { return 2 * P0 + G1; }
  static constexpr int pairs() { return lk0() + 2 * (S - 1) * P1 + G1; }
  static constexpr int tab_doubles(int nxt) { return NY + NZ + nxt; }
};

template <int S>
constexpr size_t p2_lds_bytes(int nxt) {
  return static_cast<size_t>(Geo<S>::pairs()) * 16 + static_cast<size_t>(Geo<S>::tab_doubles(nxt)) * 8;
}
// x sin table length for a chunk of xlen planes: x ∈ [x0 − S − 1, x1 + S + 2]
template <int S>
constexpr int p2_nxt(int xlen) {
  return xlen + 2 * S + 4;
}

// ---------------------------------------------------------------------------------------------------------------
// Thread → position table (compile time). Per thread: the pair (a, b) it owns (region rows a, pair columns b: nodes
// z_r = 2b, 2b+1), and its WAVE's role: kind 1 = region pairs with stage count `lv` (the wave computes stages 1..lv),
// kind 2 = ring pairs of the u^n plane (load + commit only), 0 = none.
//   * waves 0–7: the tile's own 32 × 32 nodes (level S: every stage), wave w = tile rows 4w..4w+3, one row per
//     ds_read_b128 lane group ({0–3,12–15,20–27}, …: MI355X_MICROARCH.md §LDS), so each y-neighbour read of a group is
//     256 contiguous bytes (conflict-free at any row stride);
//   * the remaining region pairs in "onion" order (pairs needed by more stages first), 64 per wave, each wave computing
//     only the stages its deepest pair needs; the chunks go to the SIMD (wave w ↦ SIMD w mod 4) with the least stage
//     work so far — the four SIMDs end within one stage-set of each other;
//   * the u^n ring pairs fill two of the remaining waves; wave 15 holds no positions (it only loads the tables).
// Idle lanes of a partial wave duplicate that wave's first pair (same loads, same values to the same LDS slot).
struct Tab {
  int d[kNT];
};
constexpr int tab_enc(int a, int b, int lv, int kind) { return (a + 2) | ((b + 2) << 8) | (lv << 16) | (kind << 20); }

template <int S>
constexpr int pair_level(int a, int b) {
  using G = Geo<S>;
  int lv = 0;
  for (int k = 1; k <= S; ++k) {
    const bool row = a >= k - 1 && a < G::HY - (k - 1);
    const int zlo = G::E - (S - k), zhi = G::E + kT + (S - k);
    const bool col = 2 * b + 1 >= zlo && 2 * b < zhi;
    if (row && col) lv = k;
  }
  return lv;
}

// LDS bank-friendly lane order of a 64-pair chunk (onion / ring waves): lane l gets a pair whose slot index is ≡
// kTgt[l] (mod 16), so the 16 lanes of each ds_read_b128 group ({0–3,12–15,20–27}, …) hit 16 different 16-byte bank
// quads and the 8 lanes of each ds_write_b128 block 8 different ones (MI355X_MICROARCH.md §LDS); pairs without a
// matching lane fill the rest. (Row-major chunks measured 2× the conflict-free LDS cycles: profiles/r5/lds_banks.md.)
constexpr int kTgt[64] = {0,  1,  2,  3,  4,  5,  6,  7,  0,  1,  2,  3,  4,  5,  6,  7,   //
                          8,  9,  10, 11, 12, 13, 14, 15, 8,  9,  10, 11, 12, 13, 14, 15,  //
                          0,  1,  2,  3,  4,  5,  6,  7,  0,  1,  2,  3,  4,  5,  6,  7,   //
                          8,  9,  10, 11, 12, 13, 14, 15, 8,  9,  10, 11, 12, 13, 14, 15};
// (the read groups: {0–3,12–15,20–27} gets 0–3, 4–7, 12–15 + 8–11; {4–11,16–19,28–31} gets 4–7, 0–3, 8–11, 12–15 —
// all 16 residues once; every contiguous 8-lane write block holds residues r and r+4 … distinct mod 8)
constexpr void bank_order(const int* ea, const int* eb, int n, int rstride, int rbase, int* oa, int* ob) {
  bool used[64] = {};
  int lane_e[64] = {};
  bool filled[64] = {};
  for (int l = 0; l < 64; ++l) {
    for (int j = 0; j < n; ++j)
      if (!used[j] && (((ea[j] + rbase) * rstride + eb[j]) % 16 + 16) % 16 == kTgt[l]) {
        used[j] = true;
        lane_e[l] = j;
        filled[l] = true;
        break;
      }
  }
  int j = 0;
  for (int l = 0; l < 64; ++l) {
    if (filled[l]) continue;
    while (j < n && used[j]) ++j;
    if (j < n) {
      used[j] = true;
      lane_e[l] = j;
    } else {
      lane_e[l] = -1;  // (an idle lane)
    }
  }
  int first = -1;  // idle lanes repeat the pair of the lowest filled lane
  for (int l = 0; l < 64 && first < 0; ++l)
    if (lane_e[l] >= 0) first = lane_e[l];
  for (int l = 0; l < 64; ++l) {
    const int e = lane_e[l] >= 0 ? lane_e[l] : first;
    oa[l] = ea[e];
    ob[l] = eb[e];
  }
}

// the 5-step load passes' halo waves by geometry (make_tab); W3D_EXPERIMENT_ONION: the onion order there too (A/B)
template <int S>
constexpr bool kBandTab =
#ifdef W3D_EXPERIMENT_ONION
    false;
#else
    S == 5;
#endif

template <int S>
struct TabBuild {
  Tab t{};
  int ring_left = 0;  // ring pairs without a lane (must be 0)
  int inner_ok = 1;   // the level-S pairs are exactly the 512 pairs of waves 0–7
};

template <int S>
constexpr TabBuild<S> make_tab() {
  using G = Geo<S>;
  TabBuild<S> r{};
  for (int i = 0; i < kNT; ++i) r.t.d[i] = 0;
  int grp[64] = {}, gpos[64] = {};
  const int rng[4][3][2] = {{{0, 3}, {12, 15}, {20, 27}},
                            {{4, 11}, {16, 19}, {28, 31}},
                            {{32, 35}, {44, 47}, {52, 59}},
                            {{36, 43}, {48, 51}, {60, 63}}};
  for (int g = 0; g < 4; ++g) {
    int n = 0;
    for (int q = 0; q < 3; ++q)
      for (int l = rng[g][q][0]; l <= rng[g][q][1]; ++l) {
        grp[l] = g;
        gpos[l] = n++;
      }
  }
  for (int w = 0; w < 8; ++w)
    for (int l = 0; l < 64; ++l) {
      const int a = S - 1 + 4 * w + grp[l], b = G::E / 2 + gpos[l];
      if (pair_level<S>(a, b) != S) r.inner_ok = 0;
      r.t.d[w * 64 + l] = tab_enc(a, b, S, 1);
    }
  int nin = 0;
  for (int a = 0; a < G::HY; ++a)
    for (int b = 0; b < G::PZ; ++b)
      if (pair_level<S>(a, b) == S) ++nin;
  if (nin != 512) r.inner_ok = 0;
  // the other region pairs, deepest first (onion order: each wave computes only the stages its pairs need). The
  // 5-step load passes take them by geometry instead (kBandTab): first the side bands beside the tile rows — 16 rows,
  // left and right columns together in one wave — then the top / bottom bands, deepest first. A side-band wave then
  // loads 32 lines per plane where an onion-ring wave touched up to 50 (one or two pairs of each of ~45 rows), and a
  // tile's halo loads 105 lines per plane instead of 170; it computes 56 instead of 54 stage-waves per plane
  // (profiles/r6/band/).
  int la[kNT] = {}, lb[kNT] = {}, ll[kNT] = {};
  int n = 0;
  auto push = [&](int a, int b) {
    if (n < kNT) {
      la[n] = a;
      lb[n] = b;
      ll[n] = pair_level<S>(a, b);
      ++n;
    }
  };
  if constexpr (kBandTab<S>) {
    const int a0 = S - 1, b0 = G::E / 2;
    for (int h = 0; h < 2; ++h)
      for (int a = a0 + 16 * h; a < a0 + 16 * h + 16; ++a)
        for (int b = 0; b < G::PZ; ++b)
          if (b < b0 || b >= b0 + kT / 2) push(a, b);
    for (int lv = S - 1; lv >= 1; --lv)
      for (int a = 0; a < G::HY; ++a)
        if (a < a0 || a >= a0 + kT)
          for (int b = 0; b < G::PZ; ++b)
            if (pair_level<S>(a, b) == lv) push(a, b);
  } else {
    for (int lv = S - 1; lv >= 1; --lv)
      for (int a = 0; a < G::HY; ++a)
        for (int b = 0; b < G::PZ; ++b)
          if (pair_level<S>(a, b) == lv) push(a, b);
  }
  bool used[16] = {};
  for (int w = 0; w < 8; ++w) used[w] = true;
  used[kTabWave] = true;
  int load[4] = {2 * S, 2 * S, 2 * S, 2 * S};
  const int nch = (n + 63) / 64;
  for (int c = 0; c < nch; ++c) {
    int best = -1;
    for (int s = 0; s < 4; ++s) {
      const bool fr = !used[8 + s] || !used[12 + s];
      if (fr && (best < 0 || load[s] < load[best])) best = s;
    }
    if (best < 0) {
      r.inner_ok = 0;
      break;
    }
    const int w = !used[8 + best] ? 8 + best : 12 + best;
    used[w] = true;
    const int cn = n - c * 64 < 64 ? n - c * 64 : 64;
    int lv = 0;  // (the wave's stage count: its deepest pair's)
    for (int l = 0; l < cn; ++l) lv = ll[c * 64 + l] > lv ? ll[c * 64 + l] : lv;
    load[best] += lv;
    int oa[64] = {}, ob[64] = {};
    bank_order(la + c * 64, lb + c * 64, cn, G::R1, 0, oa, ob);  // (the compact level planes: most of the accesses)
    for (int l = 0; l < 64; ++l) r.t.d[w * 64 + l] = tab_enc(oa[l], ob[l], lv, 1);
  }
  // u^n ring: row −1, row HY, then pair columns −1 and PZ
  int ra[4 * kNT / 4] = {}, rb[4 * kNT / 4] = {};
  int m = 0;
  for (int b = 0; b < G::PZ; ++b) {
    ra[m] = -1;
    rb[m++] = b;
  }
  for (int b = 0; b < G::PZ; ++b) {
    ra[m] = G::HY;
    rb[m++] = b;
  }
  for (int a = 0; a < G::HY; ++a) {
    ra[m] = a;
    rb[m++] = -1;
  }
  for (int a = 0; a < G::HY; ++a) {
    ra[m] = a;
    rb[m++] = G::PZ;
  }
  int q = 0;
  for (int w = 8; w < 16 && q < m; ++w) {
    if (used[w]) continue;
    used[w] = true;
    const int cn = m - q < 64 ? m - q : 64;
    int oa[64] = {}, ob[64] = {};
    // (ring waves only write the level-0 plane: slot ((a + 1)·R0 + b + 1))
    int sa[64] = {}, sb[64] = {};
    for (int l = 0; l < cn; ++l) {
      sa[l] = ra[q + l];
      sb[l] = rb[q + l] + 1;
    }
    bank_order(sa, sb, cn, G::R0, 1, oa, ob);
    for (int l = 0; l < 64; ++l) r.t.d[w * 64 + l] = tab_enc(oa[l], ob[l] - 1, 0, 2);
    q += cn;
  }
  r.ring_left = m - q;
  return r;
}

// ---------------------------------------------------------------------------------------------------------------
// One output box of a launch: its (y, z) tile grid times its x chunks, from logical workgroup blk0 on. A launch takes
// up to kP2Boxes boxes (the overlapped schedules' shell boxes in one grid: they fill the GPU together where each alone
// left CUs idle, profiles/r6/).
struct P2Box {
  int x0, x1, xlen, nxc;  // output x range; chunk length and count
  int y0, z0, y1, z1;     // output (y, z) box (local)
  int nty, ntz, blk0;
  int gxl, gxh;           // u^{n+S−1} also on plane x0 − 1 / x1 (LeapfrogTbTiling::ghost_x1)
};
constexpr int kP2Boxes = kP2MaxBoxes;
struct P2Params {
  const double* prev;  // u^{n−1} (x base: local plane x at (x + 1)·plane, as TbParams)
  const double* cur;   // u^n
  double* out1;        // u^{n+S−1}
  double* out2;        // u^{n+S}
  const double* s;     // sin table, global index −1..N+1
  Partial* partials;   // stage k's block of partials at (k−1)·lstride
  i64 plane;
  int pitch, ya, za;        // in-plane element of local (y, z): (y + ya)·pitch + z + za
  int ay0, ay1;             // allocated local y rows
  int sx0, sx1, ax0, ax1;   // x range where stage values are real; allocated planes
  int N, gx0, gy0, gz0;
  P2Box box[kP2Boxes];
  int nbox, nactive;        // boxes; workgroups with a tile (Σ over the boxes)
  int chunked, xlen_max;    // some box is split into x chunks; its longest chunk (the LDS x sin table)
  int nblocks, xcd_remap, xper, lstride;
  int check_mask;
  double tau2, half_tau2;
  double ct[5];
#ifdef W3D_EXPERIMENT_WGTIME
  unsigned long long* wgtime;  // (perf study) 4 wall-clock stamps per workgroup, pinned host memory
#endif
};

// cache-policy bits of the plane loads / stores (gfx950 CPol: 1 = sc0, 2 = nt, 16 = sc1): non-temporal stores (the new
// levels are read by the next pass, two planes later at the earliest), default-policy loads (the tile halos are read
// again by the neighbouring tiles of the same XCD)
constexpr int kStoreAux = 2;
constexpr int kLoadAux = 0;
__device__ __forceinline__ void p2_barrier() {
  // LDS writes done, then the workgroup barrier; global loads stay in flight (a __syncthreads() would add vmcnt(0))
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// f(integral_constant<int, I>) for I = B..E−1: indices stay compile-time constants before SROA (a `#pragma unroll`
// loop is unrolled after it, and a local array indexed in a not-yet-unrolled loop is demoted to scratch)
template <int B, int E, class Fn>
__device__ __forceinline__ void static_for(Fn&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// max(|e|, m) in one v_max_f64 with the |·| source modifier (fmax() adds a canonicalising v_max_f64 of the loop-carried
// accumulator per use; for the finite, non-negative values here both give the same result)
__device__ __forceinline__ double max_abs(double e, double m) {
  double r;
  asm("v_max_f64 %0, |%1|, %2" : "=v"(r) : "v"(e), "v"(m));
  return r;
}

// a 16-byte pair (a plain aggregate: HIP's double2 is a union wrapper that SROA does not always split)
struct D2 {
  double x, y;
};
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lchar;
typedef __attribute__((address_space(3))) double ldouble;
typedef double dv2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) dv2 lD2;
__device__ __forceinline__ D2 as_d2(u32x4 v) { return __builtin_bit_cast(D2, v); }
__device__ __forceinline__ u32x4 as_u4(D2 v) { return __builtin_bit_cast(u32x4, v); }
__device__ __forceinline__ D2 D2m(double x, double y) { return D2{x, y}; }

// (static: one copy per translation unit; each TU instantiates the S it needs)
static_assert(make_tab<2>().inner_ok && make_tab<2>().ring_left == 0, "p2 table S=2");
static_assert(make_tab<3>().inner_ok && make_tab<3>().ring_left == 0, "p2 table S=3");
static_assert(make_tab<4>().inner_ok && make_tab<4>().ring_left == 0, "p2 table S=4");
static_assert(make_tab<5>().inner_ok && make_tab<5>().ring_left == 0, "p2 table S=5");
static __constant__ Tab kTab2 = make_tab<2>().t;
static __constant__ Tab kTab3 = make_tab<3>().t;
static __constant__ Tab kTab4 = make_tab<4>().t;
static __constant__ Tab kTab5 = make_tab<5>().t;
template <int S>
__device__ __forceinline__ int p2_desc(int tid) {
  if constexpr (S == 2) return kTab2.d[tid];
  else if constexpr (S == 3) return kTab3.d[tid];
  else if constexpr (S == 4) return kTab4.d[tid];
  else return kTab5.d[tid];
}

// ---------------------------------------------------------------------------------------------------------------
// The pass. Iteration i (x march, phase F = (i − i0) & 3, static inside the 4-iteration blocks):
//   barrier; commit u^n plane i+1 (loaded one iteration ago) to level-0 slot (i+1)&1; load u^n plane i+2 and u^{n−1}
//   plane i+1; stage k = 1..S computes u^{n+k} at plane i − (k−1) from level k−1 (x neighbours and the centre from
//   the thread's register queue, y/z neighbours from LDS written one iteration earlier) and writes it to its LDS slot
//   (k < S) and, for the tile's own pairs at k ≥ S−1, to HBM.
// Every wave issues the same vector-memory sequence per iteration (2 loads, 2 stores; buffer offsets beyond the plane
// for pairs that must not touch memory: the range check returns 0 / drops the store). gfx950 counts loads and stores
// in one in-order vmcnt: with a wave-dependent sequence the compiler's count is the minimum over paths and the commit
// of u^n waits for the previous iteration's stores; with one sequence it waits for exactly the load it needs.
// Register queues: plane x of level j at slot (x − i0) & 3 (a 16-byte pair each), u^{n−1} at (x − i0) & 1.
// LDS addressing: three per-thread byte bases (level-0 slots, compact levels 1–2, compact levels 3–4), every access
// an immediate offset from one of them (a 1024-thread workgroup has 128 VGPRs per lane: no room for one address
// register per plane).
//
// Perf-attribution builds only (results wrong; tools/build.py W3D_EXTRA_DEFS_P2=-D…, profiles/r5/p2_attribution.md):
//   W3D_EXPERIMENT_NOLOAD    every plane load hits one of 4 resident planes (no HBM reads)
//   W3D_EXPERIMENT_NOSTORE   the pass writes nothing to HBM
//   W3D_EXPERIMENT_NOBARRIER the per-plane barrier removed
//   W3D_EXPERIMENT_NOCHECK   no fused error check; W3D_EXPERIMENT_NORED no partial reduction
//   W3D_EXPERIMENT_WGTIME    (results right) each workgroup's wall clock at entry, march start, march end and exit
// Variants measured and removed (their numbers stay in profiles/r5/: store_experiments.md, memops/README.md,
// p2_attribution.md): deferred stores, two-plane-ahead prefetch, staggered waves, conditional queue writes, the late
// u^n load point, row-major halo lanes, split stores in the analytic start, stores from every wave, a separate
// interior-tile body, Dirichlet selects after every stage, the ring waves loading u^{n−1}, a φ plane in LDS.
template <int S, int CM, bool INIT, bool CH>
__global__ __launch_bounds__(kNT) void k_leapfrog_p2(const P2Params p) {
  using G = Geo<S>;
  constexpr int E = G::E, R0 = G::R0, R1 = G::R1;
  // late loads (S ≥ 4): u^n plane i+2 right after the commit (into plane i−2's dead slot), u^{n−1} plane i+1 after
  // stage 1 (into the register stage 1 just consumed); the vector-memory sequence of an iteration is load, load,
  // stores — the next commit waits for its load, never for a store
  constexpr bool kLate = !INIT && S >= 4;
  // split stores (5-step passes): the own waves store level S, the other 8 waves level S−1 (below)
  constexpr bool kSplitSt = !INIT && S == 5;
  extern __shared__ double lds[];
  const int tid = static_cast<int>(threadIdx.x);
#ifdef W3D_EXPERIMENT_WGTIME
  auto stamp = [&](int j) __attribute__((always_inline)) {
    if (tid == 0) p.wgtime[static_cast<size_t>(blockIdx.x) * 4 + j] = wall_clock64();
  };
#else
  auto stamp = [](int) __attribute__((always_inline)) {};
#endif
  stamp(0);
  int blk = static_cast<int>(blockIdx.x);
  if (p.xcd_remap) {  // XCD k (= blockIdx % 8 in dispatch order) takes the k-th contiguous range of xper blocks
    const int j = blk >> 3;
    blk = j < p.xper ? (blk & 7) * p.xper + j : (1 << 30);
  }
  const bool active = blk < p.nactive;
  // this workgroup's box (wave-uniform: a scalar search over ≤ kP2Boxes boxes)
  int bi = 0;
  static_for<1, kP2Boxes>([&](auto kc) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    if (k < p.nbox && blk >= p.box[k].blk0) bi = k;
  });
  const P2Box B = p.box[bi];
  // error-check accumulators, one per node of the pair (lo, hi) and checked level; a pair's nodes that are not checked
  // (Dirichlet, or beyond the box) are masked out once, in the reduction, not at every plane
  // (registers: ≤ 3 checked levels, in the 5-step passes and the 4-step analytic start — the production passes; the
  // others are at or near 128 VGPRs already)
  constexpr bool kSplitAcc = __builtin_popcount(CM) <= 3 && (S == 5 || (INIT && S == 4));
  double emax[S][2], esum[S][2];
  static_for<0, S>([&](auto kc) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    emax[k][0] = esum[k][0] = emax[k][1] = esum[k][1] = 0.0;
  });
  bool okl = false, okh = false;  // this thread's nodes are own + real: checked

  if (active) {
    blk -= B.blk0;
    const int ntiles = B.nty * B.ntz;
    const int chunk = CH ? blk / ntiles : 0;
    if constexpr (CH) blk -= chunk * ntiles;
    const int tzi = blk % B.ntz, tyi = blk / B.ntz;
    const int ty0 = B.y0 + tyi * kT, tz0 = B.z0 + tzi * kT;
    const int wx0 = CH ? B.x0 + chunk * B.xlen : B.x0;
    const int wx1 = CH ? min(B.x1, wx0 + B.xlen) : B.x1;
    // level S−1 is computed one plane beyond the chunk on both sides; where the box side is a rank face whose
    // neighbour would otherwise send that plane, it is stored too (the 5-step passes' split stores reach plane wx1
    // one iteration after the march's last: one more iteration, its stages all outside their ranges)
    const int o1x0 = wx0 - (B.gxl && wx0 == B.x0 ? 1 : 0);
    const int o1x1 = wx1 + (B.gxh && wx1 == B.x1 ? 1 : 0);
    const int N = p.N;
    const i64 P = p.plane;
    auto inside = [&](int g) __attribute__((always_inline)) {
      return static_cast<unsigned>(g - 1) < static_cast<unsigned>(N - 1);
    };

    // ---- LDS: level-0 slots, compact levels, then the sin / row-factor tables
    lchar* const lds_base = (lchar*)(lds);  // (C-style: an address-space cast)
    double* const syw = lds + 2 * G::pairs();
    double* const szw = syw + G::NY;
    double* const sxw = szw + G::NZ;
    const int xtab0 = S + 1 - wx0;  // plane x ↔ sxw[x + xtab0]

    // ---- this thread's pair and its wave's role
    const int dsc = p2_desc<S>(tid);
    const int a = (dsc & 0xFF) - 2, b = ((dsc >> 8) & 0xFF) - 2;
    const int wd = __builtin_amdgcn_readfirstlane(dsc);
    const int wlv = (wd >> 16) & 0xF;           // region waves: stages 1..wlv
    const int wkind = (wd >> 20) & 0x3;         // 1 region, 2 ring, 0 none
    const bool act = wkind != 0;
    const bool reg = wkind == 1;
    const bool inner = reg && wlv == S;         // the tile's own pairs
    // stages this wave computes (a scalar: the stage tests must stay scalar branches, not lane masks)
    int wst = __builtin_amdgcn_readfirstlane(wkind == 1 ? wlv : 0);
    const bool winner = wst == S;               // (scalar) the tile's own pairs
    // levels this wave checks (a scalar int, re-asserted per iteration like wst: a loop-invariant bool is kept as a
    // 64-bit lane mask, and each stage's test then cost a v_cndmask + v_cmp pair to negate it)
    int wchk = __builtin_amdgcn_readfirstlane(winner ? p.check_mask : 0);
    const int y = ty0 - (S - 1) + a, z = tz0 - E + 2 * b;
    const int el = z + p.za;                    // element of the pair's first node in its row
    // (a pair with both nodes outside the global interior — the boundary row / planes' outer side, ghost rows and
    // columns beyond the global boundary — holds +0 at every level: it loads as out of range, +0, without touching
    // memory. Before, the tiles at the global z faces each fetched one more 128-B line per row that no other tile
    // reads, and as the pass's last workgroups they set its end: profiles/r6/wgtime/)
    const int gpy = p.gy0 + y, gpz = p.gz0 + z;
    const bool gin = gpy >= 1 && gpy <= N - 1 && gpz >= 0 && gpz <= N - 1;
    const bool ldv = act && gin && y >= p.ay0 && y < p.ay1 && el >= 0 && el + 2 <= p.pitch;
    const unsigned goff = ldv ? static_cast<unsigned>(((y + p.ya) * p.pitch + el) * 8) : kOob;
    const bool ry = inside(p.gy0 + y);
    const bool rl = ry && inside(p.gz0 + z), rh = ry && inside(p.gz0 + z + 1);
    const bool sty = inner && y < B.y1 && z < B.z1;      // own pair stored (z + 1 ≤ z1: the box ends on a whole pair)
    const unsigned soff = sty ? goff : kOob;
    okl = sty && rl;
    okh = sty && rh && z + 1 < B.z1;
    // Dirichlet nodes through τ²: a node outside the global interior has τ² = 0 and c = old = +0 at every level (zero
    // loads, zero φ, and this very update), so fma(0, Δ, fma(2, +0, −(+0))) = +0 — the select's value, bit for bit,
    // without 4 selects per pair and stage
    const double lam_lo = rl ? p.tau2 : 0.0, lam_hi = rh ? p.tau2 : 0.0;
    // per-thread LDS byte bases (all accesses: a compile-time offset from one of them)
    const int lo0 = (a + 1) * R0 + (b + 1);     // level-0 slot index of the pair
    const int lk = a * R1 + b;                  // compact slot index (region pairs)
    // (32-bit LDS-address-space pointers: a generic pointer is a 64-bit register pair)
    lchar* b0 = lds_base + (lo0 - R0 - 1) * 16;  // (neighbour offsets from −R0−1 pairs up: never negative)
    lchar* bA = lds_base + (G::lk0() + lk - R1 - 1) * 16;
    lchar* bB = bA + 4 * G::P1 * 16;
    lchar* rt = lds_base + (2 * G::pairs() + a + 2) * 8;                          // check: s_y of the own row
    lchar* szp = lds_base + (2 * G::pairs() + G::NY + 2 * b + 4) * 8;           // check: own (s_z, s_z+1)
    // Split stores (kSplitSt): the 8 waves that do not own the tile store level S−1 of the own pairs — lane j of
    // wave 8 + w the pair of lane j of own wave w, read back from the level's compact LDS plane one iteration after
    // it was computed — and the own waves store level S only. Every wave then issues exactly one store per iteration,
    // all of them real (before, each of the 16 waves issued two, half of them with every lane out of range), and the
    // in-order vmcnt sequence stays the same for every wave. (rt: that pair's compact-slot base; soff2: its offset)
    unsigned soff2 = kOob;
    if constexpr (kSplitSt) {
      const int d2 = p2_desc<S>(tid & (kNT / 2 - 1));
      const int a2 = (d2 & 0xFF) - 2, b2 = ((d2 >> 8) & 0xFF) - 2;
      const int y2 = ty0 - (S - 1) + a2, z2 = tz0 - E + 2 * b2, el2 = z2 + p.za;
      const bool st2 = y2 >= p.ay0 && y2 < p.ay1 && el2 >= 0 && el2 + 2 <= p.pitch && y2 < B.y1 && z2 < B.z1;
      soff2 = st2 ? static_cast<unsigned>(((y2 + p.ya) * p.pitch + el2) * 8) : kOob;
      rt = lds_base + (G::lk0() + a2 * R1 + b2 - R1 - 1) * 16 + 4 * G::P1 * 16;
    }
    // (re-declared opaque at every iteration: otherwise the loop-invariant "base + offset" of every access is hoisted
    // out of the x march into a register of its own — 15 address VGPRs and spills — instead of the offset field)
    auto opaque_bases = [&]() __attribute__((always_inline)) {
      if constexpr (kSplitSt)
        asm volatile("" : "+v"(b0), "+v"(bA), "+v"(bB), "+v"(rt), "+s"(wst), "+s"(wchk));
      else
        asm volatile("" : "+v"(b0), "+v"(bA), "+v"(bB), "+v"(rt), "+v"(szp), "+s"(wst), "+s"(wchk));
      wst = __builtin_amdgcn_readfirstlane(wst);  // (an asm output is not known uniform: re-assert it)
      wchk = __builtin_amdgcn_readfirstlane(wchk);
    };
    // slot / neighbour offsets (bytes): level-0 slot s, compact plane pl = (k−1)·2 + parity
    auto o0 = [](int sl, int dy, int dz) constexpr { return sl * G::P0 * 16 + ((dy + 1) * R0 + dz + 1) * 16; };
    auto ok_ = [](int pl, int dy, int dz) constexpr { return (pl & 3) * G::P1 * 16 + ((dy + 1) * R1 + dz + 1) * 16; };
    auto kb = [&](int pl) __attribute__((always_inline)) { return pl < 4 ? bA : bB; };

    // plane buffers: base = field + (x + 1)·plane, P·8 bytes (every in-plane offset < P)
    auto rsrc = [&](const double* f, int xs, int bytes) __attribute__((always_inline)) {
      return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(f) + static_cast<i64>(xs + 1) * P, (short)0, bytes,
                                               0x00020000);
    };
    const int pbytes = static_cast<int>(P * 8);
    // u^{n−1} is read by the region waves only (the stage-1 update); the u^n ring waves get a zero-size descriptor for
    // it — same instruction sequence, no memory traffic (a scalar: wd is wave-uniform)
    const int prev_bytes = ((wd >> 20) & 0x3) == 1 ? pbytes : 0;
    auto load_pair = [&](auto bkc, const double* f, int x) __attribute__((always_inline)) -> D2 {
#ifdef W3D_EXPERIMENT_NOLOAD
      const int xs = (x & 3) + 1;
#else
      const int xs = decltype(bkc)::value ? x : x < p.ax0 ? p.ax0 : x >= p.ax1 ? p.ax1 - 1 : x;
#endif
      return as_d2(__builtin_amdgcn_raw_buffer_load_b128(rsrc(f, xs, f == p.cur ? pbytes : prev_bytes),
                                                         static_cast<int>(goff), 0, kLoadAux));
    };
    auto store_pair = [&](D2 v, double* f, int x, unsigned off, bool real) __attribute__((always_inline)) {
#ifndef W3D_EXPERIMENT_NOSTORE
      // (a scalar offset past the plane drops the whole wave's store: the x test stays scalar)
      __builtin_amdgcn_raw_buffer_store_b128(as_u4(v), rsrc(f, x, pbytes), static_cast<int>(off),
                                             real ? 0 : static_cast<int>(0x80000000u), kStoreAux);
#else
      (void)v, (void)f, (void)x, (void)off, (void)real;
#endif
    };

    // the load passes' prologue loads (u^n planes i0 − 1, i0, i0 + 1, u^{n−1} plane i0) go out before the sin tables
    // are read, so their latency and the tables' overlap instead of following each other (the prologue took ≈ 4 µs per
    // pass and workgroup, profiles/r6/wgtime/)
    D2 pq[4] = {D2m(0.0, 0.0), D2m(0.0, 0.0), D2m(0.0, 0.0), D2m(0.0, 0.0)};
    if constexpr (!INIT) {
      const int x0p = wx0 - S + 1;  // (= i0 below)
      pq[0] = load_pair(std::false_type{}, p.cur, x0p - 1);
      pq[1] = load_pair(std::false_type{}, p.cur, x0p);
      pq[2] = load_pair(std::false_type{}, p.cur, x0p + 1);
      pq[3] = load_pair(std::false_type{}, p.prev, x0p);
    }
    {
      auto sc = [&](int g) __attribute__((always_inline)) { return p.s[g < -1 ? -1 : g > N + 1 ? N + 1 : g]; };
      for (int t = tid; t < G::NY; t += kNT) syw[t] = sc(p.gy0 + ty0 - (S - 1) - 2 + t);
      for (int t = tid; t < G::NZ; t += kNT) szw[t] = sc(p.gz0 + tz0 - E - 4 + t);
      if (p.check_mask || INIT)
        for (int t = tid; t < p2_nxt<S>(wx1 - wx0); t += kNT) sxw[t] = sc(p.gx0 + wx0 - S - 1 + t);
    }
    __syncthreads();  // tables

    // analytic start: φ and u¹ from the tables (stencil.hpp phi / init_first order: neighbours are (s_x·s_y)·s_z)
    const double fy = syw[a + 2];
    const double fzl = szw[2 * b + 4], fzh = szw[2 * b + 5];
    auto u1_at = [&](int x, int zr, bool real_yz) __attribute__((always_inline)) {
      const int xi = x + xtab0, yb = a + 2, zb = zr + 4;
      const double sxc = sxw[xi], sy = syw[yb], sz = szw[zb];
      const double cy = sxc * sy;
      const double c = cy * sz;
      const double lap = d2sum(c, (sxw[xi - 1] * sy) * sz, (sxw[xi + 1] * sy) * sz, (sxc * syw[yb - 1]) * sz,
                               (sxc * syw[yb + 1]) * sz, cy * szw[zb - 1], cy * szw[zb + 1]);
      return (real_yz && inside(p.gx0 + x)) ? first_step(c, lap, p.half_tau2) : 0.0;
    };
    auto u1_pair = [&](int x) __attribute__((always_inline)) {
      return D2m(u1_at(x, 2 * b, rl), u1_at(x, 2 * b + 1, rh));
    };
    auto phi_pair = [&](int x) __attribute__((always_inline)) {
      const double sx = sxw[x + xtab0];
      return D2m((sx * fy) * fzl, (sx * fy) * fzh);
    };
    (void)phi_pair;
    (void)u1_pair;

    // ---- register queues
    D2 L[S][4];
    static_for<0, 4 * S>([&](auto ic) __attribute__((always_inline)) {
      L[decltype(ic)::value / 4][decltype(ic)::value % 4] = D2m(0.0, 0.0);
    });
    D2 Lm[2] = {D2m(0.0, 0.0), D2m(0.0, 0.0)};
    D2 phq[2] = {D2m(0.0, 0.0), D2m(0.0, 0.0)};  // (analytic start: the pair's own φ by plane parity)
    (void)phq;

    const int i0 = wx0 - S + 1, i1 = wx1 + S - 2 + (kSplitSt && o1x1 > wx1 ? 1 : 0);
    auto xreal = [&](int x) __attribute__((always_inline)) {
      return x >= p.sx0 && x < p.sx1 && inside(p.gx0 + x);
    };

    auto rd2 = [](const lchar* base, int off) __attribute__((always_inline)) {
      const dv2 v = *reinterpret_cast<const lD2*>(base + off);
      return D2m(v.x, v.y);
    };
    auto wr2 = [](lchar* base, int off, D2 v) __attribute__((always_inline)) {
      dv2 w;
      w.x = v.x;
      w.y = v.y;
      *reinterpret_cast<lD2*>(base + off) = w;
    };
    auto rd1 = [](const lchar* base, int off) __attribute__((always_inline)) {
      return *reinterpret_cast<const volatile ldouble*>(base + off);  // (volatile: a ds_read_b64, never paired)
    };
    auto rdd = [](const lchar* base, int off) __attribute__((always_inline)) {
      return *reinterpret_cast<const ldouble*>(base + off);
    };

    // stage k at plane xp; D = (xp − i0) & 3 (static)
    auto stage = [&](auto kc, auto dc, auto bkc, int xp) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value, D = decltype(dc)::value;
      constexpr bool BK = decltype(bkc)::value;
      constexpr int sm = (D + 3) & 3, s0 = D, sp = (D + 1) & 3;
      const bool inr = BK || (xp >= wx0 - (S - k) && xp < wx1 + (S - k));
      const bool xown = BK || (xp >= wx0 && xp < wx1);
      const bool xown1 = BK || (xp >= o1x0 && xp < o1x1);  // (stores of level S−1; bulk planes are inside the box)
      D2 v = D2m(0.0, 0.0);
      if (inr && wst >= k) {  // (wave-uniform)
        const D2 c = L[k - 1][s0], xm = L[k - 1][sm], xq = L[k - 1][sp];
        D2 ym, yp;
        double zm, zq;
        if constexpr (k == 1) {
          ym = rd2(b0, o0(D & 1, -1, 0));
          yp = rd2(b0, o0(D & 1, 1, 0));
          zm = rd1(b0, o0(D & 1, 0, -1) + 8);
          zq = rd1(b0, o0(D & 1, 0, 1));
        } else {
          constexpr int pl = (k - 2) * 2 + (D & 1);
          const lchar* bk = kb(pl);
          ym = rd2(bk, ok_(pl, -1, 0));
          yp = rd2(bk, ok_(pl, 1, 0));
          zm = rd1(bk, ok_(pl, 0, -1) + 8);
          zq = rd1(bk, ok_(pl, 0, 1));
        }
        const double lapl = d2sum(c.x, xm.x, xq.x, ym.x, yp.x, zm, c.y);
        const double laph = d2sum(c.y, xm.y, xq.y, ym.y, yp.y, c.x, zq);
        const D2 o = k == 1 ? Lm[kLate ? 0 : (D & 1)] : L[k > 1 ? k - 2 : 0][s0];
        v = D2m(leapfrog(c.x, o.x, lapl, lam_lo), leapfrog(c.y, o.y, laph, lam_hi));
        if constexpr (!BK) {
          if (!xreal(xp)) v = D2m(0.0, 0.0);
        }
        if constexpr (k < S) {
          constexpr int pl = (k - 1) * 2 + (D & 1);
          wr2(kb(pl), ok_(pl, 0, 0), v);
        }
        constexpr bool kChk =
#ifdef W3D_EXPERIMENT_NOCHECK
            false;
#else
            ((CM >> (k - 1)) & 1) != 0;
#endif
        if constexpr (kChk) {
          if (((wchk >> (k - 1)) & 1) && xown) {  // (wchk: 0 outside the own waves)
            // u_a = ((s_x·s_y)·ct)·s_z (stencil.hpp analytic_row); s_x of the plane: one LDS broadcast read
            const double sxp = sxw[xp + xtab0];
            // (the analytic start and the 5-step passes hold the pair's s_y, s_z, s_z+1 in registers; the other
            // passes have no registers to spare and read them from LDS)
            constexpr bool kRegF = INIT || S == 5;
            const double rf = (sxp * (kRegF ? fy : rdd(rt, 0))) * p.ct[k - 1];
            const D2 sz = kRegF ? D2m(fzl, fzh) : rd2(szp, 0);
            // (d·d = |d|·|d|; the masks okl / okh are applied in the reduction — per plane they were 4 v_cndmask_b32
            // and a canonicalising v_max_f64 per pair and level, a quarter of the check's VALU)
            const double d0 = v.x - rf * sz.x, d1 = v.y - rf * sz.y;
            if constexpr (kSplitAcc) {
              emax[k - 1][0] = max_abs(d0, emax[k - 1][0]);
              esum[k - 1][0] = err_sq_acc(d0, esum[k - 1][0]);
              emax[k - 1][1] = max_abs(d1, emax[k - 1][1]);
              esum[k - 1][1] = err_sq_acc(d1, esum[k - 1][1]);
            } else {  // (4 or 5 checked levels: one accumulator pair per level, masked per plane — no spills)
              const double e0 = okl ? fabs(d0) : 0.0, e1 = okh ? fabs(d1) : 0.0;
              emax[k - 1][0] = fmax(e0, emax[k - 1][0]);
              esum[k - 1][0] = err_sq_acc(e0, esum[k - 1][0]);
              emax[k - 1][0] = fmax(e1, emax[k - 1][0]);
              esum[k - 1][0] = err_sq_acc(e1, esum[k - 1][0]);
            }
          }
        }
      }
      // (also when the stage is skipped: the slot's previous plane is dead either way, and an unconditional write
      // keeps it from staying live through the general iterations)
      if constexpr (k < S) L[k][s0] = v;
      if constexpr (kSplitSt && k == S) {
        if (winner) {
          store_pair(v, p.out2, xp, soff, xown);
        } else {
          constexpr int pl = (S - 2) * 2 + (D & 1);  // level S−1, plane xp: written by stage S−1 last iteration
          store_pair(rd2(rt, ok_(pl, 0, 0)), p.out1, xp, soff2, xown1);
        }
      } else if constexpr (!kSplitSt && k >= S - 1) {
        // the thread's store offset plus a scalar offset (0 for the own waves' planes, out of range otherwise).
        // Passes that load: every wave stores (non-owners beyond the plane: dropped), so every wave's vector-memory
        // sequence is the same and the compiler's waits for the loads can leave the stores in flight. The analytic
        // start loads nothing: only the own waves store (−2 %)
        if (!INIT || winner) store_pair(v, k == S ? p.out2 : p.out1, xp, soff, (k == S ? xown : xown1) && winner);
      }
    };

    // analytic start, iteration i: u¹ of plane i+2 (into L[0]) and u⁰ = φ of plane i+1 (into Lm) for the region
    // pairs. φ(i+3) is computed once per node (2 products) and kept in a register queue with φ(i+1), φ(i+2) (S = 4; the
    // S ≤ 3 starts have no registers to spare and form them again); φ(i+2)'s y/z neighbours are the products the
    // neighbouring pairs form, (s_x·s_y(a±1))·s_z and (s_x·s_y)·s_z(z−1 / z+2): four table reads and seven products
    // instead of a φ plane in LDS (measured: −1 % for the pass, profiles/r6/). Ring pairs compute u¹ from the tables.
    // Bit-identical to k_init_first: every neighbour value is the same product.
    auto init_iter = [&](auto fc, int i) __attribute__((always_inline)) {
      constexpr int F = decltype(fc)::value;
      const double sx3 = sxw[i + 3 + xtab0];
      const D2 f3 = D2m((sx3 * fy) * fzl, (sx3 * fy) * fzh);
      D2 u = D2m(0.0, 0.0);
      if (reg) {
        D2 f1, c;
        if constexpr (S == 4) {
          f1 = phq[(F + 1) & 1];  // (φ(i+1) and φ(i+3) share the parity slot: read, then replaced)
          c = phq[F & 1];
          phq[(F + 1) & 1] = f3;
        } else {
          f1 = phi_pair(i + 1);
          c = phi_pair(i + 2);
        }
        const double sx2 = sxw[i + 2 + xtab0];
        const double ry_m = sx2 * syw[a + 1], ry_p = sx2 * syw[a + 3], cy2 = sx2 * fy;
        const D2 ym = D2m(ry_m * fzl, ry_m * fzh), yp = D2m(ry_p * fzl, ry_p * fzh);
        const double zm = cy2 * szw[2 * b + 3], zq = cy2 * szw[2 * b + 6];
        const double lapl = d2sum(c.x, f1.x, f3.x, ym.x, yp.x, zm, c.y);
        const double laph = d2sum(c.y, f1.y, f3.y, ym.y, yp.y, c.x, zq);
        u = D2m(first_step(c.x, lapl, p.half_tau2), first_step(c.y, laph, p.half_tau2));
        u.x = rl ? u.x : 0.0;
        u.y = rh ? u.y : 0.0;
        if (!inside(p.gx0 + i + 2)) u = D2m(0.0, 0.0);
        // (u⁰ = φ is not 0 on every Dirichlet node — s(N) = sin(π) — so it is zeroed here)
        Lm[(F + 1) & 1] = D2m(rl ? f1.x : 0.0, rh ? f1.y : 0.0);
      } else if (act) {
        u = u1_pair(i + 2);
      }
      L[0][(F + 2) & 3] = u;  // (one store to the queue slot: SROA keeps the queue in registers)
    };

    // iteration i with phase F
    auto iteration = [&](auto fc, auto bkc, int i) __attribute__((always_inline)) {
      constexpr int F = decltype(fc)::value;
#ifndef W3D_EXPERIMENT_NOBARRIER
      p2_barrier();  // every read of the slots overwritten below (iteration i−1) is done; i−1's writes visible
#endif
      opaque_bases();
      if (act) wr2(b0, o0((F + 1) & 1, 0, 0), L[0][(F + 1) & 3]);  // u^n plane i+1 → LDS
      if constexpr (INIT) {
        init_iter(fc, i);
      } else if constexpr (!kLate) {
        L[0][(F + 2) & 3] = load_pair(bkc, p.cur, i + 2);
        Lm[(F + 1) & 1] = load_pair(bkc, p.prev, i + 1);
      } else {
        // u^n plane i+2 right after the commit: its slot (plane i−2's) has been dead since stage 2 of iteration i−1,
        // and issued here it has the whole iteration (≈ 2 µs) to arrive — after stage 2, as first built, the next
        // commit waited for it: −13 % per 5-step pass (profiles/r5/stores/abn_cur_early.log)
        L[0][(F + 2) & 3] = load_pair(bkc, p.cur, i + 2);
      }
      // (scheduling fences between the load passes' stages: the compiler would otherwise hoist later stages' LDS
      // reads into earlier ones and run out of the 128 VGPRs; the analytic start has the registers to overlap one
      // stage's reads with the last one's arithmetic, −2.3 %, profiles/r5/memops)
#define W3D_P2_STAGE(K)                                                                                       \
  if constexpr (K <= S) {                                                                                     \
    stage(std::integral_constant<int, K>{}, std::integral_constant<int, (F - (K - 1) + 8) & 3>{}, bkc,        \
          i - (K - 1));                                                                                       \
    if constexpr (!INIT) __builtin_amdgcn_sched_barrier(0);                                                   \
  }
      W3D_P2_STAGE(1)
      if constexpr (kLate) Lm[0] = load_pair(bkc, p.prev, i + 1);  // (its register freed by stage 1)
      W3D_P2_STAGE(2)
      W3D_P2_STAGE(3)
      W3D_P2_STAGE(4)
      W3D_P2_STAGE(5)
#undef W3D_P2_STAGE
    };

    // prologue: u^n planes i0−1, i0 (registers; plane i0 also to LDS), plane i0+1 and u^{n−1} plane i0 (loaded above)
    using Gen = std::false_type;
    using Bulk = std::true_type;
    if constexpr (INIT) {
      if (act) {
        L[0][3] = u1_pair(i0 - 1);
        L[0][0] = u1_pair(i0);
        L[0][1] = u1_pair(i0 + 1);
        if constexpr (S == 4) {
          phq[1] = phi_pair(i0 + 1);  // (plane i0+1: odd parity; i0+2: even)
          phq[0] = phi_pair(i0 + 2);
        }
      }
      if (reg) {
        const D2 f0 = phi_pair(i0);
        Lm[0] = D2m(rl ? f0.x : 0.0, rh ? f0.y : 0.0);  // (see init_iter)
      }
    } else {
      L[0][3] = pq[0];
      L[0][0] = pq[1];
    }
    if (act) wr2(b0, o0(0, 0, 0), L[0][0]);
    if constexpr (!INIT) {
      L[0][1] = pq[2];
      Lm[0] = pq[3];
    }
    // head blocks (general) until the first block inside the bulk range, bulk blocks, then the general tail
    const int blo = max(max(wx0, p.sx0), 1 - p.gx0) + (S - 1);
    const int bhi = min(min(wx1, p.sx1), N - p.gx0);
    int ib = i0;
    stamp(1);
    const int nhead = blo > i0 ? (blo - i0 + 3) / 4 : 0;
    for (int hb = 0; hb < nhead && ib + 3 <= i1; ++hb, ib += 4) {
      iteration(std::integral_constant<int, 0>{}, Gen{}, ib);
      iteration(std::integral_constant<int, 1>{}, Gen{}, ib + 1);
      iteration(std::integral_constant<int, 2>{}, Gen{}, ib + 2);
      iteration(std::integral_constant<int, 3>{}, Gen{}, ib + 3);
    }
    // (a known-empty vector-memory counter at the bulk loop's entry: its waits are then counted exactly)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    for (; ib + 3 < bhi; ib += 4) {
      iteration(std::integral_constant<int, 0>{}, Bulk{}, ib);
      iteration(std::integral_constant<int, 1>{}, Bulk{}, ib + 1);
      iteration(std::integral_constant<int, 2>{}, Bulk{}, ib + 2);
      iteration(std::integral_constant<int, 3>{}, Bulk{}, ib + 3);
    }
    // (whole blocks up to i1 leave ib = i1 + 1 at phase 0)
    for (; ib <= i1; ib += 4) {
      iteration(std::integral_constant<int, 0>{}, Gen{}, ib);
      if (ib + 1 > i1) break;
      iteration(std::integral_constant<int, 1>{}, Gen{}, ib + 1);
      if (ib + 2 > i1) break;
      iteration(std::integral_constant<int, 2>{}, Gen{}, ib + 2);
      if (ib + 3 > i1) break;
      iteration(std::integral_constant<int, 3>{}, Gen{}, ib + 3);
    }
    stamp(2);
  }

#ifdef W3D_EXPERIMENT_WGTIME
  __syncthreads();
  stamp(3);
#endif
#ifdef W3D_EXPERIMENT_NORED
  return;
#endif
  if (p.partials == nullptr) return;
  __shared__ double red_m[kNT / 64], red_s[kNT / 64];
  static_for<0, S>([&](auto kc) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    if constexpr ((CM >> k) & 1) {
      if ((p.check_mask >> k) & 1) {
        // (masked nodes hold finite or non-finite garbage: selected away, never added; max(+0, ·) and + 0 are exact)
        double m = emax[k][0], sm = esum[k][0];
        if constexpr (kSplitAcc) {
          m = fmax(okl ? emax[k][0] : 0.0, okh ? emax[k][1] : 0.0);
          sm = (okl ? esum[k][0] : 0.0) + (okh ? esum[k][1] : 0.0);
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
          const double om = __shfl_xor(m, o, 64);
          const double os = __shfl_xor(sm, o, 64);
          m = om > m ? om : m;
          sm = sm + os;
        }
        __syncthreads();
        if ((tid & 63) == 0) {
          red_m[tid >> 6] = m;
          red_s[tid >> 6] = sm;
        }
        __syncthreads();
        if (tid == 0) {
          double mm = red_m[0], ss = red_s[0];
          for (int w = 1; w < kNT / 64; ++w) {
            mm = red_m[w] > mm ? red_m[w] : mm;
            ss += red_s[w];
          }
          p.partials[k * p.lstride + static_cast<int>(blockIdx.x)] = make_double2(mm, ss);
        }
      }
    }
  });
}

}  // namespace p2k
}  // namespace wave3d
