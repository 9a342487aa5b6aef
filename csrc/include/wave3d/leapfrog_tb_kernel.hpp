// The LDS S-step kernel template and its launch helpers, shared by kernels_leapfrog_tb.hip (one rank, RCCL slab and
// block ranks: PUSH = false) and kernels_leapfrog_tb_push.hip (the push transport's instantiations, PUSH = true),
// compiled as two translation units in parallel. Design notes: kernels_leapfrog_tb.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <string>
#include <type_traits>

#include "wave3d/kernels.hpp"
#include "wave3d/stencil.hpp"

namespace wave3d {
namespace tbk {

constexpr int kTile = kTbTile;  // tile edge (y and z)

// Global-address-space views of pointers the kernel reads from memory (the push transport's staging pointers): a
// generic pointer would turn every load and store through it into a FLAT instruction (and, merged with the field
// pointers in a select, the hot loads of the march too)
typedef __attribute__((address_space(1))) double gdouble;

// A pointer read from the push table where it is used (volatile: type-based alias analysis would otherwise let the
// compiler hoist the load out of the march and keep the pointer in SGPRs for the whole pass — 4 more SGPR pairs, spilled)
template <class P>
__device__ __forceinline__ P tb_ptr_at(const P* slot) {
  return *static_cast<const volatile P*>(slot);
}

__device__ __forceinline__ void wave_reduce(double& m, double& s) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const double om = __shfl_xor(m, o, 64);
    const double os = __shfl_xor(s, o, 64);
    m = om > m ? om : m;
    s = s + os;
  }
}

// A y/z neighbour read from an LDS plane: one ds_read_b64 each. Plain reads of one base were paired by the compiler
// into ds_read2_b64 (13 per bulk iteration of the 4-step pass), which gfx950 serves at half the rate of two
// ds_read_b64 (32 banks x 4 B per cycle instead of 64: MI355X_MICROARCH.md §LDS); a volatile LDS-address-space read is
// never paired. Measured on one box, interleaved: 4-step pass 995 vs 1029 µs avg, analytic pass 772 vs 796 µs
// (profiles/r4/lds_read2.md); bit-identical (same operands, same operation order).
__device__ __forceinline__ double lds_rd(const double* p) {
  typedef __attribute__((address_space(3))) const volatile double lds_vd;  // (a ds_read, not FLAT)
  return *(lds_vd*)p;
}

struct TbParams {
  const double* prev;  // u^{n−1}
  const double* cur;   // u^n
  double* out1;        // u^{n+S−1}
  double* out2;        // u^{n+S}
  const double* s;     // sin table, global index −1..N+1
  Partial* partials;   // stage k's block of nblocks partials at (k−1)·lstride (checked stages only)
  i64 plane, pitch, zs;
  int x0, x1;          // output x range (local)
  int xlen, nxc;       // x chunk length and chunk count (block c marches [x0 + c·xlen, min(x1, x0 + (c+1)·xlen)))
  int sx0, sx1;        // x range where stage outputs are real (outside: Dirichlet 0)
  int ax0, ax1;        // allocated x range (local planes that may be read)
  int sy0, sy1, sz0, sz1;  // y / z ranges where stage outputs are real (3-D block ranks; whole planes: everything)
  int ay0, ay1, az0, az1;  // allocated y / z ranges (ghosts included)
  int zero_off;            // in-plane offset of the zero slot (Layout::zero_off)
  int yg, zg;              // y / z ghost depths (in-plane offsets count from the plane start)
  int N, gx0, gy0, gz0;
  int y0, y1, z0, z1;  // output (y, z) range (local)
  double ihx2, ihy2, ihz2, tau2, half_tau2;
  double ct[4];        // time factor of u^{n+k} (k = 1..S) for the check
  int check_mask;      // bit k−1: check u^{n+k}
  int nty, ntz, nblocks, xcd_remap;
  int xper;            // xcd_remap: blocks per XCD, ceil(active blocks / 8) (a padded grid's extra blocks get none)
  int lstride;         // partials between consecutive levels (≥ nblocks; larger when several launches share a level)
  int bby, bbz;        // > 0: each XCD's tiles form a bby × bbz block of the tile grid (else two-row strips)
  // slab peer-push transport (PUSH instantiations only): the per-pass parameters stay in device memory and are read
  // where they are used (pass start and end, ghost-plane loads, face-plane stores), so the march keeps only the two
  // scalars its tests need in registers (kernel arguments would all be hoisted into SGPRs and spill)
  const TbPush* push;
  int pnx, pT;         // push: this rank's planes, ghost depth
  unsigned ptag;       // push: the tag the table entry must carry
  int pacq;            // push: acquire at the pass start (TbPush::acquire)
  // fused z-face pack (TbPack; nullptr: none): nodes with z outside [pkza, pkzb) lie in a z send band of width w
  const TbPack* pk;
  int pkza, pkzb;
};

// Push transport memory protocol. The staging is fine-grained device memory (hipDeviceMallocFinegrained; W3D_PUSH_STAGING=
// uncached: uncached), the flags uncached (hipDeviceMallocUncached); the
// forwarded face values are stored with system-scope (write-through) stores and every flag / counter access is a
// system-scope atomic, so the WRITER needs no cache writeback: a workgroup's forwarded stores are all acknowledged
// (s_waitcnt before its barrier) before it counts itself done, and the workgroup that completes the count raises the
// neighbours' flags. (A system-scope release per workgroup instead writes back the whole L2 of its XCD — the field
// stores' dirty lines included: measured, a third of a pass when thousands of workgroups do it.) The READER still
// invalidates its XCD's L2 once per workgroup after the wait (system-scope acquire): the staging lines it read two
// passes earlier (same parity) may be held there, stale, while the neighbour's write-through went to HBM — measured on
// one GPU, where the neighbour runs on other XCDs: without the invalidate one solve in ~30 read a stale ghost plane.
__device__ __forceinline__ unsigned tb_flag_load(const unsigned* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Pass start: every workgroup waits until both neighbours have signalled the previous pass (their face planes are in
// this rank's staging, and they are done reading the staging this pass overwrites on their side). The wait is bounded:
// after spin_ticks of the wall clock (min(W3D_TIMEOUT_S, 60) s) the workgroup records a timeout and goes on, so a lost
// peer never leaves waves that do not finish (the host turns the status into an error).
__device__ __forceinline__ void tb_push_wait(const TbPush& q) {
  if (q.wait_epoch != 0) {
    // (after one timed-out wait the solve is lost: later passes do not wait again, so it fails in one bound, not K)
    if (threadIdx.x == 0 && __hip_atomic_load(q.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) {
      const unsigned long long t0 = wall_clock64();
      for (int s = 0; s < 2; ++s) {
        if (!q.wait_side[s]) continue;
        while (tb_flag_load(q.flags + s) < q.wait_epoch) {
          if (wall_clock64() - t0 > q.spin_ticks) {
            __hip_atomic_store(q.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
    }
    __syncthreads();
  }
  // a pass that reads ghosts from the staging (whichever way it waited: here or by the command processor)
  if ((q.gcur[0] != nullptr || q.gcur[1] != nullptr) && q.acquire)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // (system scope)
}

// Pass end: every workgroup's forwarded stores are acknowledged before it counts itself done; the last one raises the
// pass epoch in both neighbours' flag slots for this rank.
__device__ __forceinline__ void tb_push_signal(const TbPush& q) {
  if (q.signal_epoch == 0) return;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // (waits for this wave's outstanding stores)
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(q.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (old + 1 == q.done_target) {
      for (int s = 0; s < 2; ++s)
        if (q.rflag[s]) __hip_atomic_store(q.rflag[s], q.signal_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// RP (row-padded ring layout): the planes that keep the ring (level 0, the analytic start's φ level) get a row stride
// RS = H1 + 32 instead of W0 = H1 + 2. Consecutive positions then skip 32 doubles, not 2, where they cross a row end,
// so a half-wave that straddles a row still touches 32 distinct bank pairs: the ring-padded rows cost the
// compute-bound analytic pass 15 % bank-conflict cycles (PMC, profiles/r3/pass_attribution.md). Used where the wider
// planes fit: the analytic start at S ≤ 3 (its four ring-layout slots: 133 KiB at S = 3, with room for the 2048³ x
// sin table). The 4-step pass keeps W0: on a whole 2048³ box its x sin table would not fit next to the wider planes,
// and where it fits (512³) the wider layout moved a register to scratch inside the march and was measured slower.
template <int S, int T, int NT, bool RP = false>
struct TbGeom {
  static constexpr int H1 = T + 2 * (S - 1);  // stage-1 region edge: the thread-owned positions
  static constexpr int NP = H1 * H1;
  static constexpr int Q = (NP + NT - 1) / NT;  // positions per thread
  static constexpr int W0 = T + 2 * S;          // u^n region edge = LDS plane edge (all levels share the indexing)
  static constexpr int RS = RP ? H1 + 32 : W0;  // row stride of the ring-layout planes (≥ W0)
  static constexpr int PL = W0 * RS;            // a ring-layout plane: W0 rows of RS
  static constexpr int NR = W0 * W0 - NP;       // u^n halo ring (not thread-owned)
  // plane stride in LDS: the plane plus a pad holding a dummy node (and its 4 neighbours) for lanes without a position
  static constexpr int PLP = PL + 2 * RS + 2;
  static constexpr int DUMMY = PL + RS + 1;
  static constexpr int QR = (NR + NT - 1) / NT;
  // The stage levels 1..S−1 live in COMPACT planes: position idx = tid + q·NT (row a = idx / H1, column b = idx % H1)
  // at COFF + idx, row stride H1, no ring and no gap between rows, so the 16 lanes of every LDS access phase touch 16
  // consecutive doubles (all 32 banks once). In the W0-strided layout a group that straddled a row end skipped the
  // 2-column gap and hit 2 banks twice: 26 % of the LDS cycles were bank conflicts (PMC, profiles/r1_pmc_production_512.md).
  // Only level 0 (u^n, stage 1's input) needs the ring and keeps the W0 layout. Neighbours ±1, ±H1 of every lane of a
  // running wave (indices up to NPR − 1) stay inside the plane; the values read for positions outside a stage's region
  // are garbage and never used, as before.
  static constexpr int NPR = (NP + 63) / 64 * 64;
  static constexpr int COFF = H1 + 1;
  static constexpr int PLC = COFF + NPR + H1 + 1;
  // level 0 × 2 parity slots, levels 1..S−1 × 2 compact slots; the analytic start adds a φ level (two W0-layout slots)
  static constexpr int lds_planes(bool init) { return 2 * PLP + (S - 1) * 2 * PLC + (init ? 2 * PLP : 0); }
  // + (fac: checked passes that load u^n) the check's (s_z, row index) pair of every position, compact and thread-
  // private: position idx = tid + q·NT at pair idx, read at an immediate offset from the thread's own base address
  static constexpr int lds_doubles(bool init = false, bool fac = false) { return lds_planes(init) + (fac ? 2 * NP : 0); }
  static_assert(lds_planes(false) % 2 == 0 && lds_planes(true) % 2 == 0, "factor pairs must be 16-B aligned");
};

// + sin tables (error check, analytic start): y and z over the u^n region ± 1, x over the planes the pass touches ± 1.
// In LDS because a global load of the per-plane x factor would be a vector load (the table may alias the outputs, so
// no scalar load) whose wait drains the prefetch queue. nxo = tb_nx_table(x1 − x0) or 0 (no table needed).
template <bool INIT, int S>
constexpr bool tb_row_pad = INIT && S <= 3;  // TbGeom::RP per pass kind
template <int S, int T, int NT, bool INIT = false, bool FAC = false>
constexpr size_t tb_lds_bytes(int nxo = 0) {
  return (static_cast<size_t>(TbGeom<S, T, NT, tb_row_pad<INIT, S>>::lds_doubles(INIT, FAC)) +
          (2 + 2 * S) * (T + 2 * S + 2) +
          static_cast<size_t>(nxo)) *
         sizeof(double);
}
template <int S>
constexpr int tb_nx_table(int nx_box) {
  return nx_box + 2 * S + 4;
}

// CM: compile-time superset of the levels that may be checked (bit k−1 ↔ u^{n+k}); levels outside it carry no error
// accumulators or check code (registers: the S = 4 kernel sits at the 128-VGPR limit of 4 waves per SIMD).
// INIT: analytic start at n = 1 — u^{n−1} = u⁰ = φ and u^n = u¹ = u⁰ + τ²/2·Δ_h u⁰ are computed from the sin tables
// (k_init_first's formulas and operation order) instead of loaded: the pass reads nothing from HBM.
// CH: x-chunked launch (small boxes). Without it the block's x range is the kernel argument itself, which the compiler
// re-reads instead of keeping live (measured: a computed range costs the S = 4 kernel 5 % in extra spills).
template <int S, int T, int NT, int CM, bool INIT, bool CH, bool PUSH>
__global__ __launch_bounds__(NT) void k_leapfrog_tb(const TbParams p) {
  using G = TbGeom<S, T, NT, tb_row_pad<INIT, S>>;
  constexpr int Q = G::Q, QR = G::QR, H1 = G::H1, W0 = G::W0, RS = G::RS, PLP = G::PLP;
  constexpr int kOwn = 1 << 30;   // gof flag: tile node inside the output box
  constexpr int kReal = 1 << 29;  // gof flag: stage values are real at this node (interior ∩ stage-real range)
  constexpr int kLd = 1 << 28;    // gof flag: node inside the global interior and the allocation (loaded)
  constexpr int kOff = kLd - 1;   // gof bits of the in-plane offset
  // the check's per-position (s_z, row-table index) pairs in LDS (TbGeom::lds_doubles): a checked node then costs one
  // pair read, one row-factor read and the check's own f64 operations (one product, difference, max, fma); recomputing
  // the table indices from the position (divisions by W0, clamps, address arithmetic) cost more VALU instructions than
  // the check itself, and at S = 4 no registers are left to hold them
  constexpr bool kFac = CM != 0 && !INIT;
  extern __shared__ double lds[];
  const int tid = static_cast<int>(threadIdx.x);
  int blk = static_cast<int>(blockIdx.x);
  if (p.xcd_remap) {  // XCD k (= blockIdx % 8 in dispatch order) takes the k-th contiguous range of xper blocks
    const int j = blk >> 3;
    blk = j < p.xper ? (blk & 7) * p.xper + j : (1 << 30);
  }
  const int ntiles = p.nty * p.ntz;
  const bool active = blk < ntiles * (CH ? p.nxc : 1);
  // chunk-major: consecutive blocks (one XCD after the remap) are neighbouring tiles of one x chunk
  const int chunk = (CH && active) ? blk / ntiles : 0;
  if constexpr (CH) blk -= chunk * ntiles;
  int tzi = active ? blk % p.ntz : 0, tyi = active ? blk / p.ntz : 0;
  if (p.bby > 0) {  // XCD x (= blk / per after the remap) owns block x of the tile grid: halo re-reads stay in its L2
    const int per = p.bby * p.bbz, x = blk / per, w = blk - x * per, nbz = p.ntz / p.bbz;
    tyi = (x / nbz) * p.bby + w / p.bbz;
    tzi = (x - (x / nbz) * nbz) * p.bbz + (w - (w / p.bbz) * p.bbz);
  }
  const int ty0 = p.y0 + tyi * T, tz0 = p.z0 + tzi * T;
  // fused z-face pack: this tile's owned nodes reach into a z send band (wave-uniform)
  const bool pk_tile = p.pk != nullptr && (tz0 < p.pkza || imin(tz0 + T, p.z1) > p.pkzb);
  const int wx0 = CH ? p.x0 + chunk * p.xlen : p.x0;  // this block's output x range
  const int wx1 = CH ? imin(p.x1, wx0 + p.xlen) : p.x1;
  const int N = p.N;
  const i64 P = p.plane;
  // in-plane offsets count from the plane's first element (always ≥ 0, also for the y/z ghosts of block ranks):
  // node (y, z) at (y + yg)·pitch + z + zg + zs; the field pointers are offset by (xg − 1) planes only
  const int R = static_cast<int>(p.pitch), ya = p.yg, za = p.zg + static_cast<int>(p.zs);
  const double tau2 = p.tau2;  // = τ²/h² (the coefficient of d2sum)
  auto inside = [&](int g) { return static_cast<unsigned>(g - 1) < static_cast<unsigned>(N - 1); };
  auto in_rng = [](int v, int lo, int hi) { return static_cast<unsigned>(v - lo) < static_cast<unsigned>(hi - lo); };

  double emax[S], esum[S];
#pragma unroll
  for (int k = 0; k < S; ++k) emax[k] = esum[k] = 0.0;

  if constexpr (PUSH) {
    // the table entry was written by a host-to-device copy: drop any L1 / L2 line of its memory first (system-scope
    // acquire: invalidates this CU's L1 and the non-local lines of its XCD's L2)
    if (p.pacq) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if (threadIdx.x == 0 && tb_ptr_at(&p.push->tag) != p.ptag)  // the table entry this launch reads is not its own
      __hip_atomic_store(p.push->status, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    tb_push_wait(*p.push);
  }
  if (active) {
    // ---- per-thread descriptors of the owned positions (stage-1 region coordinates a, b ∈ [0, H1))
    const int zero_off = p.zero_off;
    int lid[Q];   // LDS index (u^n-region coordinates a+1, b+1); the pad's dummy node for lanes without a position
    int gof[Q];   // in-plane offset to load (zero node outside the interior) | kReal | kOwn
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int idx = tid + q * NT;
      const int a = idx / H1, b = idx - (idx / H1) * H1;
      const int y = ty0 - (S - 1) + a, z = tz0 - (S - 1) + b;
      const bool valid = idx < G::NP;
      // u^n / u^{n−1} are loaded wherever the rank holds them (its neighbours' ghost values included); the stage
      // values are real only in the stage-real range (S−1 into the ghosts)
      const bool ld = valid && inside(p.gy0 + y) && inside(p.gz0 + z) && in_rng(y, p.ay0, p.ay1) &&
                      in_rng(z, p.az0, p.az1);
      const bool real = ld && in_rng(y, p.sy0, p.sy1) && in_rng(z, p.sz0, p.sz1);
      const bool own = real && a >= S - 1 && a < S - 1 + T && b >= S - 1 && b < S - 1 + T && y < p.y1 && z < p.z1;
      lid[q] = valid ? (a + 1) * RS + (b + 1) : G::DUMMY;
      gof[q] = ld ? (((y + ya) * R + z + za) | kLd | (real ? kReal : 0) | (own ? kOwn : 0)) : zero_off;
    }
    // wave-uniform stage masks: bit k−1 of wsm[q] is set when some lane of this wave's position set q lies inside stage
    // k's region (rows [k−1, H1−k+1) of the stage-1 region); other (wave, q, stage) combinations are skipped with a
    // scalar branch (at 32² tiles and S = 4, 9 of 16 waves hold no position at all in their second set)
    int wsm[Q];
    {
      const int wbase = __builtin_amdgcn_readfirstlane(tid & ~63);
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int first = wbase + q * NT, last = imin(first + 63, G::NP - 1);
        int m = 0;
        if (first < G::NP) {
          const int rlo = first / H1, rhi = last / H1;
#pragma unroll
          for (int k = 1; k <= S; ++k)
            if (rhi >= k - 1 && rlo < H1 - (k - 1)) m |= 1 << (k - 1);
        }
        wsm[q] = __builtin_amdgcn_readfirstlane(m);
      }
    }
    // u^n halo ring: LDS index (dummy: no ring node) and global offset (zero node outside the interior)
    int lrid[QR], grof[QR];
#pragma unroll
    for (int r = 0; r < QR; ++r) {
      const int ridx = tid + r * NT;
      int a0 = 0, b0 = 0;
      if (ridx < W0) {
        b0 = ridx;
      } else if (ridx < 2 * W0) {
        a0 = W0 - 1;
        b0 = ridx - W0;
      } else if (ridx < 3 * W0 - 2) {
        a0 = 1 + ridx - 2 * W0;
      } else {
        a0 = 1 + ridx - (3 * W0 - 2);
        b0 = W0 - 1;
      }
      const int y = ty0 - S + a0, z = tz0 - S + b0;
      const bool valid = ridx < G::NR;
      lrid[r] = valid ? a0 * RS + b0 : G::DUMMY;
      grof[r] = (valid && inside(p.gy0 + y) && inside(p.gz0 + z) && in_rng(y, p.ay0, p.ay1) && in_rng(z, p.az0, p.az1))
                    ? ((y + ya) * R + z + za) | kLd
                    : zero_off;
    }
    // sin tables: syw[j] = s[y] for y = ty0 − S − 1 + j (the u^n region ± 1), szw likewise, sxw[i] = s[x] for
    // x = x0 − S − 1 + i; indices clamped into −1..N+1 (only nodes of the interior, and their neighbours, use them)
    constexpr int NYW = T + 2 * S + 2;
    double* syw = lds + G::lds_doubles(INIT, kFac);
    double2* fac = reinterpret_cast<double2*>(lds + G::lds_planes(INIT));  // (kFac)
    double* szw = syw + NYW;
    double* rowt = szw + NYW;  // per checked level, two plane-parity slots of NYW row factors s_x·s_y
    double* sxw = rowt + 2 * S * NYW;
    // push transport: the pass's eight staging pointers (TbPush fwd1, fwd2, gprev, gcur), copied into LDS once and
    // re-read from there where used — an LDS read does not wait behind the march's outstanding prefetch loads, as a
    // load from the table in device memory would (and kept in SGPRs for the whole pass they spill)
    unsigned long long* pbk =
        reinterpret_cast<unsigned long long*>(sxw + ((p.check_mask || INIT) ? tb_nx_table<S>(p.xlen) : 0));
    if constexpr (PUSH) {
      static_assert(offsetof(TbPush, gcur) == offsetof(TbPush, fwd1) + 6 * sizeof(void*), "TbPush pointer block");
      if (tid < 8) pbk[tid] = reinterpret_cast<const volatile unsigned long long*>(&p.push->fwd1[0])[tid];
    }
    // fused z-face pack: the TbPack block (4 staging pointers, w, ny, nz) likewise in LDS, read where used (a global
    // load there would wait behind the prefetch queue); first read after the march's first barrier
    unsigned long long* pkb = pbk + (PUSH ? 8 : 0);
    static_assert(sizeof(TbPack) == 6 * sizeof(unsigned long long), "TbPack block");
    if (p.pk != nullptr && tid < 6) pkb[tid] = reinterpret_cast<const volatile unsigned long long*>(p.pk)[tid];
    if (p.check_mask || INIT || PUSH) {
      auto sc = [&](int g) { return p.s[g < -1 ? -1 : g > N + 1 ? N + 1 : g]; };
      for (int t = tid; t < NYW && (p.check_mask || INIT); t += NT) {
        syw[t] = sc(p.gy0 + ty0 - S - 1 + t);
        szw[t] = sc(p.gz0 + tz0 - S - 1 + t);
      }
      if (p.check_mask || INIT)
        for (int i = tid; i < tb_nx_table<S>(wx1 - wx0); i += NT) sxw[i] = sc(p.gx0 + wx0 - S - 1 + i);
      __syncthreads();
    }
    (void)fac;
    // table indices of an LDS position li (u^n-region coordinates): y ↔ li / RS + 1, z ↔ li % RS + 1 (the pad's dummy
    // node is clamped into the table)
    auto ytab = [&](int li) { return imin(li / RS + 1, W0); };
    auto ztab = [&](int li) { return li - (li / RS) * RS + 1; };
    const int xtab0 = S + 1 - wx0;  // x ↔ sxw[x + xtab0]
    if constexpr (kFac) {
      if (p.check_mask) {  // (each thread writes and later reads only its own pairs: no barrier)
#pragma unroll
        for (int q = 0; q < Q; ++q)
          if (tid + q * NT < G::NP)
            fac[tid + q * NT] = make_double2(szw[ztab(lid[q])], __longlong_as_double(ytab(lid[q])));
      }
    }
    // staging pointer i of the pass (0, 1: fwd1 lo/hi; 2, 3: fwd2; 4, 5: gprev; 6, 7: gcur), wave-uniform
    auto push_ptr = [&](int i) -> gdouble* {
      typedef __attribute__((address_space(3))) const volatile unsigned long long lds_u64;  // (a ds_read, not FLAT)
      const unsigned long long v = ((lds_u64*)pbk)[i];
      const unsigned lo = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(v));
      const unsigned hi = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(v >> 32));
      return reinterpret_cast<gdouble*>((static_cast<unsigned long long>(hi) << 32) | lo);
    };
    (void)push_ptr;
    // analytic u⁰ = φ and u¹ at plane x, LDS position li (INIT)
    auto phi_at = [&](int x, int li) {
      return (sxw[x + xtab0] * syw[ytab(li)]) * szw[ztab(li)];
    };
    auto u1_at = [&](int x, int li, bool real_yz) {
      const int xi = x + xtab0, ya = ytab(li), zb = ztab(li);
      const double sxc = sxw[xi], sy = syw[ya], sz = szw[zb];
      const double cy = sxc * sy;
      const double c = cy * sz;
      const double lap = d2sum(c, (sxw[xi - 1] * sy) * sz, (sxw[xi + 1] * sy) * sz, (sxc * syw[ya - 1]) * sz,
                              (sxc * syw[ya + 1]) * sz, cy * szw[zb - 1], cy * szw[zb + 1]);
      return (real_yz && inside(p.gx0 + x)) ? first_step(c, lap, p.half_tau2) : 0.0;
    };

    // ---- register queues: plane x of level j at slot (x − i0) & 3; u^{n−1} and the ring: slot (x − i0) & 1
    // Stages also run on the positions outside their (shrinking) region: those values are never read by a node
    // inside the region (its neighbours lie in the previous stage's region), and skipping them per lane costs more
    // exec-mask branching than the arithmetic. Zero-initialised so every value is defined.
    // push transport: the upper face segment [wx1 − T, wx1) first, then [wx0, wx1 − T) (its S − 1 planes next to the
    // seam are recomputed: bit-identical values, not stored); otherwise one segment
    int nseg = 1;
    if constexpr (PUSH) nseg = (p.push->faces_first && wx1 == p.x1 && wx1 - wx0 > p.pT) ? 2 : 1;
    for (int seg = 0; seg < nseg; ++seg) {
    const int x0 = nseg == 1 || seg == 1 ? wx0 : wx1 - p.pT;
    const int x1 = nseg == 1 || seg == 0 ? wx1 : wx1 - p.pT;
    if (seg > 0) __syncthreads();  // the first segment's last LDS reads are done before this prologue writes LDS
    double L[S][Q][4] = {};  // L[0] = u^n, L[k] = u^{n+k} (k < S)
    double Lm[Q][2] = {};    // u^{n−1}
    double Rg[QR][2] = {};   // u^n ring
    const int i0 = x0 - S + 1, i1 = x1 + S - 2;
    auto lds_plane = [&](int j, int par) { return lds + par * PLP; };  // (level 0 only)
    (void)lds_plane;
    auto lds_cplane = [&](int k, int par) { return lds + 2 * PLP + ((k - 1) * 2 + par) * G::PLC + G::COFF; };

    // plane x of u^n: owned positions into L[0][q][slot], ring into Rg[r][rs]
    const int wbase_r = __builtin_amdgcn_readfirstlane(tid & ~63);
    // plane xs of a field: the ghost planes of a push-transport rank come from its staging (plane 0 = ghost plane −T
    // on the low side, nx on the high side)
    // (BK: a bulk plane, never a ghost plane — the push bulk range below keeps loads inside [0, pnx))
    auto plane_ptr = [&](auto bkc, const double* fld, int gi, int xs) -> const gdouble* {
      if constexpr (PUSH && !decltype(bkc)::value) {
        if (static_cast<unsigned>(xs) >= static_cast<unsigned>(p.pnx)) {  // a ghost plane (one scalar test)
          const gdouble* g = push_ptr(gi + (xs < 0 ? 0 : 1));
          if (g) return g + static_cast<i64>(xs < 0 ? xs + p.pT : xs - p.pnx) * P;
        }
      }
#ifdef W3D_EXPERIMENT_NOLOAD
      // (perf attribution only, results wrong: every plane load hits one of 4 cache-resident planes)
      return (const gdouble*)(fld) + static_cast<i64>(((xs + 1) & 3) + 1) * P;
#else
      return (const gdouble*)(fld) + static_cast<i64>(xs + 1) * P;
#endif
    };
    auto load_cur = [&](auto slot_c, auto rs_c, int x, auto bkc) {
      constexpr int slot = decltype(slot_c)::value, rs = decltype(rs_c)::value;
      if constexpr (INIT) {
#pragma unroll
        for (int q = 0; q < Q; ++q)
          if (wsm[q]) L[0][q][slot] = u1_at(x, lid[q], gof[q] & kLd);
#pragma unroll
        for (int r = 0; r < QR; ++r)
          if (wbase_r + r * NT < G::NR) Rg[r][rs] = u1_at(x, lrid[r], grof[r] & kLd);
      } else {
        // always an allocated plane (bulk iterations load planes inside the allocation by construction: no clamp)
        const int xs = decltype(bkc)::value ? x : x < p.ax0 ? p.ax0 : x >= p.ax1 ? p.ax1 - 1 : x;
        const gdouble* base = plane_ptr(bkc, p.cur, 6, xs);
#pragma unroll
        for (int q = 0; q < Q; ++q)
          if (wsm[q]) L[0][q][slot] = base[gof[q] & kOff];
#pragma unroll
        for (int r = 0; r < QR; ++r) Rg[r][rs] = base[grof[r] & kOff];
      }
    };
    auto load_prev = [&](auto slot_c, int x, auto bkc) {
      constexpr int slot = decltype(slot_c)::value;
      if constexpr (INIT) {
#pragma unroll
        for (int q = 0; q < Q; ++q)
          if (wsm[q]) Lm[q][slot] = phi_at(x, lid[q]);
      } else {
        const int xs = decltype(bkc)::value ? x : x < p.ax0 ? p.ax0 : x >= p.ax1 ? p.ax1 - 1 : x;
        const gdouble* base = plane_ptr(bkc, p.prev, 4, xs);
#pragma unroll
        for (int q = 0; q < Q; ++q)
          if (wsm[q]) Lm[q][slot] = base[gof[q] & kOff];
      }
    };
    auto commit_cur = [&](auto slot_c, auto rs_c, int par) {
      constexpr int slot = decltype(slot_c)::value, rs = decltype(rs_c)::value;
      double* d = lds_plane(0, par);
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (wsm[q]) d[lid[q]] = L[0][q][slot];
#pragma unroll
      for (int r = 0; r < QR; ++r) d[lrid[r]] = Rg[r][rs];
    };

    // ---- analytic start, φ stage: φ = (s_x·s_y)·s_z is computed once per node and plane (2 products with the
    // node's y/z factors held in registers) into a φ plane of LDS (two parity slots after the S levels); u¹ of the
    // owned positions is then first_step(φ, Δ_h φ) with the y/z neighbours from that plane and the x neighbours from
    // the thread's own entries of both φ slots. Every neighbour value is the product u1_at forms for it, so u¹ is
    // bit-identical to k_init_first's; 2 products + 4 LDS reads instead of 12 products + 9 table reads per node.
    // The halo ring (no φ neighbours beyond it in LDS) keeps u1_at.
    // (S = 4: the queues leave no room for them — the factors are re-read from the LDS tables per use instead)
    // (768-thread workgroups have 168 VGPRs per wave: the factors — and the check's row-table index — fit at S = 4 too)
    constexpr bool kFacReg = S < 4 || NT <= 768;
    double fy[Q], fz[Q], fyr[QR], fzr[QR];
    int yix[Q];  // check: row-table index of each position (kFacReg)
    // (the check's z factor of a position is re-read from the LDS table per use: keeping it in a register per position
    // spills at S = 4 since the y/z stage-real ranges of the block ranks were added)
    auto fyq = [&](int q) { return kFacReg ? fy[q] : syw[ytab(lid[q])]; };
    auto fzq = [&](int q) { return kFacReg ? fz[q] : szw[ztab(lid[q])]; };
    auto fyrr = [&](int r) { return kFacReg ? fyr[r] : syw[ytab(lrid[r])]; };
    auto fzrr = [&](int r) { return kFacReg ? fzr[r] : szw[ztab(lrid[r])]; };
    if constexpr ((INIT || (CM != 0 && !kFac)) && kFacReg) {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        yix[q] = ytab(lid[q]);
        fy[q] = syw[yix[q]];
        fz[q] = szw[ztab(lid[q])];
      }
      if constexpr (INIT) {
#pragma unroll
        for (int r = 0; r < QR; ++r) {
          fyr[r] = syw[ytab(lrid[r])];
          fzr[r] = szw[ztab(lrid[r])];
        }
      }
    }
    auto lds_phi = [&](int par) { return lds + 2 * PLP + (S - 1) * 2 * G::PLC + par * PLP; };
    // φ of plane x (owned positions and ring) into φ slot `par`
    auto phi_plane = [&](int x, int par) {
      double* d = lds_phi(par);
      const double sx = sxw[x + xtab0];
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (wsm[q]) d[lid[q]] = (sx * fyq(q)) * fzq(q);
#pragma unroll
      for (int r = 0; r < QR; ++r)
        if (wbase_r + r * NT < G::NR) d[lrid[r]] = (sx * fyrr(r)) * fzrr(r);
    };
    // iteration i of the analytic pass (F = (i − i0) & 3): u¹ of plane i+2 into L[0] slot (F+2)&3 / Rg slot (F+2)&1,
    // u⁰ = φ of plane i+1 into Lm slot (F+1)&1; φ of plane i+3 into its slot. φ slot (i+2)&1 was completed in the
    // previous iteration (behind this iteration's barrier); slot (i+3)&1 still holds this thread's φ(i+1) entries,
    // read before they are overwritten.
    auto init_iter = [&](auto fc, int i) {
      constexpr int F = decltype(fc)::value;
      double* p3 = lds_phi((F + 3) & 1);
      const double* p2 = lds_phi((F + 2) & 1);
      const double sx3 = sxw[i + 3 + xtab0];
      const bool xin = inside(p.gx0 + i + 2);
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if (!wsm[q]) continue;  // wave-uniform
        const int li = lid[q];
        const double f1 = p3[li];                    // φ(i+1), own entry
        const double f3 = (sx3 * fyq(q)) * fzq(q);   // φ(i+3)
        p3[li] = f3;
        const double c = p2[li];                     // φ(i+2)
        const double lap =
            d2sum(c, f1, f3, lds_rd(p2 + li - RS), lds_rd(p2 + li + RS), lds_rd(p2 + li - 1), lds_rd(p2 + li + 1));
        L[0][q][(F + 2) & 3] = ((gof[q] & kLd) && xin) ? first_step(c, lap, p.half_tau2) : 0.0;
        Lm[q][(F + 1) & 1] = f1;
      }
#pragma unroll
      for (int r = 0; r < QR; ++r) {
        if (wbase_r + r * NT < G::NR) {
          p3[lrid[r]] = (sx3 * fyrr(r)) * fzrr(r);
          Rg[r][(F + 2) & 1] = u1_at(i + 2, lrid[r], grof[r] & kLd);
        }
      }
    };

    // fused z-face pack (TbPack): an owned node of field f (0: u^{n+S}, 1: u^{n+S−1}) in the low / high z band of
    // width w − f goes to its place in that face's message part (C order (x, y, z) over nx × ny × (w − f))
    auto pack_store = [&](int f, int x, int idx, double v) {
      const int a = idx / H1;
      const int z = tz0 - (S - 1) + (idx - a * H1);
      if (z >= p.pkza && z < p.pkzb) return;  // (outside both bands of width w ⊇ w − 1: no LDS read)
      typedef __attribute__((address_space(3))) const volatile unsigned long long lds_u64;  // (a ds_read, not FLAT)
      const unsigned long long wy = ((lds_u64*)pkb)[4];  // w | ny << 32
      const int ny = static_cast<int>(wy >> 32), nz = static_cast<int>(((lds_u64*)pkb)[5] & 0xFFFFFFFFu);
      const int wf = static_cast<int>(wy & 0xFFFFFFFFu) - f;
      const int y = ty0 - (S - 1) + a;
      // staging part of face `side`, field f (the same in every lane: no readfirstlane, whose scalar result would make
      // the wave wait for all its outstanding LDS reads; null: no neighbour on that side)
      auto part = [&](int side) { return (gdouble*)(((lds_u64*)pkb)[side * 2 + f]); };
      if (z < wf) {
        gdouble* d = part(0);
        if (d) d[(x * ny + y) * wf + z] = v;
      }
      if (z >= nz - wf) {
        gdouble* d = part(1);
        if (d) d[(x * ny + y) * wf + z - (nz - wf)] = v;
      }
    };

    // stage k at plane xp; D = (xp − i0) & 3 (static), parity of xp = D & 1
    // BK (bulk): plane xp is real and owned for every stage (the x tests are compile-time true)
    auto stage = [&](auto kc, auto dc, auto bkc, int xp) {
      constexpr int k = decltype(kc)::value, D = decltype(dc)::value;
      constexpr bool BK = decltype(bkc)::value;
      constexpr int sm = (D + 3) & 3, s0 = D, sp = (D + 1) & 3;
      // stage 1 reads u^n (level 0, W0 layout); later stages read level k − 1 and write level k in compact planes
      const double* nb = k == 1 ? lds_plane(0, D & 1) : lds_cplane(k > 1 ? k - 1 : 1, D & 1);
      double* dst = lds_cplane(k < S ? k : 1, D & 1);
      const bool xreal = BK || (xp >= p.sx0 && xp < p.sx1 && inside(p.gx0 + xp));
      const bool xown = BK || (xp >= x0 && xp < x1);
      constexpr bool kChk = (CM >> (k - 1)) & 1;
      const bool chk = kChk && ((p.check_mask >> (k - 1)) & 1);
      double* outp = (k == S ? p.out2 : p.out1) + static_cast<i64>(xp + 1) * P;
      // the check's row factor (s_x·s_y)·ct of plane xp, tabulated one iteration ahead (row_tables), slot F & 1
      const double* rowk = rowt + ((k - 1) * 2 + ((D + k - 1) & 1)) * NYW;
      (void)xown;
      // fused z-face pack: stages S−1 and S of a tile next to a z face (scalar test)
      const bool pks = k >= S - 1 && pk_tile;
      // push transport: the face planes a neighbour reads as ghosts (u^{n+S}: T deep, u^{n+S−1}: T − 1 deep) also go
      // straight into its staging; the plane's destination is found once per stage (scalar), not per position
      gdouble* fwd = nullptr;
      if constexpr (PUSH && !BK && k >= S - 1) {  // (bulk planes are never face planes: see the push bulk range)
        const int d = k == S ? p.pT : p.pT - 1;
        if (xp < d || xp >= p.pnx - d) {
          const int side = xp < d ? 0 : 1;
          fwd = push_ptr((k == S ? 2 : 0) + side);
          if (fwd) fwd += static_cast<i64>(side ? xp - p.pnx + p.pT : xp) * P;
        }
      }
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        // wave-uniform: the mask stays an integer in an SGPR (bit test + scalar branch); hoisted out of the march as a
        // boolean it became a lane mask whose negation the compiler re-formed with two VALU ops per use
        int wm = wsm[q];
        asm volatile("" : "+s"(wm));
        if (!((wm >> (k - 1)) & 1)) continue;
        const int li = lid[q];
        const double c = L[k - 1][q][s0];
        double lap;
        if constexpr (k == 1) {
          lap = d2sum(c, L[k - 1][q][sm], L[k - 1][q][sp], lds_rd(nb + li - RS), lds_rd(nb + li + RS),
                      lds_rd(nb + li - 1), lds_rd(nb + li + 1));
        } else {
          const int lc = tid + q * NT;  // (compact index: the position itself)
          lap = d2sum(c, L[k - 1][q][sm], L[k - 1][q][sp], lds_rd(nb + lc - H1), lds_rd(nb + lc + H1),
                      lds_rd(nb + lc - 1), lds_rd(nb + lc + 1));
        }
        double o;
        if constexpr (k == 1)
          o = Lm[q][D & 1];
        else
          o = L[k - 2][q][s0];
        const int g = gof[q];
        // analytic-start pass: the update is computed for every lane and selected (the opaque register keeps the
        // compiler from wrapping it, and the neighbour reads feeding it, in an exec-masked branch): 712 vs 740 µs,
        // s_waitcnt per iteration 76 -> 55. The 4-step pass keeps the branch (1091 vs 1058 µs with the select;
        // profiles/r4/lds_read2.md)
        double v;
        if constexpr (INIT) {
          double lf = leapfrog(c, o, lap, tau2);
          asm volatile("" : "+v"(lf));
          v = (xreal && (gof[q] & kReal)) ? lf : 0.0;
        } else {
          v = (xreal && (gof[q] & kReal)) ? leapfrog(c, o, lap, tau2) : 0.0;
        }
        if constexpr (k < S) {
          L[k][q][s0] = v;
          dst[tid + q * NT] = v;
        }
        const bool own = xown && (g & kOwn);
        if constexpr (k >= S - 1) {
          if (own && xreal) {
#if defined(W3D_EXPERIMENT_PLAINSTORE)  // (experiment: write-back stores instead of non-temporal ones)
            outp[g & kOff] = v;
#elif !defined(W3D_EXPERIMENT_NOSTORE)  // (perf attribution only, results wrong: the pass writes nothing to HBM)
            __builtin_nontemporal_store(v, outp + (g & kOff));
#endif
            if (pks) pack_store(k == S ? 0 : 1, xp, tid + q * NT, v);
            if constexpr (PUSH && !BK)
              if (fwd) __hip_atomic_store(fwd + (g & kOff), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
        }
        if constexpr (kChk) {
          if (chk && own && xreal) {
            // u_a = ((s_x·s_y)·ct)·s_z (stencil.hpp::analytic_row): one product per node
            double a;
            if constexpr (kFac) {
              const double2 f = fac[tid + q * NT];  // (s_z, row-table index)
              a = rowk[static_cast<int>(__double_as_longlong(f.y))] * f.x;
            } else {
              a = rowk[kFacReg ? yix[q] : ytab(li)] * (kFacReg ? fz[q] : szw[ztab(li)]);
            }
            const double e = fabs(v - a);
            emax[k - 1] = fmax(e, emax[k - 1]);  // = (e > m ? e : m) for every non-NaN e; a NaN shows in the sum
            esum[k - 1] = err_sq_acc(e, esum[k - 1]);
          }
        }
      }
    };

    // check row factors: rowt[k][slot][j] = (s_x(plane of stage k) · s_y(j))·ct_k, the row factor of the check's
    // ((s_x·s_y)·ct)·s_z (stencil.hpp::analytic_row, same operands and order: bit-identical), tabulated once per plane
    // by the first NYW threads instead of once per node; iteration i fills slot ((i − i0) + 1) & 1 for the planes its
    // successor checks
    auto row_tables = [&](int i, int slot) {
      if constexpr (CM != 0) {
        if (p.check_mask && tid < NYW) {
#pragma unroll
          for (int k = 1; k <= S; ++k)
            if (((CM & p.check_mask) >> (k - 1)) & 1)
              rowt[((k - 1) * 2 + slot) * NYW + tid] = analytic_row(sxw[imax(i - (k - 1) + xtab0, 0)], syw[tid], p.ct[k - 1]);
        }
      }
    };

    // iteration i with phase F = (i − i0) & 3
    auto iteration = [&](auto fc, auto bkc, int i) {
      constexpr int F = decltype(fc)::value;
      constexpr bool BK = decltype(bkc)::value;
#ifndef W3D_EXPERIMENT_NOBARRIER  // (perf attribution only, results wrong: the per-plane barrier removed)
      __syncthreads();  // every read of the slots overwritten below (iteration i−1) is done; i−1's writes visible
#endif
      row_tables(i + 1, (F + 1) & 1);
      commit_cur(std::integral_constant<int, (F + 1) & 3>{}, std::integral_constant<int, (F + 1) & 1>{},
                 (F + 1) & 1);  // u^n plane i+1 → LDS (loaded one iteration ago)
      if constexpr (INIT) {
        init_iter(fc, i);
      } else {
        load_cur(std::integral_constant<int, (F + 2) & 3>{}, std::integral_constant<int, (F + 2) & 1>{}, i + 2, bkc);
        load_prev(std::integral_constant<int, (F + 1) & 1>{}, i + 1, bkc);
      }
#define W3D_TB_STAGE(K)                                                                                          \
  if constexpr (K <= S) {                                                                                        \
    const int xp = i - (K - 1);                                                                                  \
    if (BK || (xp >= x0 - (S - K) && xp < x1 + (S - K)))                                                         \
      stage(std::integral_constant<int, K>{}, std::integral_constant<int, (F - (K - 1) + 8) & 3>{}, bkc, xp);    \
  }
      W3D_TB_STAGE(1)
      W3D_TB_STAGE(2)
      W3D_TB_STAGE(3)
      W3D_TB_STAGE(4)
#undef W3D_TB_STAGE
    };

    // prologue: u^n planes i0−1, i0 (registers; plane i0 also to LDS), plane i0+1 and u^{n−1} plane i0 in flight
    load_cur(std::integral_constant<int, 3>{}, std::integral_constant<int, 1>{}, i0 - 1, std::false_type{});
    load_cur(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, i0, std::false_type{});
    commit_cur(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, 0);
    load_cur(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{}, i0 + 1, std::false_type{});
    load_prev(std::integral_constant<int, 0>{}, i0, std::false_type{});
    row_tables(i0, 0);
    if constexpr (INIT) {  // φ planes i0+1 (slot 1: read back as the x neighbour at i0) and i0+2 (slot 0)
      phi_plane(i0 + 1, 1);
      phi_plane(i0 + 2, 0);
    }
    // bulk iterations: every stage's plane i − (k−1) lies in [blo, bhi) (owned, real, inside the global interior),
    // so the per-stage x tests vanish; measured: the scalar unit (exec masks, compares, address math) was as busy as
    // the vector unit. Blocks of 4 iterations keep the register-queue slots static.
    using Gen = std::false_type;
    using Bulk = std::true_type;
    if constexpr (INIT && NT > 768) {
      // the 1024-thread analytic-start pass runs general blocks only: its register footprint (128 VGPRs) leaves no
      // room for a second copy (768 threads: 168 VGPRs, bulk blocks as below)
      for (int ib = i0; ib <= i1; ib += 4) {
        iteration(std::integral_constant<int, 0>{}, Gen{}, ib);
        if (ib + 1 > i1) break;
        iteration(std::integral_constant<int, 1>{}, Gen{}, ib + 1);
        if (ib + 2 > i1) break;
        iteration(std::integral_constant<int, 2>{}, Gen{}, ib + 2);
        if (ib + 3 > i1) break;
        iteration(std::integral_constant<int, 3>{}, Gen{}, ib + 3);
      }
    } else {
      // head blocks (general) until the first block inside the bulk range, bulk blocks, then the general tail
      int blo = imax(imax(x0, p.sx0), 1 - p.gx0) + (S - 1);
      int bhi = imin(imin(x1, p.sx1), N - p.gx0);
      if constexpr (PUSH) {
        // push: bulk blocks neither forward face planes (stage S−1 / S plane xp with xp < T or xp ≥ pnx − T) nor load
        // ghost planes (u^n plane i+2 ≥ pnx), so their push tests compile away; those iterations run general blocks
        blo = imax(blo, p.pT + S - 1);
        bhi = imin(bhi, imin(p.pnx - p.pT + S - 2, p.pnx - 2));
      }
      int ib = i0;
      const int nhead = blo > i0 ? (blo - i0 + 3) / 4 : 0;
      for (int b = 0; b < nhead && ib + 3 <= i1; ++b, ib += 4) {
        iteration(std::integral_constant<int, 0>{}, Gen{}, ib);
        iteration(std::integral_constant<int, 1>{}, Gen{}, ib + 1);
        iteration(std::integral_constant<int, 2>{}, Gen{}, ib + 2);
        iteration(std::integral_constant<int, 3>{}, Gen{}, ib + 3);
      }
      for (; ib + 3 < bhi; ib += 4) {
        iteration(std::integral_constant<int, 0>{}, Bulk{}, ib);
        iteration(std::integral_constant<int, 1>{}, Bulk{}, ib + 1);
        iteration(std::integral_constant<int, 2>{}, Bulk{}, ib + 2);
        iteration(std::integral_constant<int, 3>{}, Bulk{}, ib + 3);
      }
      for (; ib <= i1; ib += 4) {
        iteration(std::integral_constant<int, 0>{}, Gen{}, ib);
        if (ib + 1 > i1) break;
        iteration(std::integral_constant<int, 1>{}, Gen{}, ib + 1);
        if (ib + 2 > i1) break;
        iteration(std::integral_constant<int, 2>{}, Gen{}, ib + 2);
        if (ib + 3 > i1) break;
        iteration(std::integral_constant<int, 3>{}, Gen{}, ib + 3);
      }
    }
    }  // segments
  }
  if constexpr (PUSH) tb_push_signal(*p.push);

  if (p.partials == nullptr) return;
  __shared__ double red_m[NT / 64], red_s[NT / 64];
#pragma unroll
  for (int k = 0; k < S; ++k) {
    if (!((CM >> k) & 1) || !((p.check_mask >> k) & 1)) continue;
    double m = emax[k], sm = esum[k];
    wave_reduce(m, sm);
    __syncthreads();
    if ((tid & 63) == 0) {
      red_m[tid >> 6] = m;
      red_s[tid >> 6] = sm;
    }
    __syncthreads();
    if (tid == 0) {
      double mm = red_m[0], ss = red_s[0];
      for (int w = 1; w < NT / 64; ++w) {
        mm = red_m[w] > mm ? red_m[w] : mm;
        ss += red_s[w];
      }
      p.partials[k * p.lstride + static_cast<int>(blockIdx.x)] = make_double2(mm, ss);
    }
  }
}

struct TbPlan {
  TbParams prm{};
  int nblocks = 0;
};

// `real`: per axis, the local range where stage values are real (outside: Dirichlet 0 / unused); an axis with lo > hi
// takes the default (x: the compute box; y, z: the whole allocation, i.e. no restriction besides the global interior).
inline TbPlan make_plan_tb(const Layout& l, const LBox& b, const LeapfrogTbTiling& t, LBox real) {
  W3D_REQUIRE(t.stages >= 2 && t.stages <= 4, "leapfrog_tb: stages must be 2, 3 or 4");
  W3D_REQUIRE((t.threads == 768 || t.threads == 1024) && (t.init_threads == 768 || t.init_threads == 1024),
              "leapfrog_tb: threads must be 768 or 1024");
  const LBox full = compute_box(l);
  if (real.x0 > real.x1) {
    real.x0 = full.x0;
    real.x1 = full.x1;
  }
  if (real.y0 > real.y1) {
    real.y0 = -l.yg;
    real.y1 = l.ny + l.yg;
  }
  if (real.z0 > real.z1) {
    real.z0 = -l.zg;
    real.z1 = l.nz + l.zg;
  }
  W3D_REQUIRE(b.x0 >= full.x0 && b.x1 <= full.x1 && b.y0 >= full.y0 && b.y1 <= full.y1 && b.z0 >= full.z0 &&
                  b.z1 <= full.z1,
              "leapfrog_tb box outside the compute box");
  W3D_REQUIRE(l.N < (1 << 20) && l.plane < (1 << 28), "leapfrog_tb: plane too large for 28-bit in-plane offsets");
  const i64 S = t.stages;
  // per axis: u^{n+k} (k < S) is read up to S−k nodes beyond the box, so its values there must be real (the `real`
  // range) unless they lie beyond the global boundary (structural zeros); u^n is read S nodes beyond the box, within
  // the allocation (ghost depth g) unless beyond the global boundary
  auto axis_ok = [&](i64 b0, i64 b1, i64 r0, i64 r1, i64 g0, i64 n, i64 g, const char* ax) {
    const bool lo_ok = r0 <= b0 - (S - 1) || g0 + r0 <= 1;
    const bool hi_ok = r1 >= b1 + (S - 1) || g0 + r1 >= l.N;
    W3D_REQUIRE(lo_ok && hi_ok, std::string("leapfrog_tb: stage-1 range does not cover the box halo in ") + ax);
    W3D_REQUIRE(g0 + b0 - S <= 0 || b0 - S >= -g, std::string("leapfrog_tb: halo deeper than the ghosts in ") + ax);
    W3D_REQUIRE(g0 + b1 + S - 1 >= l.N || b1 + S - 1 < n + g,
                std::string("leapfrog_tb: halo deeper than the ghosts in ") + ax);
    W3D_REQUIRE(r0 >= -g && r1 <= n + g, std::string("leapfrog_tb: real range outside the allocation in ") + ax);
  };
  axis_ok(b.x0, b.x1, real.x0, real.x1, l.gx0, l.nx, l.xg, "x");
  axis_ok(b.y0, b.y1, real.y0, real.y1, l.gy0, l.ny, l.yg, "y");
  axis_ok(b.z0, b.z1, real.z0, real.z1, l.gz0, l.nz, l.zg, "z");
  TbPlan pl;
  TbParams& p = pl.prm;
  p.plane = l.plane;
  p.pitch = l.pitch;
  p.zs = l.zs;
  p.x0 = static_cast<int>(b.x0);
  p.x1 = static_cast<int>(b.x1);
  p.xlen = static_cast<int>(imax(1, b.x1 - b.x0));
  p.nxc = 1;
  p.sx0 = static_cast<int>(real.x0);
  p.sx1 = static_cast<int>(real.x1);
  p.ax0 = static_cast<int>(-l.xg);
  p.ax1 = static_cast<int>(l.nx + l.xg);
  p.sy0 = static_cast<int>(real.y0);
  p.sy1 = static_cast<int>(real.y1);
  p.sz0 = static_cast<int>(real.z0);
  p.sz1 = static_cast<int>(real.z1);
  p.ay0 = static_cast<int>(-l.yg);
  p.ay1 = static_cast<int>(l.ny + l.yg);
  p.az0 = static_cast<int>(-l.zg);
  p.az1 = static_cast<int>(l.nz + l.zg);
  p.zero_off = static_cast<int>(l.zero_off());
  p.yg = static_cast<int>(l.yg);
  p.zg = static_cast<int>(l.zg);
  p.N = static_cast<int>(l.N);
  p.gx0 = static_cast<int>(l.gx0);
  p.gy0 = static_cast<int>(l.gy0);
  p.gz0 = static_cast<int>(l.gz0);
  p.y0 = static_cast<int>(b.y0);
  p.y1 = static_cast<int>(b.y1);
  p.z0 = static_cast<int>(b.z0);
  p.z1 = static_cast<int>(b.z1);
  if (b.x1 <= b.x0 || b.y1 <= b.y0 || b.z1 <= b.z0) return pl;
  p.nty = static_cast<int>(ceil_div(b.y1 - b.y0, kTile));
  p.ntz = static_cast<int>(ceil_div(b.z1 - b.z0, kTile));
  const int tiles = p.nty * p.ntz;
  // x chunks when the tile grid alone leaves CUs idle (3-D block boxes): at least min_chunk planes per chunk
  if (t.target_blocks > tiles) {
    const i64 nxb = b.x1 - b.x0;
    const i64 want = imin(ceil_div(t.target_blocks, tiles), imax(1, nxb / imax(1, t.min_chunk)));
    p.xlen = static_cast<int>(ceil_div(nxb, imax(1, want)));
    p.nxc = static_cast<int>(ceil_div(nxb, p.xlen));
  }
  const int blocks = tiles * p.nxc;
  pl.nblocks = t.xcd_remap ? static_cast<int>(round_up(blocks, 8)) : blocks;
  p.nblocks = pl.nblocks;
  p.xcd_remap = t.xcd_remap ? 1 : 0;
  p.xper = pl.nblocks / 8;
  // blocked XCD ownership when the tile grid splits into 8 equal blocks (one per XCD), the squarest such block
  p.bby = p.bbz = 0;
  if (t.xcd_remap && t.xcd_blocks && p.nxc == 1 && tiles == pl.nblocks && tiles % 8 == 0) {
    const int per = tiles / 8;
    int best = 1 << 30;
    for (int by = 1; by <= per; ++by) {
      if (per % by) continue;
      const int bz = per / by;
      if (p.nty % by || p.ntz % bz) continue;
      const int perim = by + bz;
      if (perim < best) {
        best = perim;
        p.bby = by;
        p.bbz = bz;
      }
    }
  }
  return pl;
}

template <int NT>
constexpr size_t max_dyn_lds() {
  return 160 * 1024 - 2 * (NT / 64) * sizeof(double) - 64;  // minus the static reduction arrays (+ alignment)
}

// allow the dynamic LDS size once per instantiation (outside any stream capture: see leapfrog_tb_prepare): the CU's
// 160 KiB minus the kernel's static LDS (the reduction arrays as the compiler laid them out, alignment included);
// returns that limit
template <int S, int NT, int CM, bool INIT, bool CH, bool PUSH>
size_t prepare_cfg() {
  static_assert(tb_lds_bytes<S, kTile, NT, INIT, (CM != 0 && !INIT)>() <= max_dyn_lds<NT>(),
                "leapfrog_tb tile does not fit in LDS");
  static const size_t limit = [] {
    const void* fn = reinterpret_cast<const void*>(k_leapfrog_tb<S, kTile, NT, CM, INIT, CH, PUSH>);
    hipFuncAttributes fa{};
    hipError_t e = hipFuncGetAttributes(&fa, fn);
    if (e != hipSuccess) fail(std::string("leapfrog_tb attributes: ") + hipGetErrorString(e));
    const size_t lim = 160 * 1024 - fa.sharedSizeBytes;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lim));
    if (e != hipSuccess) fail(std::string("leapfrog_tb LDS attribute: ") + hipGetErrorString(e));
    return lim;
  }();
  return limit;
}

template <int S, int NT, int CM, bool INIT, bool PUSH>
void launch_cfg(const TbParams& p, int nblocks, hipStream_t st) {
  const size_t shmem = tb_lds_bytes<S, kTile, NT, INIT, (CM != 0 && !INIT)>(
                           (p.check_mask || INIT) ? tb_nx_table<S>(p.xlen) : 0) +
                       (PUSH ? 8 * sizeof(unsigned long long) : 0) +  // (the push block: staging pointers)
                       sizeof(TbPack);                                 // (the fused-pack block)
  if (p.nxc > 1) {
    const size_t lim = prepare_cfg<S, NT, CM, INIT, true, PUSH>();
    W3D_REQUIRE(shmem <= lim, "leapfrog_tb: too many planes for the LDS sin table");
    hipLaunchKernelGGL((k_leapfrog_tb<S, kTile, NT, CM, INIT, true, PUSH>), dim3(nblocks), dim3(NT), shmem, st, p);
  } else {
    const size_t lim = prepare_cfg<S, NT, CM, INIT, false, PUSH>();
    W3D_REQUIRE(shmem <= lim, "leapfrog_tb: too many planes for the LDS sin table");
    hipLaunchKernelGGL((k_leapfrog_tb<S, kTile, NT, CM, INIT, false, PUSH>), dim3(nblocks), dim3(NT), shmem, st, p);
  }
}

// instantiated check supersets per S: none, even levels, odd levels, all (checks every 2nd step hit one parity)
template <int S>
constexpr int kFull = (1 << S) - 1;
template <int S>
constexpr int kEven = 0b1010 & kFull<S>;
template <int S>
constexpr int kOdd = 0b0101 & kFull<S>;

template <int S, int NT, bool INIT, bool PUSH>
void launch_nt(const TbParams& p, int nblocks, hipStream_t st) {
  const int m = p.check_mask;
  if (m == 0)
    launch_cfg<S, NT, 0, INIT, PUSH>(p, nblocks, st);
  else if ((m & ~kEven<S>) == 0)
    launch_cfg<S, NT, kEven<S>, INIT, PUSH>(p, nblocks, st);
  else if ((m & ~kOdd<S>) == 0)
    launch_cfg<S, NT, kOdd<S>, INIT, PUSH>(p, nblocks, st);
  else
    launch_cfg<S, NT, kFull<S>, INIT, PUSH>(p, nblocks, st);
}

// workgroup size per pass kind: LeapfrogTbTiling::threads, or init_threads for the analytic-start pass
template <int S, bool PUSH>
void launch_s(const TbParams& p, int nblocks, const LeapfrogTbTiling& t, bool init, hipStream_t st) {
  // 768 threads: 12 waves (3 per SIMD, 168 VGPRs each) for the 38² = 1444 stage-1 positions of an S = 4 tile, two sets
  // per thread with 6 % idle slots; 1024: 16 waves (128 VGPRs), 30 % of the second set idle
  if ((init ? t.init_threads : t.threads) == 768)
    init ? launch_nt<S, 768, true, PUSH>(p, nblocks, st) : launch_nt<S, 768, false, PUSH>(p, nblocks, st);
  else
    init ? launch_nt<S, 1024, true, PUSH>(p, nblocks, st) : launch_nt<S, 1024, false, PUSH>(p, nblocks, st);
}

template <int S, int NT, bool INIT, bool CH, bool PUSH>
void prepare_ch() {
  prepare_cfg<S, NT, 0, INIT, CH, PUSH>();
  prepare_cfg<S, NT, kEven<S>, INIT, CH, PUSH>();
  prepare_cfg<S, NT, kOdd<S>, INIT, CH, PUSH>();
  prepare_cfg<S, NT, kFull<S>, INIT, CH, PUSH>();
}
template <int S, int NT, bool INIT, bool PUSH = false>
void prepare_nt() {
  prepare_ch<S, NT, INIT, false, PUSH>();
  prepare_ch<S, NT, INIT, true, PUSH>();
}


// push transport instantiations (kernels_leapfrog_tb_push.hip): 1024-thread workgroups (analytic start: init_threads)
void launch_push(const TbParams& p, int nblocks, int stages, bool init, int init_threads, hipStream_t st);
void prepare_push();

}  // namespace tbk
}  // namespace wave3d
