// Temporally blocked leapfrog: two time steps per pass over HBM (gfx950). See wave3d/kernels.hpp.
//
// The single-step kernel moves 24 compulsory bytes per node-step (read u^n, u^{n−1}; write u^{n+1}) and already runs
// near the HBM streaming rate, so the remaining lever is to move fewer bytes: this kernel reads u^{n−1}, u^n and writes
// u^{n+1}, u^{n+2} — 32 bytes per node for two steps (16 B/node-step, 1.5× less traffic).
//
// Structure (register-queue waves, no LDS, no barriers — like k_leapfrog_rq):
//   * a wave owns R output rows × 62 output pairs (124 z nodes) and marches along x with a two-stage pipeline:
//     stage 1 computes u^{n+1} at plane x, stage 2 computes u^{n+2} at plane x−1 from the u^{n+1} planes x−2, x−1, x
//     that stage 1 left in registers;
//   * y: stage 1 also computes the rows just above and below the tile (redundantly, their owners compute them too),
//     so u^n is loaded for R+4 rows (the outer ones L2-served: they are the neighbouring waves' rows);
//   * z: the wave's 64 lanes hold pairs [first−1, first+63): lanes 0 and npe+1 are halo pairs whose inner node is
//     still a valid stage-1 result, which is exactly the z-neighbour stage 2 needs — no extra halo loads at all;
//   * x: each x-chunk recomputes the stage-1 planes just outside it (two planes per chunk);
//   * stage-1 values outside the interior are forced to 0: the Dirichlet boundary is structural here too.
// Because step-1 halo rows of one wave read u^{n−1} rows that another wave owns, nothing is written in place: the
// pass reads buffers (prev, cur) and writes (out1, out2); the solver rotates four buffers.
#include <hip/hip_runtime.h>

#include "wave3d/kernels.hpp"
#include "wave3d/stencil.hpp"

namespace wave3d {

namespace {

using v2d = double __attribute__((ext_vector_type(2)));
constexpr int kWaves = 4;       // waves per workgroup (independent)
constexpr int kOutPairs = 62;   // output pairs per wave (64 lanes minus a halo pair on each side)

__device__ __forceinline__ v2d ld2(const double* p) { return *reinterpret_cast<const v2d*>(p); }

template <bool NT>
__device__ __forceinline__ void st2(double* p, v2d v) {
  if (NT)
    __builtin_nontemporal_store(v, reinterpret_cast<v2d*>(p));
  else
    *reinterpret_cast<v2d*>(p) = v;
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

struct Lf2Params {
  const double* prev;  // u^{n−1}
  const double* cur;   // u^n
  double* out1;        // u^{n+1}
  double* out2;        // u^{n+2}
  const double* s;
  Partial* partials;
  i64 plane, pitch, ny, gx0, gy0, gz0, zs;
  i64 x0, x1, y0, y1, zo0, zo1;  // output box (local x, y; z as row offsets)
  i64 sx0, sx1;                  // x range where stage-1 values are real (beyond: Dirichlet 0)
  i64 pz0, pz_end;
  double ihx2, ihy2, ihz2, tau2, ct2;
  int ntz, nty, xchunk, ntiles, nblocks, xcd_remap;
};

// OCC > 1 asks the compiler for at least OCC waves per SIMD (fewer VGPRs, possibly some scratch spills)
template <int R, bool CHECK, bool NT, int OCC>
__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(OCC))) void k_leapfrog2_rq(
    const Lf2Params p) {
  constexpr int E = R + 4;  // extended rows: e ↔ y = yt − 2 + e
  const int lane = static_cast<int>(threadIdx.x) & 63;
  const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);  // wave-uniform: tile math stays scalar
  int blk = static_cast<int>(blockIdx.x);
  if (p.xcd_remap) {
    const int per = p.nblocks >> 3;
    blk = (static_cast<int>(blockIdx.x) & 7) * per + (static_cast<int>(blockIdx.x) >> 3);
  }
  const int tile = blk * kWaves + wv;
  const int pidx = static_cast<int>(blockIdx.x) * kWaves + wv;
  if (tile >= p.ntiles) {
    if (CHECK && lane == 0) p.partials[pidx] = make_double2(0.0, 0.0);
    return;
  }
  int t = tile;
  const int tz = t % p.ntz;
  t /= p.ntz;
  const int ty = t % p.nty;
  const int tx = t / p.nty;

  const i64 pzt = p.pz0 + static_cast<i64>(tz) * kOutPairs;  // first output pair
  const int npe = static_cast<int>(imin(kOutPairs, p.pz_end - pzt));
  const i64 yt = p.y0 + static_cast<i64>(ty) * R;
  const i64 xs = p.x0 + static_cast<i64>(tx) * p.xchunk;
  const i64 xe = imin(xs + p.xchunk, p.x1);

  const bool ld = lane <= npe + 1;
  const bool outl = lane >= 1 && lane <= npe;
  const i64 o0 = 2 * (pzt - 1 + lane);
  const bool in0 = o0 >= p.zo0 && o0 < p.zo1;
  const bool in1 = o0 + 1 >= p.zo0 && o0 + 1 < p.zo1;
  const bool ok0 = outl && in0, ok1 = outl && in1;
  const i64 pitch = p.pitch, plane = p.plane;

  // per extended row: wave-uniform row offset (scalar registers) + one 32-bit lane offset shared by every row, so
  // each load is a scalar base + vector offset (no 64-bit address per row in VGPRs); load validity; interior mask
  const int lo = static_cast<int>(o0);
  i64 rb[E];
  bool rl[E], ri[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const i64 y = yt - 2 + e;
    rb[e] = (y + 1) * pitch;
    rl[e] = ld && y >= -1 && y <= p.ny;
    ri[e] = y >= p.y0 && y < p.y1;
  }
  bool ro[R];
#pragma unroll
  for (int r = 0; r < R; ++r) ro[r] = yt + r < p.y1;

  const double* __restrict__ cur = p.cur;
  const double* __restrict__ prev = p.prev;
  const v2d z2 = {0.0, 0.0};
  // u^n queue for rows 1..E-2 (planes x−1, x, x+1); the two outer rows only need plane x
  v2d m[E], c[E], q[E], o[E];
  // u^{n+1}: w1 = plane x−1 (rows 1..E−2), w2 = plane x−2 (rows 2..E−3)
  v2d w1[E], w2[E];
  i64 px = xs * plane;  // plane base of x = xs − 1
#pragma unroll
  for (int e = 0; e < E; ++e) {
    m[e] = z2;
    c[e] = z2;
    q[e] = z2;
    o[e] = z2;
    w1[e] = z2;
    w2[e] = z2;
    if (rl[e]) {
      c[e] = ld2(cur + (px + rb[e]) + lo);
      if (e >= 1 && e <= E - 2) {
        m[e] = ld2(cur + (px - plane + rb[e]) + lo);
        q[e] = ld2(cur + (px + plane + rb[e]) + lo);
        o[e] = ld2(prev + (px + rb[e]) + lo);
      }
    }
  }
  const double tau2 = p.tau2;  // = τ²/h² (the coefficient of d2sum)
  double emax = 0.0, esum = 0.0;
  double sz0 = 0.0, sz1 = 0.0, sx = 0.0;
  double sy[R];
#pragma unroll
  for (int r = 0; r < R; ++r) sy[r] = CHECK && ro[r] ? p.s[p.gy0 + yt + r] : 0.0;
  if (CHECK && ld) {
    sz0 = p.s[p.gz0 + o0 - 1 - p.zs];
    sz1 = p.s[p.gz0 + o0 - p.zs];
  }

  for (i64 x = xs - 1; x <= xe; ++x, px += plane) {
    const bool more = x + 1 <= xe;
    // ---- prefetch for the next plane (consumed next iteration; vector-memory completion is in order)
    v2d nq[E], nc[E], no[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      nq[e] = z2;
      nc[e] = z2;
      no[e] = z2;
      if (more && rl[e]) {
        if (e >= 1 && e <= E - 2) {
          nq[e] = ld2(cur + (px + 2 * plane + rb[e]) + lo);
          no[e] = ld2(prev + (px + plane + rb[e]) + lo);
        } else {
          nc[e] = ld2(cur + (px + plane + rb[e]) + lo);
        }
      }
    }
    const double nsx = CHECK && more ? p.s[p.gx0 + x] : 0.0;  // φ factor of plane x (stage 2 next iteration)

    // ---- stage 1: u^{n+1} at plane x, rows 1..E−2
    const bool xin = x >= p.sx0 && x < p.sx1;
    const bool xout = x >= xs && x < xe;
    v2d a[E];
#pragma unroll
    for (int e = 0; e < E; ++e) a[e] = z2;
#pragma unroll
    for (int e = 1; e <= E - 2; ++e) {
      const v2d ym = c[e - 1], yp = c[e + 1];
      const double zm = __shfl_up(c[e].y, 1, 64);
      const double zp = __shfl_down(c[e].x, 1, 64);
      const double l0 = d2sum(c[e].x, m[e].x, q[e].x, ym.x, yp.x, zm, c[e].y);
      const double l1 = d2sum(c[e].y, m[e].y, q[e].y, ym.y, yp.y, c[e].x, zp);
      const bool keep = xin && ri[e];
      a[e].x = keep && in0 ? leapfrog(c[e].x, o[e].x, l0, tau2) : 0.0;
      a[e].y = keep && in1 ? leapfrog(c[e].y, o[e].y, l1, tau2) : 0.0;
      if (e >= 2 && e <= E - 3 && xout && ro[e - 2]) {
        double* dst = p.out1 + (px + rb[e]) + lo;
        if (ok0 && ok1)
          st2<NT>(dst, a[e]);
        else if (ok0)
          dst[0] = a[e].x;
        else if (ok1)
          dst[1] = a[e].y;
      }
    }
    // ---- stage 2: u^{n+2} at plane x−1, rows 2..E−3
    if (x > xs) {  // stage-2 plane x−1 inside the chunk
#pragma unroll
      for (int e = 2; e <= E - 3; ++e) {
        const int r = e - 2;
        const v2d ctr = w1[e];
        const double zm = __shfl_up(ctr.y, 1, 64);
        const double zp = __shfl_down(ctr.x, 1, 64);
        const double l0 = d2sum(ctr.x, w2[e].x, a[e].x, w1[e - 1].x, w1[e + 1].x, zm, ctr.y);
        const double l1 = d2sum(ctr.y, w2[e].y, a[e].y, w1[e - 1].y, w1[e + 1].y, ctr.x, zp);
        v2d v;
        v.x = leapfrog(ctr.x, m[e].x, l0, tau2);
        v.y = leapfrog(ctr.y, m[e].y, l1, tau2);
        if (ro[r]) {
          double* dst = p.out2 + (px - plane + rb[e]) + lo;
          if (ok0 && ok1)
            st2<NT>(dst, v);
          else if (ok0)
            dst[0] = v.x;
          else if (ok1)
            dst[1] = v.y;
          if (CHECK) {
            const double sxy = analytic_row(sx, sy[r], p.ct2);
            if (ok0) {
              const double er = fabs(v.x - sxy * sz0);
              emax = er > emax ? er : emax;
              esum = err_sq_acc(er, esum);
            }
            if (ok1) {
              const double er = fabs(v.y - sxy * sz1);
              emax = er > emax ? er : emax;
              esum = err_sq_acc(er, esum);
            }
          }
        }
      }
    }
    // ---- rotate
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (e >= 2 && e <= E - 3) w2[e] = w1[e];
      if (e >= 1 && e <= E - 2) {
        w1[e] = a[e];
        m[e] = c[e];
        c[e] = q[e];
        q[e] = nq[e];
        o[e] = no[e];
      } else {
        c[e] = nc[e];
      }
    }
    sx = nsx;
  }
  if (CHECK) {
    wave_reduce(emax, esum);
    if (lane == 0) p.partials[pidx] = make_double2(emax, esum);
  }
}

struct Plan2 {
  Lf2Params prm;
  int nblocks;
  int npartials;
};

Plan2 make_plan2(const Layout& l, const LBox& b, const Leapfrog2Tiling& t, i64 sx0, i64 sx1) {
  W3D_REQUIRE(t.rows == 1 || t.rows == 2 || t.rows == 4, "leapfrog2 rows per wave must be 1, 2 or 4");
  const LBox full = compute_box(l);
  // one x-slab of the whole y,z interior: a single rank, or a rank of a 1-D slab decomposition with 2-deep x halos
  W3D_REQUIRE(b.y0 == full.y0 && b.y1 == full.y1 && b.z0 == full.z0 && b.z1 == full.z1 && l.gy0 == 0 &&
                  l.gz0 == 0 && l.ny == l.N + 1 && l.nz == l.N + 1,
              "leapfrog2 needs whole (y,z) planes (single rank or 1-D slab decomposition)");
  W3D_REQUIRE(b.x0 >= full.x0 && b.x1 <= full.x1, "leapfrog2 box outside the updated region");
  // stage 1 runs on planes x0−1 .. x1 and reads u^n on x0−2 .. x1+1; a stage-1 plane outside [sx0, sx1) is taken as 0,
  // which is only right on the global Dirichlet boundary planes
  const bool lo_ok = b.x0 - 1 >= sx0 || l.gx0 + b.x0 - 1 == 0;
  const bool hi_ok = b.x1 < sx1 || l.gx0 + b.x1 == l.N;
  W3D_REQUIRE(sx0 <= b.x0 && sx1 >= b.x1 && b.x0 - 2 >= -l.xg && b.x1 + 1 <= l.nx + l.xg - 1 && lo_ok && hi_ok,
              "leapfrog2 stage-1 halo planes not available (needs 2 ghost planes towards neighbours)");
  Plan2 pl{};
  Lf2Params& p = pl.prm;
  p.plane = l.plane;
  p.pitch = l.pitch;
  p.ny = l.ny;
  p.gx0 = l.gx0;
  p.gy0 = l.gy0;
  p.gz0 = l.gz0;
  p.zs = l.zs;
  p.x0 = b.x0;
  p.x1 = b.x1;
  p.y0 = b.y0;
  p.y1 = b.y1;
  p.zo0 = b.z0 + 1 + l.zs;
  p.zo1 = b.z1 + 1 + l.zs;
  p.sx0 = sx0;
  p.sx1 = sx1;
  p.pz0 = p.zo0 / 2;
  p.pz_end = (p.zo1 + 1) / 2;
  W3D_REQUIRE(p.pz0 >= 1 && 2 * p.pz_end + 2 <= l.pitch, "row layout too tight for the leapfrog2 halo lanes");
  p.ntz = static_cast<int>(ceil_div(p.pz_end - p.pz0, kOutPairs));
  p.nty = static_cast<int>(ceil_div(b.y1 - b.y0, t.rows));
  const i64 base = static_cast<i64>(p.ntz) * p.nty;
  const i64 target = t.target_waves > 0 ? t.target_waves : 256 * 8 * 4;
  const i64 nxb = b.x1 - b.x0;
  i64 chunk = imax(16, ceil_div(nxb, imax(1, ceil_div(target, base))));
  chunk = imin(chunk, nxb);
  p.xchunk = static_cast<int>(chunk);
  const i64 tiles = base * ceil_div(nxb, chunk);
  W3D_REQUIRE(tiles < (1ll << 30), "too many tiles");
  p.ntiles = static_cast<int>(tiles);
  const int units = static_cast<int>(ceil_div(tiles, kWaves));
  pl.nblocks = t.xcd_remap ? static_cast<int>(round_up(units, 8)) : units;
  p.nblocks = pl.nblocks;
  p.xcd_remap = t.xcd_remap ? 1 : 0;
  pl.npartials = pl.nblocks * kWaves;
  return pl;
}

template <int R, int OCC>
void launch_ro(const Lf2Params& p, int nblocks, bool check, bool nt, hipStream_t st) {
  const dim3 block(64 * kWaves), grid(nblocks);
  if (check) {
    if (nt)
      hipLaunchKernelGGL((k_leapfrog2_rq<R, true, true, OCC>), grid, block, 0, st, p);
    else
      hipLaunchKernelGGL((k_leapfrog2_rq<R, true, false, OCC>), grid, block, 0, st, p);
  } else {
    if (nt)
      hipLaunchKernelGGL((k_leapfrog2_rq<R, false, true, OCC>), grid, block, 0, st, p);
    else
      hipLaunchKernelGGL((k_leapfrog2_rq<R, false, false, OCC>), grid, block, 0, st, p);
  }
}

}  // namespace

int leapfrog2_partials(const Layout& l, const LBox& box, const Leapfrog2Tiling& t) {
  return make_plan2(l, box, t, box.x0 - 1, box.x1 + 1).npartials;
}

void launch_leapfrog2(const Layout& l, const Coeffs& c, const double* prev, const double* cur, double* out1,
                      double* out2, const LBox& box, const double* d_s, double ct2, Partial* partials,
                      const Leapfrog2Tiling& t, hipStream_t stream, i64 sx0, i64 sx1) {
  W3D_REQUIRE(prev != out1 && prev != out2 && cur != out1 && cur != out2 && out1 != out2,
              "leapfrog2 needs four distinct buffers");
  if (sx0 > sx1) {  // default: stage 1 real exactly on the updated region of this rank
    const LBox full = compute_box(l);
    sx0 = full.x0;
    sx1 = full.x1;
  }
  Plan2 pl = make_plan2(l, box, t, sx0, sx1);
  if (pl.nblocks == 0) return;
  Lf2Params& p = pl.prm;
  const i64 kb = l.kbase();
  p.prev = prev + kb;
  p.cur = cur + kb;
  p.out1 = out1 + kb;
  p.out2 = out2 + kb;
  p.s = d_s;
  p.partials = partials;
  p.ihx2 = c.ihx2;
  p.ihy2 = c.ihy2;
  p.ihz2 = c.ihz2;
  p.tau2 = c.lam;  // τ²/h², the coefficient of d2sum
  p.ct2 = ct2;
  const bool check = partials != nullptr;
  switch (t.rows) {
    case 1: launch_ro<1, 1>(p, pl.nblocks, check, t.nt_store, stream); break;
    case 2:
      if (t.occupancy >= 3)
        launch_ro<2, 3>(p, pl.nblocks, check, t.nt_store, stream);
      else
        launch_ro<2, 1>(p, pl.nblocks, check, t.nt_store, stream);
      break;
    default: launch_ro<4, 1>(p, pl.nblocks, check, t.nt_store, stream); break;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) fail(std::string("leapfrog2 launch: ") + hipGetErrorString(e));
}

}  // namespace wave3d
