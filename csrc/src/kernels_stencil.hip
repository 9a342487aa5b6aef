// Hand-written CDNA4 (gfx950) stencil kernels for the 3D wave equation. See wave3d/kernels.hpp for the interface.
//
// Design (MI355X-first, not a translation of the reference's inferred one-thread-per-node CUDA kernels,
// SURVEY.md §2.5 K1-K5):
//   * fp64 nodes move in 16-byte PAIRS (global_load/store_dwordx4): one wave covers 128 consecutive z nodes.
//     The row layout (wave3d/decomp.hpp::Layout) shifts each row so the first updated node is pair-aligned.
//   * k_leapfrog is 2.5-D: a workgroup owns a (TY rows × 64 pairs) tile of the (y,z) plane and marches along x.
//     Its own column's u^n at x−1, x, x+1 lives in registers (a 3-deep queue, x+2 prefetched one plane ahead);
//     plane x with a 1-node halo is staged once through a double-buffered LDS tile, so one barrier per plane.
//     Each u^n / u^{n−1} value crosses HBM once per step (+2/xchunk for the x halo of a chunk, +halo rows from L2).
//   * u^{n+1} is written in place over u^{n−1}: 2 fields, 24 B/node/step of compulsory HBM traffic.
//   * Dirichlet BC is structural: boundary nodes are never written after init, so they stay 0.
//   * The error check vs the analytic solution is a template epilogue of the update: the new value is still in
//     registers, so a check step costs no extra HBM pass. Workgroup partials are reduced in a fixed order.
//   * Workgroups are remapped so each XCD (blockIdx % 8) gets a contiguous run of tiles: y-adjacent tiles that share
//     halo rows then share one L2.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "wave3d/kernels.hpp"
#include "wave3d/stencil.hpp"

namespace wave3d {

#define W3D_HIP_CHECK(expr)                                                                          \
  do {                                                                                               \
    hipError_t _e = (expr);                                                                          \
    if (_e != hipSuccess) ::wave3d::fail(std::string(#expr) + ": " + hipGetErrorString(_e));          \
  } while (0)

namespace {

using v2d = double __attribute__((ext_vector_type(2)));

constexpr int kLanes = 64;
constexpr int kMaxBoxes = 6;

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

// ---------------------------------------------------------------------------------------------------------------
// init + first step
// ---------------------------------------------------------------------------------------------------------------
struct InitParams {
  double* u0;
  double* u1;
  const double* s;
  i64 plane, N, nx, ny, nz, gx0, gy0, gz0, zs, xg, yg, zg;
  int pairs_per_row, pairs_per_plane;
  double ihx2, ihy2, ihz2, half_tau2;
};

__global__ __launch_bounds__(256) void k_init_first(const InitParams p) {
  const int q = static_cast<int>(blockIdx.x) * 256 + static_cast<int>(threadIdx.x);
  if (q >= p.pairs_per_plane) return;
  const i64 ix = static_cast<i64>(blockIdx.y) - p.xg;
  const int r = q / p.pairs_per_row;
  const int c = q - r * p.pairs_per_row;
  const i64 iy = r - p.yg;
  const i64 gx = p.gx0 + ix, gy = p.gy0 + iy;
  const double* s = p.s;
  const bool xy_in = gx > 0 && gx < p.N && gy > 0 && gy < p.N;
  const bool xy_ok = iy < p.ny + p.yg;  // (r < ny + 2·yg always holds)
  double a0[2], a1[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const i64 iz = 2 * static_cast<i64>(c) + e - p.zg - p.zs;
    double v = 0.0, w = 0.0;
    const i64 gz = p.gz0 + iz;
    // nodes beyond the global boundary stay 0 (as on the CPU path; the sin table only spans global −1..N+1)
    if (xy_ok && iz >= -p.zg && iz < p.nz + p.zg && gx >= 0 && gx <= p.N && gy >= 0 && gy <= p.N && gz >= 0 &&
        gz <= p.N) {
      v = phi(s, gx, gy, gz);
      if (xy_in && gz > 0 && gz < p.N) {
        const double lap = d2sum(v, phi(s, gx - 1, gy, gz), phi(s, gx + 1, gy, gz), phi(s, gx, gy - 1, gz),
                                phi(s, gx, gy + 1, gz), phi(s, gx, gy, gz - 1), phi(s, gx, gy, gz + 1));
        w = first_step(v, lap, p.half_tau2);
      }
    }
    a0[e] = v;
    a1[e] = w;
  }
  const i64 o = static_cast<i64>(blockIdx.y) * p.plane + 2 * static_cast<i64>(q);
  v2d w0, w1;
  w0.x = a0[0];
  w0.y = a0[1];
  w1.x = a1[0];
  w1.y = a1[1];
  st2<false>(p.u0 + o, w0);
  st2<false>(p.u1 + o, w1);
}

// ---------------------------------------------------------------------------------------------------------------
// leapfrog
// ---------------------------------------------------------------------------------------------------------------
struct TileBox {
  i64 x0, x1;    // local x range
  i64 y0, y1;    // local y range
  i64 zo0, zo1;  // row-offset range of the updated nodes
  i64 pz0, pz_end;
  int ntz, nty, xchunk, tile_begin;
};

struct LfParams {
  const double* cur;
  double* out;
  const double* s;
  Partial* partials;
  i64 plane, pitch, gx0, gy0, gz0, zs;
  double ihx2, ihy2, ihz2, tau2, ct;
  int nbox, ntiles, nblocks, xcd_remap;
  TileBox box[kMaxBoxes];
};

template <int TY, bool CHECK, bool NT>
__global__ __launch_bounds__(kLanes* TY) void k_leapfrog_lds(const LfParams p) {
  static_assert(TY >= 4, "halo slots need at least 128 + 2*TY threads");
  __shared__ v2d lds[2][TY + 2][kLanes + 2];
  __shared__ double red_m[TY], red_s[TY];

  const int lane = static_cast<int>(threadIdx.x);
  const int row = static_cast<int>(threadIdx.y);
  const int tid = row * kLanes + lane;

  int tile = static_cast<int>(blockIdx.x);
  if (p.xcd_remap) {
    const int per = p.nblocks >> 3;
    tile = (static_cast<int>(blockIdx.x) & 7) * per + (static_cast<int>(blockIdx.x) >> 3);
  }
  if (tile >= p.ntiles) {
    if (CHECK && tid == 0) p.partials[blockIdx.x] = make_double2(0.0, 0.0);
    return;
  }
  // select the box (scalar selects, no dynamic indexing of the kernarg struct)
  TileBox B = p.box[0];
#pragma unroll
  for (int k = 1; k < kMaxBoxes; ++k)
    if (k < p.nbox && tile >= p.box[k].tile_begin) B = p.box[k];

  int t = tile - B.tile_begin;
  const int tz = t % B.ntz;
  t /= B.ntz;
  const int ty = t % B.nty;
  const int tx = t / B.nty;

  const i64 pzt = B.pz0 + static_cast<i64>(tz) * kLanes;
  const int npe = static_cast<int>(imin(kLanes, B.pz_end - pzt));
  const i64 yt = B.y0 + static_cast<i64>(ty) * TY;
  const int nre = static_cast<int>(imin(TY, B.y1 - yt));
  const i64 xs = B.x0 + static_cast<i64>(tx) * B.xchunk;
  const i64 xe = imin(xs + B.xchunk, B.x1);

  const bool active = row < nre && lane < npe;
  const i64 y = yt + row;
  const i64 o0 = 2 * (pzt + lane);
  const bool ok0 = active && o0 >= B.zo0 && o0 < B.zo1;
  const bool ok1 = active && o0 + 1 >= B.zo0 && o0 + 1 < B.zo1;
  const i64 pitch = p.pitch, plane = p.plane;
  const i64 my = (y + 1) * pitch + o0;

  // halo slot of this thread: top row, bottom row, left pair, right pair
  int hr = -1, hc = 0;
  i64 hoff = 0;
  if (tid < kLanes) {
    if (tid < npe) { hr = 0; hc = tid + 1; hoff = yt * pitch + 2 * (pzt + tid); }
  } else if (tid < 2 * kLanes) {
    const int l = tid - kLanes;
    if (l < npe) { hr = nre + 1; hc = l + 1; hoff = (yt + nre + 1) * pitch + 2 * (pzt + l); }
  } else if (tid < 2 * kLanes + TY) {
    const int r = tid - 2 * kLanes;
    if (r < nre) { hr = r + 1; hc = 0; hoff = (yt + r + 1) * pitch + 2 * (pzt - 1); }
  } else if (tid < 2 * kLanes + 2 * TY) {
    const int r = tid - 2 * kLanes - TY;
    if (r < nre) { hr = r + 1; hc = npe + 1; hoff = (yt + r + 1) * pitch + 2 * (pzt + npe); }
  }

  const double* __restrict__ cur = p.cur;
  double* __restrict__ out = p.out;
  const v2d zero2 = {0.0, 0.0};
  v2d um = zero2, uc = zero2, up = zero2, uo = zero2, hv = zero2;
  i64 px = (xs + 1) * plane;  // plane base of x
  if (active) {
    um = ld2(cur + px - plane + my);
    uc = ld2(cur + px + my);
    up = ld2(cur + px + plane + my);
    uo = ld2(out + px + my);
  }
  if (hr >= 0) hv = ld2(cur + px + hoff);

  const double tau2 = p.tau2;  // = τ²/h² (the coefficient of d2sum)
  double emax = 0.0, esum = 0.0;
  double sxy = 0.0, sz0 = 0.0, sz1 = 0.0, sxp = CHECK ? p.s[p.gx0 + xs] : 0.0;
  if (CHECK && active) {
    sxy = p.s[p.gy0 + y];
    sz0 = p.s[p.gz0 + o0 - 1 - p.zs];
    sz1 = p.s[p.gz0 + o0 - p.zs];
  }

  for (i64 x = xs; x < xe; ++x, px += plane) {
    const int buf = static_cast<int>((x - xs) & 1);
    const bool more = x + 1 < xe;
    v2d nxt = zero2, uo_n = zero2, hv_n = zero2;
    const double nsxp = CHECK && more ? p.s[p.gx0 + x + 1] : 0.0;  // one plane ahead (in-order vmcnt)
    if (more) {
      if (active) {
        nxt = ld2(cur + px + 2 * plane + my);
        uo_n = ld2(out + px + plane + my);
      }
      if (hr >= 0) hv_n = ld2(cur + px + plane + hoff);
    }
    if (active) lds[buf][row + 1][lane + 1] = uc;
    if (hr >= 0) lds[buf][hr][hc] = hv;
    __syncthreads();
    if (active) {
      const v2d ym = lds[buf][row][lane + 1];
      const v2d yp = lds[buf][row + 2][lane + 1];
      const double zm = lds[buf][row + 1][lane].y;
      const double zp = lds[buf][row + 1][lane + 2].x;
      const double l0 = d2sum(uc.x, um.x, up.x, ym.x, yp.x, zm, uc.y);
      const double l1 = d2sum(uc.y, um.y, up.y, ym.y, yp.y, uc.x, zp);
      v2d r;
      r.x = leapfrog(uc.x, uo.x, l0, tau2);
      r.y = leapfrog(uc.y, uo.y, l1, tau2);
      double* dst = out + px + my;
      if (ok0 && ok1)
        st2<NT>(dst, r);
      else if (ok0)
        dst[0] = r.x;
      else if (ok1)
        dst[1] = r.y;
      if (CHECK) {
        const double sx = analytic_row(sxp, sxy, p.ct);
        if (ok0) {
          const double e = fabs(r.x - sx * sz0);
          emax = e > emax ? e : emax;
          esum = err_sq_acc(e, esum);
        }
        if (ok1) {
          const double e = fabs(r.y - sx * sz1);
          emax = e > emax ? e : emax;
          esum = err_sq_acc(e, esum);
        }
      }
    }
    um = uc;
    uc = up;
    up = nxt;
    uo = uo_n;
    hv = hv_n;
    sxp = nsxp;
  }

  if (CHECK) {
    wave_reduce(emax, esum);
    if (lane == 0) {
      red_m[row] = emax;
      red_s[row] = esum;
    }
    __syncthreads();
    if (tid == 0) {
      double m = red_m[0], s = red_s[0];
      for (int r = 1; r < TY; ++r) {
        m = red_m[r] > m ? red_m[r] : m;
        s += red_s[r];
      }
      p.partials[blockIdx.x] = make_double2(m, s);
    }
  }
}


// ---------------------------------------------------------------------------------------------------------------
// leapfrog, variant 1: register-queue waves (no LDS, no barriers)
// ---------------------------------------------------------------------------------------------------------------
// Each WAVE independently owns R rows × 64 pairs (128 z nodes) of the (y,z) plane and marches along x. All of u^n it
// needs lives in registers: for each row the x−1 / x / x+1 queue (+ x+2 in flight), the rows above/below the tile
// (two extra row loads per plane, L2-served: they are the neighbouring waves' own rows), and per row one 8-byte z-halo
// node that lanes 0 and npe−1 fetch. z-neighbours inside the row come from the adjacent lanes (__shfl_up/_down), y-
// neighbours from the adjacent rows' registers. Nothing is staged through LDS and waves never wait for each other, so
// many independent HBM streams stay in flight (R rows × 2 fields × 1 KiB per wave per plane).
constexpr int kWavesRq = 4;  // waves per workgroup (scheduling only; they do not cooperate)

template <int R, bool CHECK, bool NT>
__global__ __launch_bounds__(64 * kWavesRq) __attribute__((amdgpu_waves_per_eu(R <= 2 ? 4 : 2))) void k_leapfrog_rq(
    const LfParams p) {
  const int lane = static_cast<int>(threadIdx.x) & 63;
  const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);  // wave-uniform: tile math stays scalar
  int blk = static_cast<int>(blockIdx.x);
  if (p.xcd_remap) {
    const int per = p.nblocks >> 3;
    blk = (static_cast<int>(blockIdx.x) & 7) * per + (static_cast<int>(blockIdx.x) >> 3);
  }
  const int tile = blk * kWavesRq + wv;
  const int pidx = static_cast<int>(blockIdx.x) * kWavesRq + wv;
  if (tile >= p.ntiles) {
    if (CHECK && lane == 0) p.partials[pidx] = make_double2(0.0, 0.0);
    return;
  }
  TileBox B = p.box[0];
#pragma unroll
  for (int k = 1; k < kMaxBoxes; ++k)
    if (k < p.nbox && tile >= p.box[k].tile_begin) B = p.box[k];
  int t = tile - B.tile_begin;
  const int tz = t % B.ntz;
  t /= B.ntz;
  const int ty = t % B.nty;
  const int tx = t / B.nty;

  const i64 pzt = B.pz0 + static_cast<i64>(tz) * kLanes;
  const int npe = static_cast<int>(imin(kLanes, B.pz_end - pzt));
  const i64 yt = B.y0 + static_cast<i64>(ty) * R;
  const int nre = static_cast<int>(imin(R, B.y1 - yt));
  const i64 xs = B.x0 + static_cast<i64>(tx) * B.xchunk;
  const i64 xe = imin(xs + B.xchunk, B.x1);

  const bool act = lane < npe;
  const i64 o0 = 2 * (pzt + lane);
  const bool ok0 = act && o0 >= B.zo0 && o0 < B.zo1;
  const bool ok1 = act && o0 + 1 >= B.zo0 && o0 + 1 < B.zo1;
  const i64 pitch = p.pitch, plane = p.plane;
  const i64 base = (yt + 1) * pitch + o0;   // row yt (r = 0), element 0 of my pair
  const i64 top = base - pitch;              // row yt − 1
  const i64 bot = base + nre * pitch;        // row yt + nre
  // z halo: lane 0 fetches node 2·pzt − 1 (left of the tile); the right neighbour 2·(pzt+npe) is fetched by lane
  // npe − 1, or by lane 1 when the tile is a single pair (lane 0 then reads it with a shuffle)
  const int rlane = npe == 1 ? 1 : npe - 1;
  const bool hzl = lane == 0, hzr = lane == rlane;
  const i64 hzoff = (yt + 1) * pitch + (hzl ? 2 * pzt - 1 : 2 * (pzt + npe));

  const double* __restrict__ cur = p.cur;
  double* __restrict__ out = p.out;
  const v2d z2 = {0.0, 0.0};
  v2d m[R], c[R], q[R], o[R];
  double hz[R];
  v2d ht = z2, hb = z2;
  i64 px = (xs + 1) * plane;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    m[r] = z2;
    c[r] = z2;
    q[r] = z2;
    o[r] = z2;
    hz[r] = 0.0;
    if (r < nre) {
      if (act) {
        m[r] = ld2(cur + px - plane + base + r * pitch);
        c[r] = ld2(cur + px + base + r * pitch);
        q[r] = ld2(cur + px + plane + base + r * pitch);
        o[r] = ld2(out + px + base + r * pitch);
      }
      if (hzl || hzr) hz[r] = cur[px + hzoff + r * pitch];
    }
  }
  if (act) {
    ht = ld2(cur + px + top);
    hb = ld2(cur + px + bot);
  }
  const double tau2 = p.tau2;  // = τ²/h² (the coefficient of d2sum)
  double emax = 0.0, esum = 0.0;
  // error-epilogue factors of φ are loaded up front / one plane ahead, like every other load: vector-memory
  // completion is in order, so a load consumed in the same iteration would drain the whole prefetch queue
  double sz0 = 0.0, sz1 = 0.0, sx = 0.0;
  double sy[R];
#pragma unroll
  for (int r = 0; r < R; ++r) sy[r] = CHECK && r < nre ? p.s[p.gy0 + yt + r] : 0.0;
  if (CHECK) {
    if (act) {
      sz0 = p.s[p.gz0 + o0 - 1 - p.zs];
      sz1 = p.s[p.gz0 + o0 - p.zs];
    }
    sx = p.s[p.gx0 + xs];
  }

  for (i64 x = xs; x < xe; ++x, px += plane) {
    const bool more = x + 1 < xe;
    v2d nq[R], no[R];
    double nhz[R];
    v2d nht = z2, nhb = z2;
    const double nsx = CHECK && more ? p.s[p.gx0 + x + 1] : 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      nq[r] = z2;
      no[r] = z2;
      nhz[r] = 0.0;
      if (more && r < nre) {
        if (act) {
          nq[r] = ld2(cur + px + 2 * plane + base + r * pitch);
          no[r] = ld2(out + px + plane + base + r * pitch);
        }
        if (hzl || hzr) nhz[r] = cur[px + plane + hzoff + r * pitch];
      }
    }
    if (more && act) {
      nht = ld2(cur + px + plane + top);
      nhb = ld2(cur + px + plane + bot);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r < nre) {
        const v2d ym = r == 0 ? ht : c[r - 1];
        const v2d yp = (r + 1 < nre && r + 1 < R) ? c[r + 1 < R ? r + 1 : r] : hb;
        const double up_y = __shfl_up(c[r].y, 1, 64);
        const double dn_x = __shfl_down(c[r].x, 1, 64);
        const double hzs = npe == 1 ? __shfl_down(hz[r], 1, 64) : hz[r];
        const double zm = lane == 0 ? hz[r] : up_y;
        const double zp = lane == npe - 1 ? hzs : dn_x;
        const double l0 = d2sum(c[r].x, m[r].x, q[r].x, ym.x, yp.x, zm, c[r].y);
        const double l1 = d2sum(c[r].y, m[r].y, q[r].y, ym.y, yp.y, c[r].x, zp);
        v2d v;
        v.x = leapfrog(c[r].x, o[r].x, l0, tau2);
        v.y = leapfrog(c[r].y, o[r].y, l1, tau2);
        double* dst = out + px + base + r * pitch;
        if (ok0 && ok1)
          st2<NT>(dst, v);
        else if (ok0)
          dst[0] = v.x;
        else if (ok1)
          dst[1] = v.y;
        if (CHECK) {
          const double sxy = analytic_row(sx, sy[r], p.ct);
          if (ok0) {
            const double e = fabs(v.x - sxy * sz0);
            emax = e > emax ? e : emax;
            esum = err_sq_acc(e, esum);
          }
          if (ok1) {
            const double e = fabs(v.y - sxy * sz1);
            emax = e > emax ? e : emax;
            esum = err_sq_acc(e, esum);
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      m[r] = c[r];
      c[r] = q[r];
      q[r] = nq[r];
      o[r] = no[r];
      hz[r] = nhz[r];
    }
    ht = nht;
    hb = nhb;
    sx = nsx;
  }
  if (CHECK) {
    wave_reduce(emax, esum);
    if (lane == 0) p.partials[pidx] = make_double2(emax, esum);
  }
}

template <int R>
void launch_rq(const LfParams& p, int nblocks, bool check, bool nt, hipStream_t st);

// Host-side tiling plan shared by leapfrog_blocks() and launch_leapfrog().
struct Plan {
  LfParams prm;
  int nblocks;    // workgroups launched
  int npartials;  // error partials written (v0: per workgroup, v1: per wave)
};

Plan make_plan(const Layout& l, const LBox* boxes, int nbox, const LeapfrogTiling& t) {
  W3D_REQUIRE(nbox >= 0 && nbox <= kMaxBoxes, "too many boxes in one leapfrog launch");
  const bool rq = t.variant == 1;
  W3D_REQUIRE(t.variant == 0 || t.variant == 1, "leapfrog variant must be 0 (lds) or 1 (rq)");
  W3D_REQUIRE(rq || t.ty == 4 || t.ty == 8 || t.ty == 16, "leapfrog tile rows must be 4, 8 or 16");
  W3D_REQUIRE(!rq || t.rows == 1 || t.rows == 2 || t.rows == 4 || t.rows == 8, "rows per wave must be 1, 2, 4 or 8");
  const int trows = rq ? t.rows : t.ty;
  Plan pl{};
  LfParams& p = pl.prm;
  p.plane = l.plane;
  p.pitch = l.pitch;
  p.gx0 = l.gx0;
  p.gy0 = l.gy0;
  p.gz0 = l.gz0;
  p.zs = l.zs;
  // v0: one tile per workgroup, aim for 8 workgroups per CU; v1: one tile per wave, aim for 16 waves per CU
  const int target = t.target_blocks > 0 ? t.target_blocks : (rq ? 256 * 16 : 256 * 8);
  // tiles before x-chunking, to spread the x-chunk count over boxes
  i64 base_total = 0;
  for (int b = 0; b < nbox; ++b) {
    const LBox& x = boxes[b];
    if (x.empty()) continue;
    const i64 zo0 = x.z0 + 1 + l.zs, zo1 = x.z1 + 1 + l.zs;
    base_total += ceil_div((zo1 + 1) / 2 - zo0 / 2, kLanes) * ceil_div(x.y1 - x.y0, trows);
  }
  const i64 want = base_total > 0 ? imax(1, ceil_div(target, base_total)) : 1;
  int nb = 0, tiles = 0;
  for (int b = 0; b < nbox; ++b) {
    const LBox& x = boxes[b];
    if (x.empty()) continue;
    W3D_REQUIRE(x.x0 >= 0 && x.x1 <= l.nx && x.y0 >= 0 && x.y1 <= l.ny && x.z0 >= 0 && x.z1 <= l.nz,
                "leapfrog box outside the owned region");
    TileBox& tb = p.box[nb];
    tb.x0 = x.x0;
    tb.x1 = x.x1;
    tb.y0 = x.y0;
    tb.y1 = x.y1;
    tb.zo0 = x.z0 + 1 + l.zs;
    tb.zo1 = x.z1 + 1 + l.zs;
    tb.pz0 = tb.zo0 / 2;
    tb.pz_end = (tb.zo1 + 1) / 2;
    W3D_REQUIRE(2 * tb.pz_end + 2 <= l.pitch, "row pitch too small for the pair tiling");
    tb.ntz = static_cast<int>(ceil_div(tb.pz_end - tb.pz0, kLanes));
    tb.nty = static_cast<int>(ceil_div(x.y1 - x.y0, trows));
    const i64 nxb = x.x1 - x.x0;
    const i64 min_chunk = 16;
    i64 chunk = imax(min_chunk, ceil_div(nxb, want));
    chunk = imin(chunk, nxb);
    tb.xchunk = static_cast<int>(chunk);
    const i64 nxc = ceil_div(nxb, chunk);
    tb.tile_begin = tiles;
    const i64 bt = static_cast<i64>(tb.ntz) * tb.nty * nxc;
    W3D_REQUIRE(tiles + bt < (1ll << 30), "too many tiles");
    tiles += static_cast<int>(bt);
    ++nb;
  }
  p.nbox = nb;
  p.ntiles = tiles;
  p.xcd_remap = t.xcd_remap ? 1 : 0;
  const int units = rq ? static_cast<int>(ceil_div(tiles, kWavesRq)) : tiles;  // workgroups
  pl.nblocks = t.xcd_remap ? static_cast<int>(round_up(units, 8)) : units;
  p.nblocks = pl.nblocks;
  pl.npartials = rq ? pl.nblocks * kWavesRq : pl.nblocks;
  return pl;
}

template <int TY>
void launch_lf_ty(const LfParams& p, int nblocks, bool check, bool nt, hipStream_t st) {
  const dim3 block(kLanes, TY), grid(nblocks);
  if (check) {
    if (nt)
      hipLaunchKernelGGL((k_leapfrog_lds<TY, true, true>), grid, block, 0, st, p);
    else
      hipLaunchKernelGGL((k_leapfrog_lds<TY, true, false>), grid, block, 0, st, p);
  } else {
    if (nt)
      hipLaunchKernelGGL((k_leapfrog_lds<TY, false, true>), grid, block, 0, st, p);
    else
      hipLaunchKernelGGL((k_leapfrog_lds<TY, false, false>), grid, block, 0, st, p);
  }
}

template <int R>
void launch_rq(const LfParams& p, int nblocks, bool check, bool nt, hipStream_t st) {
  const dim3 block(64 * kWavesRq), grid(nblocks);
  if (check) {
    if (nt)
      hipLaunchKernelGGL((k_leapfrog_rq<R, true, true>), grid, block, 0, st, p);
    else
      hipLaunchKernelGGL((k_leapfrog_rq<R, true, false>), grid, block, 0, st, p);
  } else {
    if (nt)
      hipLaunchKernelGGL((k_leapfrog_rq<R, false, true>), grid, block, 0, st, p);
    else
      hipLaunchKernelGGL((k_leapfrog_rq<R, false, false>), grid, block, 0, st, p);
  }
}

// ---------------------------------------------------------------------------------------------------------------
// standalone error check (step 1 and diagnostics)
// ---------------------------------------------------------------------------------------------------------------
struct ErrParams {
  const double* u;
  const double* s;
  Partial* partials;
  i64 plane, pitch, gx0, gy0, gz0, zs;
  i64 x0, y0, z0, ny, nz;  // box origin and extents (y,z)
  double ct;
};

__global__ __launch_bounds__(256) void k_error(const ErrParams p) {
  __shared__ double red_m[4], red_s[4];
  const i64 x = p.x0 + blockIdx.y;
  const i64 q = static_cast<i64>(blockIdx.x) * 256 + threadIdx.x;
  double emax = 0.0, esum = 0.0;
  if (q < p.ny * p.nz) {
    const i64 y = p.y0 + q / p.nz, z = p.z0 + q % p.nz;
    const double v = p.u[(x + 1) * p.plane + (y + 1) * p.pitch + (z + 1 + p.zs)];
    const double e = fabs(v - analytic_row(p.s[p.gx0 + x], p.s[p.gy0 + y], p.ct) * p.s[p.gz0 + z]);
    emax = e;
    esum = err_sq_acc(e, 0.0);
  }
  wave_reduce(emax, esum);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red_m[w] = emax;
    red_s[w] = esum;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = red_m[0], s = red_s[0];
    for (int r = 1; r < 4; ++r) {
      m = red_m[r] > m ? red_m[r] : m;
      s += red_s[r];
    }
    p.partials[static_cast<i64>(blockIdx.y) * gridDim.x + blockIdx.x] = make_double2(m, s);
  }
}

// ---------------------------------------------------------------------------------------------------------------
// fixed-order reduction of partials
// ---------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ void reduce_block(const Partial* __restrict__ in, int n, Partial* out);

__global__ __launch_bounds__(1024) void k_reduce(const Partial* __restrict__ in, int n, Partial* out) {
  reduce_block(in, n, out);
}

constexpr int kReduceBatch = 64;  // jobs per launch (kernel-argument struct: 64 × 24 B)
struct ReduceBatch {
  ReduceJob job[kReduceBatch];
};

__global__ __launch_bounds__(1024) void k_reduce_batch(const ReduceBatch b) {
  const ReduceJob j = b.job[blockIdx.x];
  reduce_block(j.in, j.n, j.out);
}

__device__ __forceinline__ void reduce_block(const Partial* __restrict__ in, int n, Partial* out) {
  __shared__ double sm[16], ss[16];
  double m = 0.0, s = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) {
    const Partial v = in[i];
    m = v.x > m ? v.x : m;
    s += v.y;
  }
  wave_reduce(m, s);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sm[w] = m;
    ss[w] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double mm = sm[0], sss = ss[0];
    for (int r = 1; r < 16; ++r) {
      mm = sm[r] > mm ? sm[r] : mm;
      sss += ss[r];
    }
    out[0] = make_double2(mm, sss);
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------------------------------
namespace {
InitParams init_params(const Layout& l, const Coeffs& c, const double* d_s, double* a, double* b) {
  InitParams p;
  p.u0 = a;
  p.u1 = b;
  p.s = d_s;
  p.plane = l.plane;
  p.N = l.N;
  p.nx = l.nx;
  p.ny = l.ny;
  p.nz = l.nz;
  p.gx0 = l.gx0;
  p.gy0 = l.gy0;
  p.gz0 = l.gz0;
  p.zs = l.zs;
  p.xg = l.xg;
  p.yg = l.yg;
  p.zg = l.zg;
  W3D_REQUIRE(l.pitch % 2 == 0 && l.plane / 2 < (1ll << 31), "plane too large for the init kernel");
  W3D_REQUIRE(l.nx + 2 * l.xg <= 65535, "too many planes for the init kernel grid");
  p.pairs_per_row = static_cast<int>(l.pitch / 2);
  p.pairs_per_plane = static_cast<int>(l.plane / 2);
  p.ihx2 = c.ihx2;
  p.ihy2 = c.ihy2;
  p.ihz2 = c.ihz2;
  p.half_tau2 = c.half_lam;  // τ²/(2h²), the coefficient of d2sum
  return p;
}
}  // namespace

void launch_init_first(const Layout& l, const Coeffs& c, const double* d_s, double* u0, double* u1,
                       hipStream_t stream) {
  const InitParams p = init_params(l, c, d_s, u0, u1);
  const dim3 grid(static_cast<unsigned>(ceil_div(p.pairs_per_plane, 256)), static_cast<unsigned>(l.nx + 2 * l.xg));
  hipLaunchKernelGGL(k_init_first, grid, dim3(256), 0, stream, p);
  W3D_HIP_CHECK(hipGetLastError());
}

int leapfrog_blocks(const Layout& l, const LBox* boxes, int nbox, const LeapfrogTiling& t) {
  return make_plan(l, boxes, nbox, t).npartials;
}

void launch_leapfrog(const Layout& l, const Coeffs& c, const double* cur, double* old_out, const LBox* boxes, int nbox,
                     const double* d_s, double ct, Partial* partials, const LeapfrogTiling& t, hipStream_t stream) {
  Plan pl = make_plan(l, boxes, nbox, t);
  if (pl.nblocks == 0) return;
  LfParams& p = pl.prm;
  p.cur = cur + l.kbase();
  p.out = old_out + l.kbase();
  p.s = d_s;
  p.partials = partials;
  p.ihx2 = c.ihx2;
  p.ihy2 = c.ihy2;
  p.ihz2 = c.ihz2;
  p.tau2 = c.lam;  // τ²/h², the coefficient of d2sum
  p.ct = ct;
  const bool check = partials != nullptr;
  if (t.variant == 1) {
    switch (t.rows) {
      case 1: launch_rq<1>(p, pl.nblocks, check, t.nt_store, stream); break;
      case 2: launch_rq<2>(p, pl.nblocks, check, t.nt_store, stream); break;
      case 4: launch_rq<4>(p, pl.nblocks, check, t.nt_store, stream); break;
      default: launch_rq<8>(p, pl.nblocks, check, t.nt_store, stream); break;
    }
  } else {
    switch (t.ty) {
      case 4: launch_lf_ty<4>(p, pl.nblocks, check, t.nt_store, stream); break;
      case 8: launch_lf_ty<8>(p, pl.nblocks, check, t.nt_store, stream); break;
      default: launch_lf_ty<16>(p, pl.nblocks, check, t.nt_store, stream); break;
    }
  }
  W3D_HIP_CHECK(hipGetLastError());
}

int error_blocks(const Layout& /*l*/, const LBox& b) {
  if (b.empty()) return 0;
  return static_cast<int>(ceil_div((b.y1 - b.y0) * (b.z1 - b.z0), 256) * (b.x1 - b.x0));
}

void launch_error(const Layout& l, const double* u, const LBox& b, const double* d_s, double ct, Partial* partials,
                  hipStream_t stream) {
  if (b.empty()) return;
  ErrParams p;
  p.u = u + l.kbase();
  p.s = d_s;
  p.partials = partials;
  p.plane = l.plane;
  p.pitch = l.pitch;
  p.gx0 = l.gx0;
  p.gy0 = l.gy0;
  p.gz0 = l.gz0;
  p.zs = l.zs;
  p.x0 = b.x0;
  p.y0 = b.y0;
  p.z0 = b.z0;
  p.ny = b.y1 - b.y0;
  p.nz = b.z1 - b.z0;
  p.ct = ct;
  W3D_REQUIRE(b.x1 - b.x0 <= 65535, "too many planes for the error kernel grid");
  const dim3 grid(static_cast<unsigned>(ceil_div(p.ny * p.nz, 256)), static_cast<unsigned>(b.x1 - b.x0));
  hipLaunchKernelGGL(k_error, grid, dim3(256), 0, stream, p);
  W3D_HIP_CHECK(hipGetLastError());
}

void launch_reduce(const Partial* partials, int n, Partial* out, hipStream_t stream) {
  hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, stream, partials, n, out);
  W3D_HIP_CHECK(hipGetLastError());
}

void launch_reduce_batch(const ReduceJob* jobs, int njobs, hipStream_t stream) {
  for (int j0 = 0; j0 < njobs; j0 += kReduceBatch) {
    ReduceBatch b{};
    const int nb = njobs - j0 < kReduceBatch ? njobs - j0 : kReduceBatch;
    for (int j = 0; j < nb; ++j) b.job[j] = jobs[j0 + j];
    hipLaunchKernelGGL(k_reduce_batch, dim3(nb), dim3(1024), 0, stream, b);
    W3D_HIP_CHECK(hipGetLastError());
  }
}

}  // namespace wave3d
