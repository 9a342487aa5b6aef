// Deep temporal blocking: S (2..4) leapfrog steps per pass over HBM, intermediate levels on chip (gfx950).
// See wave3d/kernels.hpp.
//
// The two-step register-queue kernel (kernels_leapfrog2.hip) moves 16 B per node-step and already streams at the HBM
// rate of a half-write workload, so the remaining lever is more steps per pass. Design:
//   * a workgroup owns a 32 × 32 tile of the (y,z) plane (256 tiles at 512³: one per CU) and marches along x through
//     the whole box. Iteration i loads plane i+2 of u^n, and stage k = 1..S computes u^{n+k} at plane i−(k−1) — a
//     skewed wavefront over the shrinking regions "tile + (S−k) halo" (redundant halo work ≈ 1.2× at S = 4);
//   * every thread owns fixed (y,z) nodes of the stage-1 region in EVERY level, so the x neighbours and the "old"
//     level of a node are the thread's own earlier results: per level a 4-deep register queue of planes (the x loop
//     is unrolled by 4 so queue slots are static registers);
//   * only the four y/z neighbours go through LDS: one plane per level in two parity slots. Stage k reads the plane
//     of u^{n+k−1} that stage k−1 wrote in the PREVIOUS iteration, so one barrier per iteration suffices;
//   * u^n is prefetched two planes ahead (global → register queue; the halo ring of the tile → two ring registers),
//     u^{n−1} one plane ahead straight into registers (it is only ever the "old" level of the thread's own nodes);
//   * stages S−1 and S store the tile (u^{n+S−1}, u^{n+S}): 2 reads + 2 writes per node per pass = 32/S B/node-step;
//   * (y,z) positions outside the global interior, outside the rank's allocation, or (thread-owned positions) outside
//     the range where stage values are real, load the plane's zero slot instead (Layout::zero_off, a padding double
//     that only ever holds 0), so no select follows a load and its wait is deferred to the first use; such positions
//     only feed stage values that no owned output reads, forced to 0 like every stage output outside the real range;
//   * 3-D block ranks (S-deep ghosts on the split y/z axes too) pass their real y/z ranges like the x one; small
//     boxes split x into chunks (each workgroup marches one chunk, recomputing S−1 planes on each side) so that a
//     launch still fills the 256 CUs;
//   * any subset of the S new levels can carry the fused error check (per-stage partials); the check's s_x·s_y row
//     factor is tabulated once per plane (row_tables) and each position's s_z factor sits in a register;
//   * the analytic-start variant (INIT) reads nothing: a φ stage computes u⁰ = φ once per node and plane into an extra
//     LDS level and u¹ = first_step(φ, d2sum φ) from its neighbours (bit-identical to k_init_first).
// Formulas and operation order are those of stencil.hpp (d2sum with the folded coefficient λ = τ²/h²): one pass is
// bit-identical to S single steps. Measured variants that lost (dense 768-thread layouts, 3-deep queues, 5-step
// passes, deeper prefetch, half tiles, branch-free selects, a conflict-free position order) are documented with their
// numbers in profiles/r1_tb_queue_experiments.md. The pass
// semantics (which plane of which level each stage reads) are mirrored by tools/tb_emulate.py (CPU tests).
#include <algorithm>

#include "wave3d/leapfrog_tb_kernel.hpp"

namespace wave3d {

using namespace tbk;

namespace {
__global__ __launch_bounds__(64) void k_l2_flush() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, ""); }
}  // namespace

void l2_flush_all(hipStream_t stream) {
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) !=
      hipSuccess)
    fail("l2 flush: no device");
  hipLaunchKernelGGL(k_l2_flush, dim3(static_cast<unsigned>(8 * ncu)), dim3(64), 0, stream);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) fail(std::string("l2 flush launch: ") + hipGetErrorString(e));
}

void leapfrog_tb_prepare(bool push) {
  leapfrog_p2_prepare();
  if (push) prepare_push();
  prepare_nt<2, 768, false>();
  prepare_nt<3, 768, false>();
  prepare_nt<4, 768, false>();
  prepare_nt<2, 768, true>();
  prepare_nt<3, 768, true>();
  prepare_nt<4, 768, true>();
  prepare_nt<2, 1024, false>();
  prepare_nt<3, 1024, false>();
  prepare_nt<4, 1024, false>();
  prepare_nt<2, 1024, true>();
  prepare_nt<3, 1024, true>();
  prepare_nt<4, 1024, true>();
}

size_t leapfrog_tb_lds_bytes(int stages) {
  return stages == 2 ? tb_lds_bytes<2, kTile, 512>() : stages == 3 ? tb_lds_bytes<3, kTile, 512>()
                                                                   : tb_lds_bytes<4, kTile, 512>();
}

int leapfrog_tb_partials(const Layout& l, const LBox& box, const LeapfrogTbTiling& t) {
  // the block count depends on the (y,z) tiling and the x chunks only: the widest real ranges pass the halo checks
  const LBox real{-l.xg, l.nx + l.xg, -l.yg, l.ny + l.yg, -l.zg, l.nz + l.zg};
  LeapfrogTbTiling t1 = t;
  t1.stages = 2;  // (block count independent of S; S = 2 keeps the ghost-depth checks satisfiable)
  const int n = make_plan_tb(l, box, t1, real).nblocks;
  // (the pair-tiled pass may split x differently: a slot holds either kernel's partials)
  return t.p2 && leapfrog_p2_supported(l, box, 2) ? std::max(n, leapfrog_p2_partials(l, box, t)) : n;
}

void launch_leapfrog_tb(const Layout& l, const Coeffs& c, const double* prev, const double* cur, double* out1,
                        double* out2, const LBox& box, const double* d_s, const double* ct, int check_mask,
                        Partial* partials, const LeapfrogTbTiling& t, hipStream_t stream, const LBox& real,
                        bool analytic_start, int level_stride, int grid_blocks, const TbPush* push,
                        const TbPush* push_dev, const TbPack* pack, const TbPack* pack_dev) {
  W3D_REQUIRE(out1 != out2 && (analytic_start || (prev != out1 && prev != out2 && cur != out1 && cur != out2)),
              "leapfrog_tb needs four distinct buffers");
  if (t.p2 && (push == nullptr || !push->on) && pack == nullptr && leapfrog_p2_supported(l, box, t.stages) &&
      (!analytic_start || t.stages <= 4)) {
    launch_leapfrog_p2(l, c, prev, cur, out1, out2, box, d_s, ct, check_mask, partials, t, stream, real,
                       analytic_start, level_stride, grid_blocks);
    return;
  }
  W3D_REQUIRE(t.stages <= 4, "leapfrog_tb: 5-step passes need the pair-tiled kernel (tiling.p2)");
  W3D_REQUIRE(t.ghost_x1 == 0, "leapfrog_tb: ghost-plane stores (tiling.ghost_x1) need the pair-tiled kernel");
  TbPlan pl = make_plan_tb(l, box, t, real);
  if (pl.nblocks == 0) return;
  TbParams& p = pl.prm;
  if (push != nullptr && push->on) {
    // the staging holds T planes per side in this rank's plane geometry; the forwarded planes are this rank's own
    W3D_REQUIRE(push->T == l.xg && push->nx == l.nx && t.stages <= push->T && l.yg == 1 && l.zg == 1,
                "leapfrog_tb push: slab ranks with T-deep x ghosts only");
    W3D_REQUIRE(push->T >= 2 && l.nx >= push->T, "leapfrog_tb push: a rank needs at least T planes");
    W3D_REQUIRE(push_dev != nullptr, "leapfrog_tb push: the pass parameters must be in device memory");
    p.push = push_dev;
    p.pnx = push->nx;
    p.pT = push->T;
    p.ptag = push->tag;
    p.pacq = push->acquire;
  }
  if (pack != nullptr) {  // fused z-face pack: the host copy gives the band limits, the kernel reads the rest on use
    W3D_REQUIRE(pack_dev != nullptr && pack->w >= 2 && pack->w <= kTile && pack->ny == l.ny && pack->nz == l.nz,
                "leapfrog_tb pack: bad parameters");
    p.pk = pack_dev;
    p.pkza = pack->zf[0][0] ? pack->w : 0;
    p.pkzb = pack->zf[1][0] ? pack->nz - pack->w : pack->nz;
  }
  // a padded grid (several launches sharing one level's partial slots, each of grid_blocks entries): the extra
  // workgroups have no tile and write (0, 0) partials, so every slot entry a reduction reads is written
  if (grid_blocks > 0) {
    W3D_REQUIRE(grid_blocks >= pl.nblocks && (!t.xcd_remap || grid_blocks % 8 == 0), "leapfrog_tb: bad grid_blocks");
    pl.nblocks = p.nblocks = grid_blocks;
    p.bby = p.bbz = 0;
  }
  const i64 kb = (l.xg - 1) * l.plane;  // x base only: in-plane offsets are plane-relative (non-negative)
  p.prev = analytic_start ? nullptr : prev + kb;
  p.cur = analytic_start ? nullptr : cur + kb;
  p.out1 = out1 + kb;
  p.out2 = out2 + kb;
  p.s = d_s;
  p.ihx2 = c.ihx2;
  p.ihy2 = c.ihy2;
  p.ihz2 = c.ihz2;
  p.tau2 = c.lam;  // τ²/h² and τ²/(2h²): the coefficients of d2sum
  p.half_tau2 = c.half_lam;
  p.check_mask = partials != nullptr ? (check_mask & ((1 << t.stages) - 1)) : 0;
  p.partials = p.check_mask != 0 ? partials : nullptr;
  W3D_REQUIRE(level_stride == 0 || level_stride >= pl.nblocks, "leapfrog_tb: level stride below the block count");
  p.lstride = level_stride > 0 ? level_stride : pl.nblocks;
  for (int k = 0; k < 4; ++k) p.ct[k] = (ct != nullptr && k < t.stages) ? ct[k] : 0.0;
  if (push != nullptr && push->on && push->signal_epoch != 0)  // (every pass of a solve: one full grid)
    W3D_REQUIRE(push->done_target % static_cast<unsigned>(pl.nblocks) == 0,
                "leapfrog_tb push: done_target must be a multiple of the grid");
  if (push != nullptr && push->on) {
    launch_push(p, pl.nblocks, t.stages, analytic_start, t.init_threads, stream);
  } else {
    switch (t.stages) {
      case 2: launch_s<2, false>(p, pl.nblocks, t, analytic_start, stream); break;
      case 3: launch_s<3, false>(p, pl.nblocks, t, analytic_start, stream); break;
      default: launch_s<4, false>(p, pl.nblocks, t, analytic_start, stream); break;
    }
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) fail(std::string("leapfrog_tb launch: ") + hipGetErrorString(e));
}

}  // namespace wave3d
