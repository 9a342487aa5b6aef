// Hand-written CDNA4 (gfx950) HIP kernels: launch interface.
//
//   k_init_first  : u⁰ = φ and u¹ = u⁰ + τ²/2·Δ_h u⁰ in one write-only pass (16 B/node), ghosts included
//                   (reference kernels K1 + K2).
//   k_leapfrog    : the hot loop — 2.5-D tiled 7-point leapfrog, x-marching register queue, LDS-staged (y,z) tile,
//                   16-byte node pairs, in place over u^{n−1}, Dirichlet BC by construction, optional fused error
//                   epilogue (reference kernels K3 + K4 + K5).
//   k_reduce      : fixed-order reduction of per-block error partials (deterministic).
//   k_pack/unpack : strided y/z halo faces ↔ contiguous RCCL staging buffers (reference kernel K6).
#pragma once

#include <vector>

#include <hip/hip_runtime.h>

#include "wave3d/cpu.hpp"
#include "wave3d/decomp.hpp"
#include "wave3d/deep_plan.hpp"
#include "wave3d/problem.hpp"

namespace wave3d {

// Error partial: x = L∞ candidate, y = Σe².
using Partial = double2;

// Tiling knobs of the leapfrog kernel (runtime-selectable so the tuner/bench can sweep them).
struct LeapfrogTiling {
  int variant = 1;        // 0 = LDS-staged workgroup tile (k_leapfrog_lds), 1 = register-queue waves (k_leapfrog_rq)
  int rows = 2;           // variant 1: rows (y) per wave held in registers (1, 2, 4 or 8)
  int ty = 8;             // variant 0: tile rows (y) per workgroup; block = 64 × ty threads
  int target_blocks = 0;  // x-chunking aims for at least this many work items (v0: workgroups, v1: waves; 0 = auto)
  bool xcd_remap = true;  // give each XCD a contiguous range of tiles (L2 reuse of tile halos)
  bool nt_store = true;   // non-temporal stores of u^{n+1} (measured faster on MI355X, profiles/)
};

// Number of error partials (v0: workgroups, v1: waves) a leapfrog launch over `boxes` writes.
int leapfrog_blocks(const Layout& l, const LBox* boxes, int nbox, const LeapfrogTiling& t);

void launch_init_first(const Layout& l, const Coeffs& c, const double* d_s, double* u0, double* u1,
                       hipStream_t stream);

// u¹ and u² (the first leapfrog step) computed analytically from φ in one write-only pass, ghosts included:
// bit-identical to launch_init_first followed by one launch_leapfrog over the whole interior. With `partials`
// the error of u² vs φ·ct2 over the owned interior is reduced per workgroup (init_two_partials() of them).
int init_two_partials(const Layout& l);
void launch_init_two(const Layout& l, const Coeffs& c, const double* d_s, double* u1, double* u2, double ct2,
                     Partial* partials, hipStream_t stream);

// Runs one leapfrog step over up to 6 boxes in a single launch. If `partials` is non-null the error vs φ·ct is reduced
// per workgroup into partials[0 .. leapfrog_blocks()).
void launch_leapfrog(const Layout& l, const Coeffs& c, const double* cur, double* old_out, const LBox* boxes, int nbox,
                     const double* d_s, double ct, Partial* partials, const LeapfrogTiling& t, hipStream_t stream);

// Temporal blocking: TWO leapfrog steps in one pass over HBM (u^{n+1}, u^{n+2} from u^{n−1}, u^n), 16 instead of
// 24 compulsory bytes per node-step. Needs every node of `box` to be updatable without a halo exchange (single rank:
// box = the whole global interior) and four distinct buffers (the redundant halo rows of step 1 read u^{n−1} that a
// neighbouring wave may not yet have consumed, so nothing is overwritten in place). If `partials` is non-null the
// error of u^{n+2} vs φ·ct2 is reduced per wave.
struct Leapfrog2Tiling {
  int rows = 2;           // output rows per wave (1, 2 or 4)
  int occupancy = 0;      // rows = 2 only: >= 3 builds for 3 waves/SIMD (register cap, some spills)
  int target_waves = 0;   // x-chunking target (0 = auto)
  bool xcd_remap = true;
  bool nt_store = true;
};
// [sx0, sx1): local x range where stage-1 (u^{n+1}) values are real; it extends one plane beyond `box` towards a
// neighbouring rank of a slab decomposition (those ghost planes are recomputed redundantly from 2-deep halos).
// Default (sx0 > sx1): this rank's updated region.
int leapfrog2_partials(const Layout& l, const LBox& box, const Leapfrog2Tiling& t);
void launch_leapfrog2(const Layout& l, const Coeffs& c, const double* prev, const double* cur, double* out1,
                      double* out2, const LBox& box, const double* d_s, double ct2, Partial* partials,
                      const Leapfrog2Tiling& t, hipStream_t stream, i64 sx0 = 1, i64 sx1 = 0);

// Deep temporal blocking: S = 2..4 leapfrog steps in one pass, all intermediate levels in LDS (32 × 32 (y,z) tiles
// marching in x (or in x chunks when the tiles alone do not fill the GPU), one workgroup per CU). Reads u^{n−1}, u^n; writes u^{n+S−1} into out1 and u^{n+S} into out2: 32/S
// compulsory bytes per node-step. Same preconditions as launch_leapfrog2 with S−1 stage-1 planes beyond the box.
// Error check of u^{n+k} when bit k−1 of `check_mask` is set (ct[k−1] = its time factor); stage k's partials go to
// partials + (k−1)·level_stride (0: leapfrog_tb_partials(), the launch's block count). analytic_start: the pass starts at n = 1 from u⁰ = φ and u¹ computed in
// the kernel (init_first's formulas, bit-identical), prev/cur are not read: it writes u^S, u^{S+1} with no HBM reads.
constexpr int kTbTile = 32;  // (y, z) tile edge of the LDS S-step passes (leapfrog_tb_kernel.hpp tbk::kTile)
struct LeapfrogTbTiling {
  int stages = 4;         // steps per pass: 2..4 (k_leapfrog_tb), 2..5 (k_leapfrog_p2)
  int threads = 1024;     // workgroup size (768 or 1024)
  int init_threads = 768; // ... of the analytic-start pass (measured at 512³, S = 3: 768 → 932 µs, 1024 → 1027 µs;
                          // the S = 4 passes go the other way: 768 → 1123 µs, 1024 → 1076 µs)
  bool xcd_remap = true;  // (stores are always non-temporal: measured faster at every S)
  bool xcd_blocks = false; // with xcd_remap: each XCD owns a square-ish tile block, not two-row strips (measured: no gain)
  int target_blocks = 256; // fewer (y,z) tiles than this: split x into chunks (one workgroup per CU at 1 WG/CU)
  int min_chunk = 16;      // ... of at least this many planes (each chunk recomputes S−1 planes on both sides)
  bool p2 = true;          // the pair-tiled pass (k_leapfrog_p2, S ≤ 5) wherever it applies (leapfrog_p2_supported)
  // (pair-tiled pass only) bit 0 / 1: also store u^{n+S−1} on the x ghost plane −1 / nx where a box starts / ends at
  // the rank's first / last plane. The pass computes that plane anyway (level S−1 reaches one node beyond the box), so
  // the slab exchange that follows sends S − 2 planes of u^{n+S−1} per face instead of S − 1 (solver_gpu.cpp
  // ghost_bits). The 4-step k_leapfrog_tb refuses it.
  int ghost_x1 = 0;
};
// Slab peer-push transport of an LDS pass (x faces only; every slab rank has the same plane geometry, so a plane's
// in-plane offsets are the same on both sides). The pass
//   * marches the upper face segment [x1 − T, x1) first, then [x0, x1 − T) (faces_first), so both face regions are
//     produced at the start of the pass;
//   * stores u^{n+S} of planes [0, T) / [nx − T, nx) and u^{n+S−1} of planes [0, T−1) / [nx − T + 1, nx) a second time,
//     straight into the lower / upper neighbour's staging over xGMI (fwd2 / fwd1: the neighbour's staging plane 0 of
//     the matching side and pass parity; nullptr: no neighbour);
//   * reads its own ghost planes [−T, 0) / [nx, nx + T) of u^n and u^{n−1} from its staging (gcur / gprev, plane 0 =
//     ghost plane −T resp. nx) instead of the field buffers;
//   * waits (wait_epoch > 0) for both neighbours' flags to reach wait_epoch before its first load, and raises its slot
//     in both neighbours' flags (rflag) to signal_epoch once every workgroup's stores are visible (the workgroup that
//     brings `done` to done_target).
struct TbPush {
  int on = 0, faces_first = 0;
  int T = 0;                          // ghost depth (planes) = the deepest pass
  int nx = 0;                         // this rank's planes
  double* fwd1[2] = {nullptr, nullptr};        // [lo, hi] neighbour staging for u^{n+S−1}
  double* fwd2[2] = {nullptr, nullptr};        // ... for u^{n+S}
  const double* gprev[2] = {nullptr, nullptr}; // own staging holding the ghost planes of u^{n−1} [lo, hi]
  const double* gcur[2] = {nullptr, nullptr};  // ... of u^n
  unsigned* flags = nullptr;          // own flags: [0] raised by the lower neighbour, [1] by the upper
  unsigned* rflag[2] = {nullptr, nullptr};     // this rank's slot in the lower / upper neighbour's flags
  int wait_side[2] = {0, 0};
  unsigned wait_epoch = 0, signal_epoch = 0;
  unsigned cp_wait = 0;               // host side: epoch the command processor waits for before the launch (0: none)
  unsigned tag = 0;                   // integrity check: the kernel compares it with its argument (else status = 2)
  int acquire = 1;                    // system-scope acquire at the pass start (perf attribution only: 0)
  unsigned* done = nullptr;           // workgroups done (local counter, zeroed per solve)
  unsigned done_target = 0;
  unsigned* status = nullptr;         // set to 1 when a wait timed out
  unsigned long long spin_ticks = 0;  // wait bound (100 MHz wall clock)
};

// Fused z-face pack of a 3-D block pass that precedes an exchange: stages S−1 and S store the owned
// nodes of the two z-face message parts (deep_plan.hpp: direction (0, 0, ∓1), w = the next pass's depth deep for
// u^{n+S}, w − 1 for u^{n+S−1}) straight into the send staging next to their field store. The z faces are the strided
// ones — rows of w ≤ 4 doubles one pitch apart, which a pack kernel reads at a fraction of the copy rate; x / y faces,
// edges and corners are whole-row copies and stay with k_box_copy. Send-region nodes on the global boundary are never
// computed and never written: the receiving pass loads the zero slot for them, not their ghosts (kernel `ld`).
struct TbPack {
  double* zf[2][2] = {};  // [low / high z face][field 0: u^{n+S}, 1: u^{n+S−1}]: the part in the send staging (or null)
  int w = 0;              // band width of u^{n+S}; u^{n+S−1}: w − 1
  int ny = 0, nz = 0;     // owned box
};

// Stage-real ranges of an LDS pass: per axis, where the intermediate levels hold real values (S−1 nodes into the
// S-deep ghosts towards neighbouring ranks); lo > hi: the axis default (x: compute box, y/z: no restriction).
inline LBox tb_default_real() { return LBox{1, 0, 1, 0, 1, 0}; }
// Write back and invalidate every XCD's L2 (and the L1s): enough workgroups to reach every CU each run a system-scope
// fence. Called once after allocating uncached buffers: lines of the same physical memory that a freed CACHED
// allocation left dirty in some L2 would otherwise be evicted over the new buffer's contents later (measured: an
// intermittent O(1) error in a fresh push staging after other solvers had been freed).
void l2_flush_all(hipStream_t stream);
// Raise the dynamic-LDS limit of every instantiation (call before capturing launches into a graph).
void leapfrog_tb_prepare(bool push = false);  // push: also the push-transport instantiations
size_t leapfrog_tb_lds_bytes(int stages);
int leapfrog_tb_partials(const Layout& l, const LBox& box, const LeapfrogTbTiling& t);
void launch_leapfrog_tb(const Layout& l, const Coeffs& c, const double* prev, const double* cur, double* out1,
                        double* out2, const LBox& box, const double* d_s, const double* ct, int check_mask,
                        Partial* partials, const LeapfrogTbTiling& t, hipStream_t stream,
                        const LBox& real = tb_default_real(), bool analytic_start = false, int level_stride = 0,
                        int grid_blocks = 0, const TbPush* push = nullptr, const TbPush* push_dev = nullptr,
                        const TbPack* pack = nullptr, const TbPack* pack_dev = nullptr);

// The pair-tiled S-step pass (kernels_leapfrog_p2.hip): the same contract as launch_leapfrog_tb for boxes inside the
// rank's y/z range that start and end on whole 16-byte pairs (leapfrog_p2_supported) and S = 2..5 (analytic start:
// 2..4); no push / fused pack. launch_leapfrog_tb dispatches to it when tiling.p2 is set and it applies.
// launch_leapfrog_p2_boxes: up to kP2MaxBoxes boxes in ONE launch (one grid, the x-chunk target shared by work), for the
// overlapped schedules' shell boxes; their partials share one slot of `grid_blocks` entries.
bool leapfrog_p2_supported(const Layout& l, const LBox& box, int stages);
int leapfrog_p2_partials(const Layout& l, const LBox& box, const LeapfrogTbTiling& t);
// (tests) the pair-tiled pass's thread → position table for S stages (kNT descriptors: (a+2) | (b+2)<<8 | lv<<16 |
// kind<<20) and its geometry {E, HY, HZ, PZ, tile, LDS bytes at xlen 512 (pass, analytic start), max xlen (same)}
std::vector<int> leapfrog_p2_table(int stages, std::vector<long>* geometry = nullptr);
void leapfrog_p2_prepare();
void launch_leapfrog_p2(const Layout& l, const Coeffs& c, const double* prev, const double* cur, double* out1,
                        double* out2, const LBox& box, const double* d_s, const double* ct, int check_mask,
                        Partial* partials, const LeapfrogTbTiling& t, hipStream_t stream, const LBox& real,
                        bool analytic_start, int level_stride = 0, int grid_blocks = 0);
constexpr int kP2MaxBoxes = 6;  // boxes per pair-tiled launch (deep_split: up to 6 shells)
void launch_leapfrog_p2_boxes(const Layout& l, const Coeffs& c, const double* prev, const double* cur, double* out1,
                              double* out2, const LBox* boxes, int nbox, const double* d_s, const double* ct,
                              int check_mask, Partial* partials, const LeapfrogTbTiling& t, hipStream_t stream,
                              const LBox& real, bool analytic_start, int level_stride = 0, int grid_blocks = 0);

// Error of a stored field vs φ·ct over `box` (step 1 / standalone check). Writes leapfrog-compatible partials and
// returns how many.
int error_blocks(const Layout& l, const LBox& box);
void launch_error(const Layout& l, const double* u, const LBox& box, const double* d_s, double ct, Partial* partials,
                  hipStream_t stream);

// out[0] = (max_i partials[i].x, Σ_i partials[i].y), in a fixed order.
void launch_reduce(const Partial* partials, int n, Partial* out, hipStream_t stream);
// Several independent reductions in one launch (one workgroup each, k_reduce's order: bit-identical results).
struct ReduceJob {
  const Partial* in;
  int n;
  Partial* out;
};
void launch_reduce_batch(const ReduceJob* jobs, int njobs, hipStream_t stream);

// S-deep exchange regions (deep_plan.hpp) <-> contiguous staging buffers. The job table is built once per plan and kept
// in device memory. mode 0: pack the send regions of u^{n+S} (u_s) and u^{n+S−1} (u_s1) into buf; 1: unpack buf into
// their receive (ghost) regions; 2: fill the receive regions with NaN (--poison-ghosts).
struct BoxJob {
  i64 buf;        // offset of the region in the staging buffer
  int count;      // nodes in the region
  int field;      // 0: u_s, 1: u_s1
  int x0, y0, z0; // first node (local)
  int ny, nz;     // extents of the region in y and z
  int blk0;       // first workgroup of this job
};
struct BoxCopyTable {
  BoxJob* jobs = nullptr;  // device
  int njobs = 0, nblocks = 0;
};
// skip_zfaces: leave out the parts of the pure z-face messages (direction (0, 0, ±1)): the pass packs them (TbPack)
BoxCopyTable make_box_copy_table(const DeepPlan& plan, bool recv_side, bool skip_zfaces = false);
void free_box_copy_table(BoxCopyTable& t);
void launch_box_copy(const Layout& l, const BoxCopyTable& t, int mode, double* u_s, double* u_s1, double* buf,
                     hipStream_t stream);

// Cross-rank flag words (copy-engine transport): one launch first waits until every word of `wait` equals wait.value
// (bounded by wait.ticks; a timeout sets *wait.status = 1), then stores signal.value into every word of `signal`.
struct FlagOp {
  static constexpr int kMax = 32;
  unsigned* addr[kMax] = {};
  int n = 0;
  unsigned value = 0;
  unsigned* status = nullptr;
  unsigned long long ticks = 0;
};
void launch_flag_sync(const FlagOp& wait, const FlagOp& signal, hipStream_t stream);

// Order-independent hash of the owned nodes of field f (Σ mix64(bits ^ mix64(global index)) mod 2⁶⁴), added into *out
// (zeroed by the caller): equal for bit-identical fields whatever the decomposition (GpuSolver::field_hash).
void launch_field_hash(const Layout& l, const double* f, unsigned long long* out, hipStream_t stream);

// Pack all strided faces of `plan` from `u` into `buf`, or unpack `buf` into the ghost layers of `u`.
void launch_pack(const Layout& l, const HaloPlan& plan, const double* u, double* buf, hipStream_t stream);
void launch_unpack(const Layout& l, const HaloPlan& plan, const double* buf, double* u, hipStream_t stream);

}  // namespace wave3d
