// GPU solver runtime. See wave3d/solver.hpp.
#include "wave3d/capture_guard.hpp"
#include "wave3d/solver.hpp"

#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace wave3d {

#define W3D_NCCL(expr)                                                                               \
  do {                                                                                               \
    ncclResult_t _r = (expr);                                                                        \
    if (_r != ncclSuccess) ::wave3d::fail(std::string(#expr) + ": " + ncclGetErrorString(_r));        \
  } while (0)

// ------------------------------------------------------------------------------------------------------------------
// Comm
// ------------------------------------------------------------------------------------------------------------------
std::string Comm::make_unique_id() {
  ncclUniqueId id;
  W3D_NCCL(ncclGetUniqueId(&id));
  return std::string(id.internal, sizeof(id.internal));
}

Comm::Comm(int rank, int world, const std::string& unique_id) : rank_(rank), world_(world) {
  ncclUniqueId id;
  W3D_REQUIRE(unique_id.size() == sizeof(id.internal), "bad RCCL unique id size");
  std::memcpy(id.internal, unique_id.data(), sizeof(id.internal));
  ncclComm_t c = nullptr;
  W3D_NCCL(ncclCommInitRank(&c, world, id, rank));
  comm_ = c;
  // self-test: one all-reduce of 1 per rank must give the world size, and RCCL must report `world` ranks. A
  // communicator that cannot move data fails here (with RCCL's error or the GPU-wait timeout) instead of inside a
  // captured solve. Run for every size (a one-rank communicator of the rccl-self group included).
  try {
    W3D_REQUIRE(count() == world, "RCCL self-test: ncclCommCount gave " + std::to_string(count()));
    const double n = comm_allreduce(*this, 1.0, false);
    W3D_REQUIRE(n == static_cast<double>(world), "RCCL self-test: all-reduce of 1 per rank gave " + std::to_string(n));
  } catch (...) {
    ncclCommAbort(c);  // the destructor does not run for a throwing constructor
    comm_ = nullptr;
    throw;
  }
}

std::vector<std::shared_ptr<Comm>> Comm::init_all(int world) {
  W3D_REQUIRE(world >= 1, "init_all: world must be >= 1");
  std::vector<ncclComm_t> raw(static_cast<size_t>(world), nullptr);
  std::vector<int> devs(static_cast<size_t>(world));
  for (int r = 0; r < world; ++r) devs[static_cast<size_t>(r)] = r;
  W3D_NCCL(ncclCommInitAll(raw.data(), world, devs.data()));
  std::vector<std::shared_ptr<Comm>> out;
  for (int r = 0; r < world; ++r) {
    std::shared_ptr<Comm> c(new Comm());
    c->rank_ = r;
    c->world_ = world;
    c->comm_ = raw[static_cast<size_t>(r)];
    out.push_back(std::move(c));
  }
  return out;
}

int Comm::count() const {
  int n = 0;
  W3D_NCCL(ncclCommCount(static_cast<ncclComm_t>(comm_), &n));
  return n;
}

int Comm::device() const {
  int d = -1;
  W3D_NCCL(ncclCommCuDevice(static_cast<ncclComm_t>(comm_), &d));
  return d;
}

Comm::~Comm() {
  if (comm_) ncclCommDestroy(static_cast<ncclComm_t>(comm_));
}

void Comm::check_async() const {
  ncclResult_t st = ncclSuccess;
  W3D_NCCL(ncclCommGetAsyncError(static_cast<ncclComm_t>(comm_), &st));
  if (st != ncclSuccess && st != ncclInProgress) fail(std::string("RCCL async error: ") + ncclGetErrorString(st));
}

// ------------------------------------------------------------------------------------------------------------------
// GpuSolver
// ------------------------------------------------------------------------------------------------------------------
namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Upper bound for one blocking wait on the GPU (env W3D_TIMEOUT_S, default 300 s): a lost peer or a stuck halo
// exchange turns into an error instead of a hang.
double gpu_timeout_s() {
  static const double t = [] {
    const char* v = std::getenv("W3D_TIMEOUT_S");
    const double x = v ? std::atof(v) : 0.0;
    return x > 0.0 ? x : 300.0;
  }();
  return t;
}

// Wait for a stream while polling RCCL for asynchronous failures (a dead peer must not hang the job forever).
void wait_stream(hipStream_t s, const Comm* comm, double timeout_s) {
  const double t0 = now_s();
  for (;;) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) fail(std::string("stream failed: ") + hipGetErrorString(e));
    if (comm) comm->check_async();
    if (now_s() - t0 > timeout_s) fail("timed out waiting for the GPU (halo exchange stuck?)");
    std::this_thread::yield();
  }
}

}  // namespace

// Multi-stream captures with cross-stream event joins repeated per unit (the multi-rank schedules: side-stream
// exchange joined back every pass) crash inside hipStreamEndCapture of the HIP 7.0 runtime that PyTorch-ROCm bundles
// (tools/probes/capture_probe.hip pattern 5, capture_probe2.hip); the system ROCm 7.2 runtime captures them correctly
// (probed, and the rccl-self group graphs). Multi-rank solves are therefore captured only on HIP >= 7.2 (the native
// CLI, which bench.py runs per rank, always is); inside a torch process they run eagerly. W3D_FORCE_CAPTURE=1
// overrides the check.
bool multistream_capture_safe() {
  static const bool ok = [] {
    if (const char* f = std::getenv("W3D_FORCE_CAPTURE"); f && *f == '1') return true;
    int v = 0;
    if (hipRuntimeGetVersion(&v) != hipSuccess) return false;
    return v >= 70200000;
  }();
  return ok;
}

GpuSolver::GpuSolver(const Problem& prob, const SolverOptions& opt, int rank, int world, std::shared_ptr<Comm> comm,
                     bool loopback)
    : prob_(prob), opt_(opt), coef_(Coeffs::from(prob)), rank_(rank), world_(world), comm_(std::move(comm)),
      loopback_(loopback) {
  prob_.validate();
  W3D_HIP(hipGetDevice(&dev_));
  // (perf studies: tiling overrides of the LDS S-step kernel; W3D_TB_TARGET=B splits the x march into chunks when the
  // tile grid has fewer than B tiles, W3D_TB_MINCHUNK its minimum planes, W3D_TB_XCDBLOCKS=1 square XCD blocks)
  if (const char* v = std::getenv("W3D_TB_TARGET")) opt_.tiling_tb.target_blocks = std::atoi(v);
  if (const char* v = std::getenv("W3D_RESERVE_CUS")) opt_.reserve_cus = std::atoi(v);
  if (const char* v = std::getenv("W3D_TB_MINCHUNK")) opt_.tiling_tb.min_chunk = std::atoi(v);
  if (const char* v = std::getenv("W3D_TB_XCDBLOCKS")) opt_.tiling_tb.xcd_blocks = *v == '1';
  if (const char* v = std::getenv("W3D_TB_XCDREMAP")) opt_.tiling_tb.xcd_remap = *v == '1';  // (A/B runs)
  W3D_REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad rank/world");
  W3D_REQUIRE(world == 1 || comm_ || loopback_ || opt_.fake_comm || ((opt_.push || opt_.sdma) && opt_.push_no_collective),
              "world > 1 needs an RCCL communicator (or the loopback group, or the push / sdma transport without one)");
  W3D_REQUIRE(!(opt_.push && opt_.sdma), "push and sdma are two different transports");
  dims_ = parse_dims(opt_.decomp, world, prob_.N);
  const Box box = rank_box(prob_, dims_, rank);
  W3D_REQUIRE(box.nx() >= 1 && box.ny() >= 1 && box.nz() >= 1,
              "decomposition leaves a rank without nodes; use fewer ranks or a larger N");
  // schedule mode: temporal blocking on one rank, or on a 1-D slab decomposition with `temporal`-deep x halos (LDS
  // passes) or 2-deep ones (two-step passes). Decided from the SMALLEST rank box so every rank picks the same mode.
  mode_ = Mode::kSingleStep;
  W3D_REQUIRE(opt_.temporal >= 1 && opt_.temporal <= 5, "temporal must be 1..5");
  // 5-step passes: the pair-tiled kernel only (one rank, slab ranks; below: 3-D blocks and the push transport keep
  // k_leapfrog_tb's S ≤ 4)
  if (opt_.temporal == 5 && (!opt_.tb || !opt_.tiling_tb.p2)) opt_.temporal = 4;
  if (opt_.temporal >= 2 && world == 1) mode_ = Mode::kFusedSingle;
  const bool slab = dims_.py == 1 && dims_.pz == 1;
  if (opt_.temporal >= 2 && world > 1) {
    // smallest extent of any rank along each axis (every rank must be able to feed its neighbours' deep halos)
    i64 mn[3] = {box.nx(), box.ny(), box.nz()};
    for (int r = 0; r < world; ++r) {
      const Box b = rank_box(prob_, dims_, r);
      mn[0] = imin(mn[0], b.nx());
      mn[1] = imin(mn[1], b.ny());
      mn[2] = imin(mn[2], b.nz());
    }
    const int rem = prob_.K - (analytic_ok() ? 1 : 2);  // steps left to the passes (each takes 2..temporal)
    // (the pass depth every rank will use: 5-step passes everywhere but on the push transport, see below)
    const i64 T2 = 2 * (opt_.push ? std::min(opt_.temporal, 4) : opt_.temporal);
    // 3-D blocks: S-deep ghosts on every split axis, one exchange (faces, edges, corners) between passes
    const bool block_fits = (dims_.px == 1 || mn[0] >= imax(T2, 8)) && (dims_.py == 1 || mn[1] >= imax(T2, 8)) &&
                            (dims_.pz == 1 || mn[2] >= imax(T2, 8));
    if (opt_.tb && opt_.init2 && rem >= 2 && slab && mn[0] >= imax(opt_.tb_min_planes, T2))
      mode_ = Mode::kDeepTb;
    else if (opt_.tb && opt_.init2 && rem >= 2 && !slab && block_fits)
      mode_ = Mode::kDeepTb;
    // (two-step passes, measured with --fake-rank on 512³: they win from ~128 local planes up, but at 64 planes the
    // two 2-plane shell passes and the per-chunk stage-1 recompute cost more than the saved traffic)
    else if (slab && mn[0] >= opt_.deep_min_planes && mn[0] >= 3 && pairable())
      mode_ = Mode::kDeep;
  }
  block_tb_ = mode_ == Mode::kDeepTb && !slab;
  // (3-D blocks, overlapped or not, take 5-step pair-tiled passes: the overlapped schedule's shell and interior boxes
  // are cut on whole pairs, cpu.hpp deep_split; the push transport's forwarding stores are k_leapfrog_tb's)
  if (opt_.temporal == 5 && world > 1 && (mode_ != Mode::kDeepTb || opt_.push)) opt_.temporal = 4;
  // (the fused z-face pack lives in k_leapfrog_tb: with the pair-tiled pass the pack kernel packs the z faces too)
  if (block_tb_ && opt_.tiling_tb.p2) opt_.fused_pack = false;
  if (opt_.push && world > 1) {
    W3D_REQUIRE(mode_ == Mode::kDeepTb && !block_tb_, "push transport: slab LDS passes (deep-tb) only, not " + mode());
    push_ = true;
  }
  for (int attempt = 0; attempt < 2; ++attempt) {
    const i64 T = opt_.temporal;
    lay_ = make_layout(prob_, box, 16, mode_ == Mode::kDeep ? 2 : (mode_ == Mode::kDeepTb && dims_.px > 1) ? T : 1,
                       block_tb_ && dims_.py > 1 ? T : 1, block_tb_ && dims_.pz > 1 ? T : 1);
    // memory plan: temporal blocking needs four field buffers; fall back to the two-buffer in-place scheme when four
    // do not fit next to the other allocations (2049³ fp64 is 68.8 GB per buffer)
    size_t free_b = 0, total_b = 0;
    W3D_HIP(hipMemGetInfo(&free_b, &total_b));
    const double need2 = 2.0 * static_cast<double>(lay_.bytes()), headroom = 2.0e9;
    if (mode_ != Mode::kSingleStep && 2.0 * need2 + headroom > static_cast<double>(free_b)) {
      W3D_REQUIRE(!push_, "push transport: four field buffers do not fit");
      mode_ = Mode::kSingleStep;
      block_tb_ = false;
      continue;
    }
    W3D_REQUIRE(need2 + 1.0e8 < static_cast<double>(free_b),
                "not enough device memory for two field buffers of " + std::to_string(lay_.bytes()) + " bytes");
    break;
  }
  if (opt_.sdma && world > 1) {
    W3D_REQUIRE(mode_ == Mode::kDeepTb, "sdma transport: LDS multi-step passes (deep-tb, slab or block) only, not " + mode());
    sdma_ = true;
  }
  plan_ = make_halo_plan(lay_, dims_, rank);
  full_ = compute_box(lay_);

  // interior = compute box minus one layer on every side that has a neighbour; shell = the rest (cpu.hpp shell_split)
  bool nb[3][2];
  for (int a = 0; a < 3; ++a)
    for (int s = 0; s < 2; ++s) nb[a][s] = neighbor_rank(dims_, rank, a, s) >= 0;
  shell_split(full_, nb, shell_, interior_);

  // deep-halo slab: the 2 owned planes next to each neighbour are the shell (they are what the neighbours receive);
  // stage-1 values are real one ghost plane beyond each neighbour face
  if (mode_ == Mode::kDeep) {
    i64 lo = full_.x0, hi = full_.x1;
    if (nb[0][0]) {
      const i64 e = imin(full_.x0 + 2, full_.x1);
      dshell_.push_back(LBox{full_.x0, e, full_.y0, full_.y1, full_.z0, full_.z1});
      lo = e;
    }
    if (nb[0][1]) {
      const i64 b = imax(full_.x1 - 2, lo);
      if (b < full_.x1) dshell_.push_back(LBox{b, full_.x1, full_.y0, full_.y1, full_.z0, full_.z1});
      hi = b;
    }
    dint_ = hi > lo ? LBox{lo, hi, full_.y0, full_.y1, full_.z0, full_.z1} : LBox{};
    sx0_ = full_.x0 - (nb[0][0] ? 1 : 0);
    sx1_ = full_.x1 + (nb[0][1] ? 1 : 0);
  }
  // deep-tb slab: stage values are real up to temporal − 1 planes beyond each neighbour face (recomputed from the
  // temporal-deep halo); the shell/interior split depends on the next pass's depth and is made per unit
  nb_lo_ = nb[0][0];
  nb_hi_ = nb[0][1];
  if (mode_ == Mode::kDeepTb) {
    const i64 T1 = opt_.temporal - 1;
    sx0_ = full_.x0 - (nb_lo_ ? T1 : 0);
    sx1_ = full_.x1 + (nb_hi_ ? T1 : 0);
    sreal_ = LBox{sx0_, sx1_, full_.y0 - (nb[1][0] ? T1 : 0), full_.y1 + (nb[1][1] ? T1 : 0),
                  full_.z0 - (nb[2][0] ? T1 : 0), full_.z1 + (nb[2][1] ? T1 : 0)};
  }
  // 3-D block passes: one plan (and device job tables) per pass depth that can follow an exchange
  if (block_tb_) {
    // the send staging holds one region per depth (sbase_): the fused z-face pack writes only the real nodes of its
    // message parts and leaves the global-boundary entries at their initial zero, which a region shared with the
    // messages of another depth (whose parts land at other offsets) would overwrite — measured: a depth-3 exchange
    // followed by a depth-4 one sent the depth-3 values of those entries as boundary ghosts
    for (int st = 2; st <= opt_.temporal; ++st) {
      deep_[st] = make_deep_plan(lay_, dims_, rank_, st);
      deep_max_ = imax(deep_max_, deep_[st].total);
      sbase_[st] = send_total_;
      send_total_ += round_up(deep_[st].total, 32);
    }
  }

  // device memory
  if (const char* cs = std::getenv("W3D_CU_SPLIT"); cs && !loopback_ && (std::strchr(cs, '/') || !std::strcmp(cs, "auto"))) {
    // rehearsal of several ranks on ONE GPU with truly concurrent passes (W3D_CU_SPLIT=r/P, or auto = rank/world):
    // this rank's compute stream only gets the r-th of P disjoint CU ranges, so a pass waiting in the kernel for a
    // peer can never hold the CUs the peer's pass needs
    const bool au = !std::strcmp(cs, "auto");
    const int r = au ? rank : std::atoi(cs), P = au ? world : std::atoi(std::strchr(cs, '/') + 1);
    int dev = 0, ncu = 0;
    W3D_HIP(hipGetDevice(&dev));
    W3D_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    W3D_REQUIRE(P >= 1 && r >= 0 && r < P && ncu >= P, "W3D_CU_SPLIT must be r/P with 0 <= r < P <= CUs");
    std::vector<uint32_t> mask(static_cast<size_t>((ncu + 31) / 32), 0u);
    for (int c = r * ncu / P; c < (r + 1) * ncu / P; ++c) mask[static_cast<size_t>(c / 32)] |= 1u << (c % 32);
    W3D_HIP(hipExtStreamCreateWithCUMask(&s0_, static_cast<uint32_t>(mask.size()), mask.data()));
  } else if (opt_.reserve_cus > 0) {
    int dev = 0, ncu = 0;
    W3D_HIP(hipGetDevice(&dev));
    W3D_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    W3D_REQUIRE(opt_.reserve_cus < ncu, "reserve_cus must leave the passes at least one CU");
    std::vector<uint32_t> mask(static_cast<size_t>((ncu + 31) / 32), 0u);
    for (int c = 0; c < ncu - opt_.reserve_cus; ++c) mask[static_cast<size_t>(c / 32)] |= 1u << (c % 32);
    W3D_HIP(hipExtStreamCreateWithCUMask(&s0_, static_cast<uint32_t>(mask.size()), mask.data()));
    if (opt_.tiling_tb.target_blocks == LeapfrogTbTiling{}.target_blocks) opt_.tiling_tb.target_blocks = ncu - opt_.reserve_cus;
  } else {
    W3D_HIP(hipStreamCreateWithFlags(&s0_, hipStreamNonBlocking));
  }
  {
    // the exchange stream gets the highest priority so RCCL's copy kernels are dispatched ahead of the waiting
    // interior workgroups: the halo overlaps the interior update instead of queueing behind it
    int lo = 0, hi = 0;
    W3D_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    W3D_HIP(hipStreamCreateWithPriority(&s1_, hipStreamNonBlocking, hi));
  }
  W3D_HIP(hipEventCreateWithFlags(&ev_shell_, hipEventDisableTiming));
  W3D_HIP(hipEventCreateWithFlags(&ev_halo_, hipEventDisableTiming));
  W3D_HIP(hipEventCreateWithFlags(&ev_packed_, hipEventDisableTiming));
  nbuf_ = mode_ == Mode::kSingleStep ? 2 : 4;
  for (int b = 0; b < nbuf_; ++b) {
    W3D_HIP(hipMalloc(&u_[b], static_cast<size_t>(lay_.bytes())));
    W3D_HIP(hipMemset(u_[b], 0, static_cast<size_t>(lay_.bytes())));
  }
  if (push_) {
    // staging in fine-grained device memory (W3D_PUSH_STAGING=uncached: uncached), flags uncached: the neighbours'
    // stores are write-through (system scope) and a reader invalidates its L2 once per pass after its wait
    // (system-scope acquire, leapfrog_tb_kernel.hpp)
    const size_t sb = static_cast<size_t>(8 * lay_.xg * lay_.plane) * sizeof(double);
    const char* mt = std::getenv("W3D_PUSH_STAGING");  // (experiment: "uncached" instead of fine-grained)
    const unsigned stg_flags = mt && !std::strcmp(mt, "uncached") ? hipDeviceMallocUncached : hipDeviceMallocFinegrained;
    W3D_HIP(hipExtMallocWithFlags(reinterpret_cast<void**>(&stg_), sb, stg_flags));
    W3D_HIP(hipMemset(stg_, 0, sb));
    W3D_HIP(hipExtMallocWithFlags(reinterpret_cast<void**>(&flags_), 256, hipDeviceMallocUncached));
    l2_flush_all(nullptr);  // (no stale dirty line of a freed cached buffer may land on them later: kernels.hpp)
    W3D_HIP(hipDeviceSynchronize());
    W3D_HIP(hipMemset(stg_, 0, sb));
    W3D_HIP(hipMemset(flags_, 0, 256));
    const size_t tb = static_cast<size_t>(prob_.K) * sizeof(TbPush);  // (a solve has at most K passes)
    // two host tables: [0, K) for the captured solve (its H2D copy node reads the table at every replay), [K, 2K) for
    // eager solves — an eager solve after the capture (e.g. the phase-timer solve) must not rewrite the tags the graph's
    // kernel nodes were captured with
    W3D_HIP(hipHostMalloc(reinterpret_cast<void**>(&push_host_), 2 * tb, hipHostMallocDefault));
    // (fine-grained device memory for the pass table: the table is rewritten by host-to-device copies, and each pass
    // starts with a system-scope acquire, so no pass reads it through an L2 line the same memory held for an earlier,
    // freed buffer — measured: a fresh solver's passes once read the previous solver's table there)
    W3D_HIP(hipExtMallocWithFlags(reinterpret_cast<void**>(&push_dev_), tb, hipDeviceMallocFinegrained));
    // (stream memops are not captured into graphs; running epochs are per-launch arguments)
    if (opt_.push_cp_wait || opt_.push_no_collective) opt_.graph = false;
  }
  const std::vector<double> s = sin_table_ext(prob_);
  W3D_HIP(hipMalloc(&d_s_, s.size() * sizeof(double)));
  W3D_HIP(hipMemcpy(d_s_, s.data(), s.size() * sizeof(double), hipMemcpyHostToDevice));
  const i64 stage = imax(plan_.packed_doubles, deep_max_);
  if (stage > 0) {
    const i64 sstage = imax(stage, send_total_);
    W3D_HIP(hipMalloc(&send_buf_, static_cast<size_t>(sstage) * sizeof(double)));
    W3D_HIP(hipMalloc(&recv_buf_, static_cast<size_t>(stage) * sizeof(double)));
    W3D_HIP(hipMemset(send_buf_, 0, static_cast<size_t>(sstage) * sizeof(double)));
  }
  if (sdma_) sdma_alloc();
  if (block_tb_) {
    // fused z-face pack (its message parts live in send_buf_, zeroed once: nodes on the global boundary are never
    // written — each exchange depth has its own send region, sbase_ — and arrive as the zero boundary ghosts)
    const bool fused = opt_.fused_pack && opt_.tb;
    for (int st = 2; st <= opt_.temporal; ++st) {
      pack_tab_[st] = make_box_copy_table(deep_[st], false, fused);
      unpack_tab_[st] = make_box_copy_table(deep_[st], true);
      if (!fused) continue;
      TbPack& k = pk_host_[st];
      k.w = st;
      k.ny = static_cast<int>(lay_.ny);
      k.nz = static_cast<int>(lay_.nz);
      for (const DeepPeer& q : deep_[st].peers)
        if (q.dir[0] == 0 && q.dir[1] == 0)
          for (const DeepPart& part : q.parts) k.zf[q.dir[2] > 0 ? 1 : 0][part.field] = send_buf_ + sbase_[st] + q.buf_off + part.off;
    }
    if (fused) {
      W3D_HIP(hipMalloc(&pk_dev_, sizeof(pk_host_)));
      W3D_HIP(hipMemcpy(pk_dev_, pk_host_, sizeof(pk_host_), hipMemcpyHostToDevice));
    }
  }
  n_full_ = leapfrog_blocks(lay_, &full_, 1, opt_.tiling);
  n_shell_ = leapfrog_blocks(lay_, shell_.data(), static_cast<int>(shell_.size()), opt_.tiling);
  n_int_ = leapfrog_blocks(lay_, &interior_, 1, opt_.tiling);
  n_fused_ = (mode_ == Mode::kFusedSingle && !full_.empty()) ? leapfrog2_partials(lay_, full_, opt_.tiling2) : 0;
  if ((mode_ == Mode::kFusedSingle || mode_ == Mode::kDeepTb) && opt_.tb && !full_.empty()) {
    LeapfrogTbTiling t = opt_.tiling_tb;
    t.stages = opt_.temporal;  // partials per level do not depend on the stage count
    n_tb_ = leapfrog_tb_partials(lay_, full_, t);
    // multi-rank units also launch sub-boxes of the compute box (shells, interior), whose fewer tiles may be split into
    // more x chunks: at most tiles · ceil(target / tiles) < tiles + target blocks (their slots are n_tb_ wide)
    if (mode_ == Mode::kDeepTb)
      n_tb_ = static_cast<int>(imax(n_tb_, round_up(ceil_div(full_.y1 - full_.y0, kTbTile) *
                                                            ceil_div(full_.z1 - full_.z0, kTbTile) +
                                                        t.target_blocks, 8)));
    leapfrog_tb_prepare(push_);
  }
  int n_deep = 0;
  for (const LBox& b : dshell_) {
    n_dshell_.push_back(leapfrog2_partials(lay_, b, opt_.tiling2));
    n_deep += n_dshell_.back();
  }
  n_dint_ = dint_.empty() ? 0 : leapfrog2_partials(lay_, dint_, opt_.tiling2);
  n_deep += n_dint_;
  n_partials_ = std::max({n_full_, n_shell_ + n_int_, error_blocks(lay_, full_), n_fused_, n_deep,
                          opt_.init2 ? init_two_partials(lay_) : 0, 1});
  W3D_HIP(hipMalloc(&partials_, static_cast<size_t>(n_partials_) * sizeof(Partial)));
  // the LDS passes' partials live apart: their reductions are deferred, so the immediate users of partials_ (init,
  // single steps between passes) must not overwrite them
  if (n_tb_ > 0)
    W3D_HIP(hipMalloc(&tb_partials_, static_cast<size_t>(kTbRegions) * kTbLevels * kTbSlots * n_tb_ * sizeof(Partial)));
  W3D_HIP(hipMalloc(&errlog_, static_cast<size_t>(prob_.K + 1) * sizeof(Partial)));
  W3D_HIP(hipMemset(errlog_, 0, static_cast<size_t>(prob_.K + 1) * sizeof(Partial)));
  W3D_HIP(hipMalloc(&errall_, static_cast<size_t>(world_) * (prob_.K + 1) * sizeof(Partial)));
  ct_.resize(static_cast<size_t>(prob_.K + 1));
  for (int n = 0; n <= prob_.K; ++n) ct_[static_cast<size_t>(n)] = time_factor(prob_, n);
  // (group ranks: the GpuGroup captures the whole group solve itself)
  if (opt_.timers || opt_.debug_sync || loopback_) opt_.graph = false;
}

GpuSolver::~GpuSolver() {
  // a destructor must not throw: release errors are dropped on purpose (the device may already be in an error state)
  if (graph_exec_) (void)hipGraphExecDestroy(graph_exec_);
  for (hipGraphExec_t g : xgraph_)
    if (g) (void)hipGraphExecDestroy(g);
  for (XLink& l : xlinks_)
    if (l.ipc) {
      for (double* p : {l.u[0], l.u[1], l.u[2], l.u[3], l.recv})
        if (p) (void)hipIpcCloseMemHandle(p);
      if (l.flags) (void)hipIpcCloseMemHandle(l.flags);
    }
  if (xflags_) (void)hipFree(xflags_);
  if (xvals_) (void)hipFree(xvals_);
  for (hipStream_t c : xcs_) (void)hipStreamDestroy(c);
  for (hipEvent_t e : xcev_) (void)hipEventDestroy(e);
  if (xfork_) (void)hipEventDestroy(xfork_);
  for (BoxCopyTable& t : pack_tab_) free_box_copy_table(t);
  for (BoxCopyTable& t : unpack_tab_) free_box_copy_table(t);
  if (pk_dev_) (void)hipFree(pk_dev_);
  for (double* p : {u_[0], u_[1], u_[2], u_[3], d_s_, send_buf_, recv_buf_})
    if (p) (void)hipFree(p);
  if (partials_) (void)hipFree(partials_);
  if (tb_partials_) (void)hipFree(tb_partials_);
  if (errlog_) (void)hipFree(errlog_);
  if (errall_) (void)hipFree(errall_);
  for (hipEvent_t e : ev_pool_) (void)hipEventDestroy(e);
  if (ev_shell_) (void)hipEventDestroy(ev_shell_);
  if (ev_halo_) (void)hipEventDestroy(ev_halo_);
  if (ev_packed_) (void)hipEventDestroy(ev_packed_);
  for (int k = 0; k < 2; ++k)
    if (peer_ipc_[k]) {
      (void)hipIpcCloseMemHandle(peer_stg_[k]);
      (void)hipIpcCloseMemHandle(peer_flags_[k]);
    }
  if (stg_) (void)hipFree(stg_);
  if (push_host_) (void)hipHostFree(push_host_);
  if (hbatch_) (void)hipHostFree(hbatch_);
  if (push_dev_) (void)hipFree(push_dev_);
  if (flags_) (void)hipFree(flags_);
  if (s0_ && own_s0_) (void)hipStreamDestroy(s0_);
  if (s1_) (void)hipStreamDestroy(s1_);
}

size_t GpuSolver::device_bytes() const {
  return static_cast<size_t>(nbuf_) * static_cast<size_t>(lay_.bytes()) +
         static_cast<size_t>(imax(plan_.packed_doubles, deep_max_) + imax(plan_.packed_doubles, send_total_)) *
             sizeof(double) +
         static_cast<size_t>(n_partials_) * sizeof(Partial) + static_cast<size_t>(prob_.N + 3) * sizeof(double) +
         static_cast<size_t>(kTbRegions) * kTbLevels * kTbSlots * static_cast<size_t>(n_tb_) * sizeof(Partial);
}

void GpuSolver::set_state(const double* prev, const double* cur, int n0) {
  W3D_REQUIRE(n0 >= 1 && n0 < prob_.K, "resume step must be in [1, K)");
  W3D_REQUIRE(mode_ != Mode::kDeepTb || prob_.K - n0 >= 2, "resume: the multi-rank LDS passes need >= 2 steps left");
  W3D_REQUIRE(mode_ != Mode::kDeep || (prob_.K - n0) % 2 == 0, "resume: two-step passes need an even step count left");
  for (int k = 0; k < 2; ++k) {
    resume_[k].assign(static_cast<size_t>(lay_.total), 0.0);
    global_to_local(lay_, k == 0 ? prev : cur, resume_[k].data());
  }
  resume_n_ = n0;
}

std::vector<int> GpuSolver::check_steps() const {
  std::vector<int> v;
  const int ce = opt_.check_every;
  for (int n = resume_n_ + 1; n <= prob_.K; ++n)
    if ((ce > 0 && n % ce == 0) || n == prob_.K) v.push_back(n);
  return v;
}

std::string GpuSolver::transport() const {
  if (world_ == 1) return "none";
  if (sdma_) return "sdma";
  if (push_) return "push";
  if (opt_.fake_comm) return opt_.fake_traffic && comm_ ? "fake-rccl-self" : "fake";
  if (loopback_) return comm_ ? "rccl-self" : "loopback";
  return "rccl";
}

// (the schedule of the last run(): units_ and analytic_ are rebuilt at the start of every solve)
GpuSolver::Traffic GpuSolver::traffic() {
  Traffic t;
  const double node_bytes = static_cast<double>(lay_.cx1 - lay_.cx0) * static_cast<double>(lay_.cy1 - lay_.cy0) *
                            static_cast<double>(lay_.cz1 - lay_.cz0) * sizeof(double);
  if (!analytic_ && resume_n_ == 0) t.field_bytes += 2.0 * node_bytes;  // init kernel: u¹, u² (or u⁰, u¹)
  for (const Unit& u : units_) t.field_bytes += node_bytes * (u.analytic ? 2.0 : u.fused() ? 4.0 : 3.0);
  if (push_) {  // each pass but the last forwards T planes of u^{n+S} and T − 1 of u^{n+S−1} per face
    const double T = static_cast<double>(lay_.xg);
    t.halo_bytes = static_cast<double>(plan_.faces.size()) * (2.0 * T - 1.0) * static_cast<double>(lay_.plane) *
                   sizeof(double) * static_cast<double>(units_.empty() ? 0 : units_.size() - 1);
    return t;
  }
  const std::vector<Msg> keep = msgs_;
  const int keep_s = deep_s_;
  for (int i = 0; i < static_cast<int>(units_.size()); ++i) {
    const int gb = ghost_bits(i);  // (the stored u^{n+S−1} ghost planes: one plane per face)
    t.field_bytes += static_cast<double>((gb & 1) + (gb >> 1)) * static_cast<double>(lay_.plane) * sizeof(double);
    if (!needs_exchange(i)) continue;
    build_msgs(i);
    for (const Msg& m : msgs_) t.halo_bytes += static_cast<double>(m.count) * sizeof(double);
  }
  msgs_ = keep;
  deep_s_ = keep_s;
  return t;
}

std::string GpuSolver::mode() const {
  switch (mode_) {
    case Mode::kFusedSingle: return "fused-single";
    case Mode::kDeep: return "deep-halo";
    case Mode::kDeepTb: return block_tb_ ? "deep-tb-block" : "deep-tb";
    default: return "single-step";
  }
}

// ------------------------------------------------------------------------------------------------------------------
// schedule
// ------------------------------------------------------------------------------------------------------------------
bool GpuSolver::split() const { return opt_.overlap && plan_.any(); }
bool GpuSolver::post_exchange() const { return mode_ == Mode::kDeep || mode_ == Mode::kDeepTb || split(); }

// (3-D block passes always exchange after the whole pass: the y/z face shells of S-deep halos would be thin tile
// strips recomputing most of their tiles)
bool GpuSolver::late_exchange() const { return mode_ == Mode::kDeepTb && !opt_.overlap; }

bool GpuSolver::needs_exchange(int i) const {
  if (!plan_.any() || push_) return false;  // (push: the passes deliver the ghosts themselves)
  return post_exchange() ? i + 1 < static_cast<int>(units_.size()) : i > 0;
}

// u^{n+S−1} ghost-plane stores (SolverOptions::ghost_store): unit i's pair-tiled passes also store that level on the
// ghost plane beyond each x face with a neighbour (bit 0: plane −1, bit 1: plane nx), which exchange i then leaves out.
// Slab ranks only (a 3-D block rank's edge and corner regions would become L-shaped messages), and only where every
// pass of the unit runs on the pair-tiled kernel (launch_leapfrog_tb refuses the bits otherwise). Every rank computes
// the same bits for the same exchange (same units, same options), so both ends of a face agree on the message size.
int GpuSolver::ghost_bits(int i) const {
  if (!opt_.ghost_store || mode_ != Mode::kDeepTb || block_tb_ || push_ || !opt_.tiling_tb.p2 || pk_dev_ != nullptr ||
      i < 0 || i >= static_cast<int>(units_.size()) || !needs_exchange(i))
    return 0;
  const Unit& u = units_[static_cast<size_t>(i)];
  if ((u.analytic && u.steps > 4) || !leapfrog_p2_supported(lay_, full_, u.steps)) return 0;
  int bits = 0;
  for (const Face& f : plan_.faces)
    if (f.axis == 0) bits |= 1 << f.side;
  return bits;
}

hipStream_t GpuSolver::xstream() const {
  return post_exchange() && opt_.overlap && !late_exchange() && !push_ ? s1_ : s0_;
}

// Deep-halo fused passes need every unit to be a pair with no error check on its intermediate step, starting from the
// analytic (u¹, u²): K even and no odd check step below K.
bool GpuSolver::pairable() const {
  const int K = prob_.K;
  if (!opt_.init2 || K < 4 || (K - 2) % 2 != 0) return false;
  for (int n : check_steps())
    if (n > 2 && n < K && (n % 2) != 0) return false;
  return true;
}

bool GpuSolver::analytic_ok() const {
  if (!opt_.tb || !opt_.init2 || opt_.temporal < 2 || prob_.K < 3) return false;
  for (int n : check_steps())
    if (n == 1) return false;  // u¹ is the pass's input level: it cannot carry a check
  return true;
}

void GpuSolver::build_units() {
  units_.clear();
  const int K = prob_.K;
  int n = start_n_;
  if ((mode_ == Mode::kFusedSingle && opt_.tb) || mode_ == Mode::kDeepTb) {
    // split the K − n remaining steps into passes of 1..temporal steps minimising the summed cost: µs per step of a
    // pass of s steps with every 2nd level checked, measured at 512³ (tools/tune_leapfrog.py --tb); the analytic
    // first pass reads nothing but computes u⁰, u¹ (compute-bound). Slab ranks (deep-tb) take passes of ≥ 2 steps
    // only: every pass writes the two levels the next one reads, so each exchange is one message pair per face.
    static const double kStepCostTb[6] = {0.0, 610.0, 437.0, 302.0, 258.0, 1e9};
    // (analytic: φ-stage start, re-measured)
    static const double kAnalyticCostTb[6] = {0.0, 1e9, 346.0, 300.0, 318.0, 1e9};
    // the pair-tiled passes (k_leapfrog_p2, one rank): µs per step at 512³ (profiles/r5/)
    static const double kStepCostP2[6] = {0.0, 610.0, 430.0, 290.0, 225.0, 180.0};
    static const double kAnalyticCostP2[6] = {0.0, 1e9, 300.0, 200.0, 135.0, 1e9};
    // (slab ranks and 3-D block ranks too: their shell / interior boxes are cut on whole pairs)
    const bool p2 = opt_.tiling_tb.p2 && !push_ && leapfrog_p2_supported(lay_, full_, 2);
    const double* kStepCost = p2 ? kStepCostP2 : kStepCostTb;
    const double* kAnalyticCost = p2 ? kAnalyticCostP2 : kAnalyticCostTb;
    const int rem = K - n, smax = opt_.temporal, smin = mode_ == Mode::kDeepTb ? 2 : 1;
    std::vector<double> best(static_cast<size_t>(rem + 1), 1e300);
    std::vector<int> take(static_cast<size_t>(rem + 1), 1);
    best[0] = 0.0;
    for (int r = 1; r <= rem; ++r)
      for (int st = smin; st <= std::min(smax, r); ++st) {
        const double c = best[static_cast<size_t>(r - st)] + st * kStepCost[st];
        if (c < best[static_cast<size_t>(r)]) {
          best[static_cast<size_t>(r)] = c;
          take[static_cast<size_t>(r)] = st;
        }
      }
    if (analytic_) {
      // the analytic first pass takes 2..temporal steps: minimise its cost plus the best split of the rest
      int bf = 2;
      double bc = 1e300;
      for (int f = 2; f <= std::min(smax, rem); ++f) {
        const double c = f * kAnalyticCost[f] + best[static_cast<size_t>(rem - f)];
        if (c < bc) {
          bc = c;
          bf = f;
        }
      }
      units_.push_back(Unit{n, bf, true});
      n += bf;
    }
    W3D_REQUIRE(best[static_cast<size_t>(K - n)] < 1e299, "no pass schedule for the remaining steps");
    for (int r = K - n; r > 0; r -= take[static_cast<size_t>(r)]) {
      units_.push_back(Unit{n, take[static_cast<size_t>(r)]});
      n += take[static_cast<size_t>(r)];
    }
  } else if (mode_ == Mode::kFusedSingle) {
    while (n <= K - 1) {
      const bool f = n + 2 <= K && !is_check_[static_cast<size_t>(n + 1)];
      units_.push_back(Unit{n, f ? 2 : 1});
      n += f ? 2 : 1;
    }
  } else if (mode_ == Mode::kDeep) {
    for (; n <= K - 1; n += 2) units_.push_back(Unit{n, 2});
  } else {
    for (; n <= K - 1; ++n) units_.push_back(Unit{n, 1});
  }
}

void GpuSolver::build_msgs(int i) {
  msgs_.clear();
  if (block_tb_) {
    // one packed message per neighbour (faces, edges, corners): u^{n+S} s deep, then u^{n+S−1} s − 1 deep
    deep_s_ = units_[static_cast<size_t>(i) + 1].steps;
    for (const DeepPeer& q : deep_[deep_s_].peers)
      msgs_.push_back(Msg{q.peer, 0, send_buf_ + sbase_[deep_s_] + q.buf_off, recv_buf_ + q.buf_off, q.count});
    return;
  }
  if (mode_ == Mode::kDeepTb) {
    // the next pass of s steps reads u^{n+S} (this pass's out2) on s ghost planes and u^{n+S−1} (out1) on s − 1
    const i64 s = units_[static_cast<size_t>(i) + 1].steps, P = lay_.plane, nx = lay_.nx;
    double* out1 = u_[uf_[0]];
    double* out2 = u_[uf_[1]];
    // (ghost_bits: the pass stored u^{n+S−1} on the first ghost plane itself; that part then starts one plane further
    // from the face on both ends: our planes 1..s−2 / nx−s+1..nx−2 into the peer's ghosts at distance 2..s−1)
    const int gb = ghost_bits(i);
    for (const Face& f : plan_.faces) {
      W3D_REQUIRE(f.axis == 0, "deep-tb mode is slab-only");
      const i64 g = (gb >> f.side) & 1, d1 = s - 1 - g;
      const i64 s2 = f.side == 0 ? 0 : nx - s, s1 = f.side == 0 ? g : nx - (s - 1);
      const i64 r2 = f.side == 0 ? -s : nx, r1 = f.side == 0 ? -(s - 1) : nx + g;
      msgs_.push_back(Msg{f.peer, 0, out2 + lay_.plane_off(s2), out2 + lay_.plane_off(r2), s * P});
      if (d1 > 0) msgs_.push_back(Msg{f.peer, 1, out1 + lay_.plane_off(s1), out1 + lay_.plane_off(r1), d1 * P});
    }
    return;
  }
  if (mode_ == Mode::kDeep) {
    // after a fused pass the next one needs u^{n+2} on 2 ghost planes and u^{n+1} on 1 (x faces of a slab rank)
    double* out1 = u_[uf_[0]];
    double* out2 = u_[uf_[1]];
    const i64 P = lay_.plane, nx = lay_.nx;
    for (const Face& f : plan_.faces) {
      W3D_REQUIRE(f.axis == 0, "deep-halo mode is slab-only");
      if (f.side == 0) {
        msgs_.push_back(Msg{f.peer, 0, out2 + lay_.plane_off(0), out2 + lay_.plane_off(-2), 2 * P});
        msgs_.push_back(Msg{f.peer, 1, out1 + lay_.plane_off(0), out1 + lay_.plane_off(-1), P});
      } else {
        msgs_.push_back(Msg{f.peer, 0, out2 + lay_.plane_off(nx - 2), out2 + lay_.plane_off(nx), 2 * P});
        msgs_.push_back(Msg{f.peer, 1, out1 + lay_.plane_off(nx - 1), out1 + lay_.plane_off(nx), P});
      }
    }
    return;
  }
  double* field = post_exchange() ? u_[old_] : u_[cur_];
  for (const Face& f : plan_.faces) {
    const double* sp = f.contiguous ? field + f.send_off : send_buf_ + f.pack_off;
    double* rp = f.contiguous ? field + f.recv_off : recv_buf_ + f.pack_off;
    msgs_.push_back(Msg{f.peer, 0, sp, rp, f.count});
  }
}

void GpuSolver::phase_init() {
  const int K = prob_.K;
  const double* s = d_s_ + 1;
  is_check_.assign(static_cast<size_t>(K + 1), 0);
  for (int n : check_steps()) is_check_[static_cast<size_t>(n)] = 1;
  cur_unit_ = -1;
  ev_next_ = 0;
  marks_.clear();
  // (the log's checked entries are rewritten by every solve and the others stay 0 from the allocation: cleared only
  // where something else writes into it — the copy-engine and push waits report their status there — or a resumed
  // solve leaves the entries below its start alone)
  if (sdma_ || push_ || resume_n_ > 0)
    W3D_HIP(hipMemsetAsync(errlog_, 0, static_cast<size_t>(K + 1) * sizeof(Partial), s0_));
  if (push_) {
    W3D_HIP(hipMemsetAsync(flags_ + 8, 0, sizeof(unsigned), s0_));  // workgroups done (the passes' signal counter)
    // (in-process group only: there every rank's init precedes every pass, so no neighbour has written yet)
    if (opt_.poison_ghosts && loopback_) {
      W3D_HIP(hipMemsetAsync(stg_, 0xFF, static_cast<size_t>(8 * lay_.xg * lay_.plane) * sizeof(double), s0_));
      // ... except each staging plane's zero slot (Layout::zero_off), which positions outside the global interior load
      const size_t pb = static_cast<size_t>(lay_.plane) * sizeof(double);
      W3D_HIP(hipMemset2DAsync(stg_ + lay_.zero_off(), pb, 0, sizeof(double), static_cast<size_t>(8 * lay_.xg), s0_));
    }
  }
  // one rank on the LDS kernel: the first pass starts from the analytic u⁰, u¹ itself (no init kernel, no reads)
  analytic_ = (mode_ == Mode::kFusedSingle || mode_ == Mode::kDeepTb) && analytic_ok() && resume_n_ == 0;
  if (resume_n_ > 0) {  // loaded state: u^{n0−1} → buf 0, u^{n0} → buf 1 (ghosts included)
    const size_t bytes = static_cast<size_t>(lay_.bytes());
    timed(kPhaseInit, s0_, [&] {
      W3D_HIP(hipMemcpyAsync(u_[0], resume_[0].data(), bytes, hipMemcpyHostToDevice, s0_));
      W3D_HIP(hipMemcpyAsync(u_[1], resume_[1].data(), bytes, hipMemcpyHostToDevice, s0_));
    });
    start_n_ = resume_n_;
  } else if (analytic_) {
    start_n_ = 1;
  } else if (opt_.init2 && K >= 2) {
    // u¹ -> buf 0, u² -> buf 1 analytically (no read pass), ghosts included; the first leapfrog step is n = 2
    timed(kPhaseInit, s0_, [&] {
      launch_init_two(lay_, coef_, s, u_[0], u_[1], ct_[2], is_check_[2] ? partials_ : nullptr, s0_);
    });
    timed(kPhaseCheck, s0_, [&] {
      if (is_check_[2]) launch_reduce(partials_, init_two_partials(lay_), errlog_ + 2, s0_);
      if (is_check_[1]) {
        launch_error(lay_, u_[0], full_, s, ct_[1], partials_, s0_);
        launch_reduce(partials_, error_blocks(lay_, full_), errlog_ + 1, s0_);
      }
    });
    start_n_ = 2;
  } else {
    timed(kPhaseInit, s0_, [&] { launch_init_first(lay_, coef_, s, u_[0], u_[1], s0_); });
    timed(kPhaseCheck, s0_, [&] {
      if (is_check_[1]) {
        launch_error(lay_, u_[1], full_, s, ct_[1], partials_, s0_);
        launch_reduce(partials_, error_blocks(lay_, full_), errlog_ + 1, s0_);
      }
    });
    start_n_ = 1;
  }
  cur_ = 1;
  old_ = 0;
  build_units();
  if (push_) {  // every pass's push parameters, in device memory before the first pass reads them
    const int npass = static_cast<int>(units_.size());
    W3D_REQUIRE(npass <= prob_.K, "push: more passes than steps");
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    W3D_HIP(hipStreamIsCapturing(s0_, &cs));
    push_tab_ = push_host_ + (cs == hipStreamCaptureStatusActive ? 0 : prob_.K);
    for (int j = 1; j <= npass; ++j) push_tab_[j - 1] = make_push(j, npass);
    W3D_HIP(hipMemcpyAsync(push_dev_, push_tab_, static_cast<size_t>(npass) * sizeof(TbPush), hipMemcpyHostToDevice,
                           s0_));
  }
}

void GpuSolver::unit_shell(int i) {
  cur_unit_ = i;
  const Unit& u = units_[static_cast<size_t>(i)];
  if (u.fused()) {
    int k = 0;
    for (int b = 0; b < 4; ++b)
      if (b != cur_ && b != old_) uf_[k++] = b;
  }
  const int nc = u.n + u.steps;
  const bool chk = is_check_[static_cast<size_t>(nc)] != 0;
  if (mode_ == Mode::kDeep) {
    int off = 0;
    for (size_t k = 0; k < dshell_.size(); ++k) {
      timed(kPhaseShell, s0_, [&] {
        launch_leapfrog2(lay_, coef_, u_[old_], u_[cur_], u_[uf_[0]], u_[uf_[1]], dshell_[k], d_s_ + 1,
                         ct_[static_cast<size_t>(nc)], chk ? partials_ + off : nullptr, opt_.tiling2, s0_, sx0_, sx1_);
      });
      off += n_dshell_[k];
    }
  } else if (mode_ == Mode::kDeepTb) {
    // the regions the neighbours receive (tb_shells) first, on the side stream, CONCURRENTLY with the interior pass
    // that unit_interior launches on s0 (same inputs, disjoint outputs): the shells' partial last waves leave CUs the
    // interior fills, and the exchange follows the shells on the same side stream (no wait between sibling streams)
    tb_slots_ = 0;
    if (needs_exchange(i) && !late_exchange()) {
      build_msgs(i);
      hipStream_t xs = xstream();
      if (opt_.shells_concurrent) {
        capture::record(ev_shell_, s0_);  // (the unit's inputs are ready: fork)
        capture::wait(xs, ev_shell_);
        for (const LBox& b : tb_shells(i)) tb_pass(u, b, kPhaseShell, xs);
      } else {
        // (serial: the shells own the GPU and finish first, so the exchange starts as early as possible; all of them
        // in one pair-tiled launch where that applies — each alone left CUs idle, profiles/r6/)
        const std::vector<LBox> sh = tb_shells(i);
        if (!tb_pass_boxes(u, sh, kPhaseShell, s0_))
          for (const LBox& b : sh) tb_pass(u, b, kPhaseShell, s0_);
        capture::record(ev_shell_, s0_);
        capture::wait(xs, ev_shell_);
      }
      return;
    }
  } else if (mode_ == Mode::kSingleStep && split()) {
    timed(kPhaseShell, s0_, [&] {
      launch_leapfrog(lay_, coef_, u_[cur_], u_[old_], shell_.data(), static_cast<int>(shell_.size()), d_s_ + 1,
                      ct_[static_cast<size_t>(nc)], chk ? partials_ : nullptr, opt_.tiling, s0_);
    });
  }
  if (needs_exchange(i)) {
    build_msgs(i);
    capture::record(ev_shell_, s0_);
  }
}

const GpuSolver::Msg& GpuSolver::peer_msg(const Msg& m, const std::vector<GpuSolver*>& ranks) const {
  const GpuSolver* q = ranks[static_cast<size_t>(m.peer)];
  const Msg* g = nullptr;
  for (const Msg& h : q->msgs_)
    if (h.peer == rank_ && h.tag == m.tag) g = &h;
  W3D_REQUIRE(g && g->count == m.count, "group exchange: mismatched messages");
  return *g;
}

bool GpuSolver::packs() const { return (mode_ == Mode::kSingleStep && plan_.packed_doubles > 0) || block_tb_; }

void GpuSolver::pack_halo(hipStream_t st) {
  if (block_tb_)
    launch_box_copy(lay_, pack_tab_[deep_s_], 0, u_[uf_[1]], u_[uf_[0]], send_buf_ + sbase_[deep_s_], st);
  else if (mode_ == Mode::kSingleStep && plan_.packed_doubles > 0)
    launch_pack(lay_, plan_, post_exchange() ? u_[old_] : u_[cur_], send_buf_, st);
}

void GpuSolver::unpack_halo(hipStream_t st) {
  if (block_tb_)
    launch_box_copy(lay_, unpack_tab_[deep_s_], 1, u_[uf_[1]], u_[uf_[0]], recv_buf_, st);
  else if (mode_ == Mode::kSingleStep && plan_.packed_doubles > 0)
    launch_unpack(lay_, plan_, recv_buf_, post_exchange() ? u_[old_] : u_[cur_], st);
}

void GpuSolver::exchange(hipStream_t st, const std::vector<GpuSolver*>* pull) {
  const bool packed = packs();
  if (packed && !pull) pack_halo(st);  // (group: each rank packed its own faces)
  if (opt_.fake_comm && opt_.fake_traffic && comm_) {
    // perf study: the rank's real message set, sent to and received from itself over a
    // one-rank communicator — RCCL's copy kernels, CU and LDS use and bytes as in the real exchange
    ncclComm_t c = static_cast<ncclComm_t>(comm_->raw());
    W3D_NCCL(ncclGroupStart());
    for (const Msg& m : msgs_) {
      W3D_NCCL(ncclSend(m.send, static_cast<size_t>(m.count), ncclFloat64, 0, c, st));
      W3D_NCCL(ncclRecv(m.recv, static_cast<size_t>(m.count), ncclFloat64, 0, c, st));
    }
    W3D_NCCL(ncclGroupEnd());
  } else if (!opt_.fake_comm) {  // fake_comm (perf study): one rank's schedule timed alone, ghosts keep stale values
    ncclComm_t c = static_cast<ncclComm_t>(comm_->raw());
    W3D_NCCL(ncclGroupStart());
    for (const Msg& m : msgs_) {
      if (pull) {  // one-rank communicator: the k-th send to self pairs with the k-th receive from self
        const Msg& g = peer_msg(m, *pull);
        W3D_NCCL(ncclSend(g.send, static_cast<size_t>(m.count), ncclFloat64, 0, c, st));
        W3D_NCCL(ncclRecv(m.recv, static_cast<size_t>(m.count), ncclFloat64, 0, c, st));
      } else {
        W3D_NCCL(ncclSend(m.send, static_cast<size_t>(m.count), ncclFloat64, m.peer, c, st));
        W3D_NCCL(ncclRecv(m.recv, static_cast<size_t>(m.count), ncclFloat64, m.peer, c, st));
      }
    }
    W3D_NCCL(ncclGroupEnd());
  }
  if (packed) unpack_halo(st);
}

void GpuSolver::unit_exchange_rccl(int i) {
  if (!needs_exchange(i)) return;
  hipStream_t xs = xstream();
  // (deep-tb: the shells ran on xs itself, after its wait for the unit's inputs)
  if (xs != s0_ && mode_ != Mode::kDeepTb) capture::wait(xs, ev_shell_);
  if (opt_.poison_ghosts) poison(xs);
  timed(kPhaseComm, xs, [&] { exchange(xs); });
  if (xs != s0_) capture::record(ev_halo_, xs);
}

// One LDS S-step pass of unit u over `box` on stream st (s0 unless given). Its checked levels' partials go to slot
// tb_slots_ of each level: one slot per level on one rank, up to kTbSlots on multi-rank ranks (the shell boxes, then
// the interior), reduced together after the interior.
void GpuSolver::tb_pass(const Unit& u, const LBox& box, int phase, hipStream_t st) {
  if (st == nullptr) st = s0_;
  LeapfrogTbTiling t = opt_.tiling_tb;
  t.stages = u.steps;
  t.ghost_x1 = ghost_bits(cur_unit_);
  double cts[5] = {0, 0, 0, 0, 0};
  int mask = 0;
  for (int k = 1; k <= u.steps; ++k) {
    cts[k - 1] = ct_[static_cast<size_t>(u.n + k)];
    if (is_check_[static_cast<size_t>(u.n + k)]) mask |= 1 << (k - 1);
  }
  const int slots = mode_ == Mode::kDeepTb ? kTbSlots : 1;
  W3D_REQUIRE(tb_slots_ < slots, "leapfrog_tb: too many launches in one unit");
  Partial* part = mask ? tb_partials_ + tb_region_ * (kTbLevels * slots * n_tb_) + tb_slots_ * n_tb_ : nullptr;
  const LBox real = mode_ == Mode::kDeepTb ? sreal_ : tb_default_real();
  // push transport: this pass's parameters (make_push) from the table phase_init uploaded; the command-processor
  // waits (push_cp_wait) are stream operations issued here, before the launch
  const TbPush* qh = nullptr;
  const TbPush* qd = nullptr;
  if (push_) {
    const int j = cur_unit_ + 1;
    qh = push_tab_ + (j - 1);
    qd = push_dev_ + (j - 1);
    if (opt_.push_cp_wait)
      for (int side = 0; side < 2; ++side)
        if (qh->wait_side[side] && qh->cp_wait > 0)
          W3D_HIP(hipStreamWaitValue32(s0_, flags_ + side, qh->cp_wait, hipStreamWaitValueGte, 0xFFFFFFFFu));
  }
  // fused z-face pack of the exchange that follows this unit (its depth: deep_s_, set by build_msgs before the passes)
  const bool pk = pk_dev_ != nullptr && needs_exchange(cur_unit_) && pk_host_[deep_s_].w == deep_s_;
  timed(phase, st, [&] {
    // (every launch fills its whole slot of n_tb_ partials: shell and interior boxes may have fewer x chunks)
    launch_leapfrog_tb(lay_, coef_, u_[old_], u_[cur_], u_[uf_[0]], u_[uf_[1]], box, d_s_ + 1, cts, mask, part, t,
                       st, real, u.analytic, slots * n_tb_, n_tb_, qh, qd, pk ? &pk_host_[deep_s_] : nullptr,
                       pk ? pk_dev_ + deep_s_ : nullptr);
  });
  if (mask) ++tb_slots_;
}

bool GpuSolver::tb_pass_boxes(const Unit& u, const std::vector<LBox>& boxes, int phase, hipStream_t st) {
  if (boxes.size() < 2 || boxes.size() > static_cast<size_t>(kP2MaxBoxes) || !opt_.tiling_tb.p2 || push_ ||
      (pk_dev_ != nullptr && pk_host_[deep_s_].w == deep_s_) || (u.analytic && u.steps > 4))
    return false;
  // (only where the shells' tiles alone do not fill the GPU: a 2048³ block rank's x-slab shell has 961 tiles of 5
  // planes beside 63 border tiles of 1024 — one grid then runs no faster than three, and measured slower)
  i64 tiles = 0;
  for (const LBox& b : boxes) {
    if (!leapfrog_p2_supported(lay_, b, u.steps)) return false;
    tiles += ceil_div(imax(0, b.y1 - b.y0), kTbTile) * ceil_div(imax(0, b.z1 - b.z0), kTbTile);
  }
  if (tiles > opt_.tiling_tb.target_blocks) return false;
  LeapfrogTbTiling t = opt_.tiling_tb;
  t.stages = u.steps;
  // (no XCD remap: the boxes' workgroups differ in length, and a contiguous logical range per XCD put the long ones
  // on a few XCDs; dispatch order deals consecutive workgroups to the XCDs round-robin)
  t.xcd_remap = false;
  t.ghost_x1 = ghost_bits(cur_unit_);
  double cts[5] = {0, 0, 0, 0, 0};
  int mask = 0;
  for (int k = 1; k <= u.steps; ++k) {
    cts[k - 1] = ct_[static_cast<size_t>(u.n + k)];
    if (is_check_[static_cast<size_t>(u.n + k)]) mask |= 1 << (k - 1);
  }
  const int slots = mode_ == Mode::kDeepTb ? kTbSlots : 1;
  W3D_REQUIRE(tb_slots_ < slots, "leapfrog_tb: too many launches in one unit");
  Partial* part = mask ? tb_partials_ + tb_region_ * (kTbLevels * slots * n_tb_) + tb_slots_ * n_tb_ : nullptr;
  const LBox real = mode_ == Mode::kDeepTb ? sreal_ : tb_default_real();
  timed(phase, st, [&] {
    launch_leapfrog_p2_boxes(lay_, coef_, u_[old_], u_[cur_], u_[uf_[0]], u_[uf_[1]], boxes.data(),
                             static_cast<int>(boxes.size()), d_s_ + 1, cts, mask, part, t, st, real, u.analytic,
                             slots * n_tb_, n_tb_);
  });
  if (mask) ++tb_slots_;
  return true;
}

// The shell / interior split of a deep-tb unit whose exchange overlaps the next part of the pass: cpu.hpp deep_split
// with w = the next pass's depth (its z cuts lie on whole pairs, so every box runs on the pair-tiled pass).
void GpuSolver::tb_split(int i, std::vector<LBox>& shells, LBox& interior) const {
  shells.clear();
  interior = full_;
  if (!needs_exchange(i) || late_exchange()) return;
  bool nb[3][2];
  for (int a = 0; a < 3; ++a)
    for (int sd = 0; sd < 2; ++sd) nb[a][sd] = neighbor_rank(dims_, rank_, a, sd) >= 0;
  deep_split(full_, nb, units_[static_cast<size_t>(i) + 1].steps, kTbTile, shells, interior);
  W3D_REQUIRE(static_cast<int>(shells.size()) < kTbSlots, "deep-tb: too many shell boxes");
}

std::vector<LBox> GpuSolver::tb_shells(int i) const {
  std::vector<LBox> s;
  LBox in;
  tb_split(i, s, in);
  return s;
}

LBox GpuSolver::tb_interior(int i) const {
  std::vector<LBox> s;
  LBox in;
  tb_split(i, s, in);
  return in;
}

void GpuSolver::unit_interior(int i) {
  const Unit& u = units_[static_cast<size_t>(i)];
  const int nc = u.n + u.steps;
  const bool chk = is_check_[static_cast<size_t>(nc)] != 0;
  const double ct = ct_[static_cast<size_t>(nc)];
  const double* s = d_s_ + 1;
  // (group ranks: lb_fence already put s0 behind every rank's pull, ev_halo_ included; a second, redundant wait on
  // the own side stream after that fence crashes HIP 7.2's hipStreamEndCapture — tools/probes/capture_probe2.hip flag 36)
  const bool wait = needs_exchange(i) && xstream() != s0_ && (!loopback_ || sdma_);
  int np = 0;  // partials to reduce
  bool joined = false;
  if (mode_ == Mode::kDeep) {
    int off = 0;
    for (int n : n_dshell_) off += n;
    if (!dint_.empty()) {
      timed(kPhaseCompute, s0_, [&] {
        launch_leapfrog2(lay_, coef_, u_[old_], u_[cur_], u_[uf_[0]], u_[uf_[1]], dint_, s, ct,
                         chk ? partials_ + off : nullptr, opt_.tiling2, s0_, sx0_, sx1_);
      });
    }
    np = off + n_dint_;
  } else if ((mode_ == Mode::kFusedSingle && opt_.tb && u.fused()) || mode_ == Mode::kDeepTb) {
    // S steps in one LDS pass (on slab ranks: the interior left between this unit's shells); every checked level
    // has its own block of partials
    if (mode_ != Mode::kDeepTb) tb_slots_ = 0;
    const LBox b = mode_ == Mode::kDeepTb ? tb_interior(i) : full_;
    if (!b.empty()) tb_pass(u, b, kPhaseCompute);
    // (the shells ran on the side stream: join it before the reductions read their partials)
    if (wait) {
      capture::wait(s0_, ev_halo_);
      joined = true;
    }
    const int slots = mode_ == Mode::kDeepTb ? kTbSlots : 1;
    if (tb_slots_ > 0) {
      Partial* region = tb_partials_ + tb_region_ * (kTbLevels * slots * n_tb_);
      for (int k = 1; k <= u.steps; ++k)
        if (is_check_[static_cast<size_t>(u.n + k)])
          pending_.push_back(ReduceJob{region + (k - 1) * slots * n_tb_, tb_slots_ * n_tb_, errlog_ + u.n + k});
      tb_region_ = (tb_region_ + 1) % kTbRegions;
      if (tb_region_ == 0 || opt_.timers) flush_reduces();  // the next unit reuses region 0 / per-unit check time
    }
  } else if (mode_ == Mode::kFusedSingle) {
    timed(kPhaseCompute, s0_, [&] {
      if (u.fused())
        launch_leapfrog2(lay_, coef_, u_[old_], u_[cur_], u_[uf_[0]], u_[uf_[1]], full_, s, ct,
                         chk ? partials_ : nullptr, opt_.tiling2, s0_);
      else
        launch_leapfrog(lay_, coef_, u_[cur_], u_[old_], &full_, 1, s, ct, chk ? partials_ : nullptr, opt_.tiling,
                        s0_);
    });
    np = u.fused() ? n_fused_ : n_full_;
  } else if (split()) {
    timed(kPhaseCompute, s0_, [&] {
      launch_leapfrog(lay_, coef_, u_[cur_], u_[old_], &interior_, 1, s, ct, chk ? partials_ + n_shell_ : nullptr,
                      opt_.tiling, s0_);
    });
    np = n_shell_ + n_int_;
  } else {
    timed(kPhaseCompute, s0_, [&] {
      launch_leapfrog(lay_, coef_, u_[cur_], u_[old_], &full_, 1, s, ct, chk ? partials_ : nullptr, opt_.tiling,
                      s0_);
    });
    np = n_full_;
  }
  if (wait && !joined) capture::wait(s0_, ev_halo_);
  if (chk && np > 0) timed(kPhaseCheck, s0_, [&] { launch_reduce(partials_, np, errlog_ + nc, s0_); });
  if (opt_.debug_sync) W3D_HIP(hipDeviceSynchronize());
  if (u.fused()) {
    old_ = uf_[0];
    cur_ = uf_[1];
  } else {
    std::swap(cur_, old_);
  }
  final_buf_ = cur_;
  prev_buf_ = old_;
}

void GpuSolver::flush_reduces() {
  if (pending_.empty()) return;
  timed(kPhaseCheck, s0_, [&] { launch_reduce_batch(pending_.data(), static_cast<int>(pending_.size()), s0_); });
  pending_.clear();
}

void GpuSolver::enqueue_solve() {
  if (sdma_) sdma_check_connected();
  phase_init();
  // copy-engine flag values are 16-bit unit indices under a parity bit (xval / xend): more units per solve would alias
  // the end-of-solve word and the other parity's range
  W3D_REQUIRE(!sdma_ || units_.size() < 0xFFFEu, "sdma transport: too many passes in one solve for the flag encoding");
  tb_region_ = 0;
  pending_.clear();
  const bool late = late_exchange();
  for (int i = 0; i < static_cast<int>(units_.size()); ++i) {
    if (sdma_) sdma_receive(i);
    unit_shell(i);
    if (!late) sdma_ ? unit_exchange_sdma(i) : unit_exchange_rccl(i);
    unit_interior(i);
    if (late) sdma_ ? unit_exchange_sdma(i) : unit_exchange_rccl(i);
  }
  flush_reduces();
  if (push_) push_finish(s0_);
  if (sdma_) sdma_finish();
  push_epoch_ += static_cast<int>(units_.size());
  final_buf_ = cur_;
  prev_buf_ = old_;
}

// Debug aid: fill the ghost regions that the next exchange must overwrite with NaN, so a halo that
// is not delivered shows up in the error norms at once instead of silently reusing stale values.
void GpuSolver::poison(hipStream_t st) {
  if (block_tb_) {  // the ghost regions themselves (the messages land in a staging buffer first)
    launch_box_copy(lay_, unpack_tab_[deep_s_], 2, u_[uf_[1]], u_[uf_[0]], nullptr, st);
    return;
  }
  for (const Msg& m : msgs_)
    W3D_HIP(hipMemsetAsync(m.recv, 0xFF, static_cast<size_t>(m.count) * sizeof(double), st));
}

void GpuSolver::collect_phases(RunResult& r) {
  if (!opt_.timers) return;
  double acc[kNumPhases] = {};
  r.trace.assign(units_.size(), UnitTrace{});
  for (size_t i = 0; i < units_.size(); ++i) {
    r.trace[i].unit = static_cast<int>(i);
    r.trace[i].n = units_[i].n;
    r.trace[i].steps = units_[i].steps;
  }
  for (const auto& m : marks_) {
    float ms = 0.0f;
    W3D_HIP(hipEventElapsedTime(&ms, m.b, m.e));
    acc[m.phase] += ms;
    if (m.unit < 0 || m.unit >= static_cast<int>(r.trace.size())) continue;
    UnitTrace& t = r.trace[static_cast<size_t>(m.unit)];
    (m.phase == kPhaseShell ? t.shell_ms : m.phase == kPhaseComm ? t.comm_ms : m.phase == kPhaseCheck ? t.check_ms
                                                                                                 : t.compute_ms) += ms;
  }
  r.phases.init_ms = acc[kPhaseInit];
  r.phases.shell_ms = acc[kPhaseShell];
  r.phases.interior_ms = acc[kPhaseCompute];
  r.phases.comm_ms = acc[kPhaseComm];
  r.phases.check_ms = acc[kPhaseCheck];
  r.phases.gather_ms = acc[kPhaseGather];  // device: the error log's all-gather and D2H copy after the last pass
}

// ------------------------------------------------------------------------------------------------------------------
// loopback transport (GpuGroup): P ranks in one process on one device, halos moved by device copies. Test-only
// stand-in for RCCL that exercises the identical schedules, shell/interior splits, message plans, pack/unpack and
// stream/event ordering of the production path on a single GPU (RCCL refuses two ranks on one device).
// ------------------------------------------------------------------------------------------------------------------
void GpuSolver::lb_pack(int i) {
  if (!needs_exchange(i)) return;
  hipStream_t xs = xstream();
  if (xs != s0_ && mode_ != Mode::kDeepTb) capture::wait(xs, ev_shell_);
  pack_halo(xs);
  capture::record(ev_packed_, xs);
}

void GpuSolver::lb_pull(int i, const std::vector<GpuSolver*>& ranks, hipEvent_t all_packed) {
  if (!needs_exchange(i)) return;
  hipStream_t xs = xstream();
  if (opt_.poison_ghosts) poison(xs);
  capture::wait(xs, all_packed);  // every peer's faces are packed
  if (comm_) {  // rccl-self: the production exchange (RCCL send/recv on xs) over this rank's one-rank communicator
    timed(kPhaseComm, xs, [&] { exchange(xs, &ranks); });
  } else {
    for (const Msg& m : msgs_) {
      const Msg& g = peer_msg(m, ranks);
      W3D_HIP(hipMemcpyAsync(m.recv, g.send, static_cast<size_t>(m.count) * sizeof(double), hipMemcpyDeviceToDevice,
                             xs));
    }
    unpack_halo(xs);
  }
  capture::record(ev_halo_, xs);
}

void GpuSolver::lb_fence(int i, hipEvent_t all_pulled) {
  // the peers have read this rank's send regions once their pulls are done: keep both streams behind them (the side
  // stream only when this schedule uses it: a captured stream that only ever waits trips HIP 7.2's end of capture)
  if (!needs_exchange(i)) return;
  capture::wait(s0_, all_pulled);
  if (xstream() != s0_) capture::wait(s1_, all_pulled);
}

void GpuSolver::gather_errors(RunResult& r) {
  const int K = prob_.K;
  const size_t per = static_cast<size_t>(K + 1);
  std::vector<Partial> host(per * static_cast<size_t>(world_));
  cur_unit_ = -1;
  timed(kPhaseGather, s0_, [&] {
    if (world_ > 1 && comm_ && !opt_.fake_comm) {  // (a fake rank's communicator is its own one-rank one)
      W3D_NCCL(ncclAllGather(errlog_, errall_, 2 * per, ncclFloat64, static_cast<ncclComm_t>(comm_->raw()), s0_));
      W3D_HIP(hipMemcpyAsync(host.data(), errall_, host.size() * sizeof(Partial), hipMemcpyDeviceToHost, s0_));
    } else {
      host.resize(per);
      W3D_HIP(hipMemcpyAsync(host.data(), errlog_, per * sizeof(Partial), hipMemcpyDeviceToHost, s0_));
    }
  });
  wait_stream(s0_, comm_.get(), gpu_timeout_s());
  push_check();
  decode_log(host.data(), static_cast<int>(host.size() / per), r);
}

void GpuSolver::decode_log(const Partial* host, int nsrc, RunResult& r) const {
  const size_t per = static_cast<size_t>(prob_.K + 1);
  // copy-engine transport: a flag wait that timed out marked word 0 of that rank's log (step 0 is never checked)
  for (int q = 0; q < nsrc && sdma_; ++q)
    W3D_REQUIRE(host[static_cast<size_t>(q) * per].x == 0.0,
                "sdma transport: a flag wait timed out on rank " + std::to_string(nsrc > 1 ? q : rank_) +
                    " (a neighbour stopped or its copies never arrived)");
  const double n_int = static_cast<double>(prob_.N - 1);
  const double denom = n_int * n_int * n_int;
  for (int n : check_steps()) {
    double m = 0.0, sum = 0.0;
    for (int q = 0; q < nsrc; ++q) {  // fixed rank order
      const Partial& v = host[static_cast<size_t>(q) * per + static_cast<size_t>(n)];
      m = v.x > m || std::isnan(v.x) ? v.x : m;
      sum += v.y;
    }
    r.steps.push_back(n);
    r.max_err.push_back(m);
    r.rms_err.push_back(std::sqrt(sum / denom));
    if (!std::isfinite(m) || !std::isfinite(sum)) r.finite = false;
  }
}

RunResult GpuSolver::run() {
  RunResult r;
  // RCCL ranks run their first solve eagerly: the peer connections (and RCCL's proxy threads) are set up at the
  // first send/recv, which must not happen inside a stream capture; the capture follows on the second run
  if (world_ > 1 && !multistream_capture_safe()) opt_.graph = false;
  const bool capture_ok = !(world_ > 1 && comm_) || runs_ >= 1;
  // (copy-engine ranks: the flag values of a solve depend on its parity, so there is one graph per parity)
  xpar_ = static_cast<int>(xsolves_ & 1);
  hipGraphExec_t& gx = sdma_ ? xgraph_[xpar_] : graph_exec_;
  if (opt_.graph && !gx && capture_ok && !opt_.timers && resume_n_ == 0) {
    // capture once (outside the timed region of later runs); fall back to eager launches if capture is refused
    hipGraph_t g = nullptr;
    bool ok = hipStreamBeginCapture(s0_, hipStreamCaptureModeThreadLocal) == hipSuccess;
    std::string thrown;
    if (ok) {
      capture::begin(s0_);  // (every cross-stream wait checked: wave3d/capture_guard.hpp)
      try {
        enqueue_solve();
        capture::finish();
      } catch (const std::exception& ex) {
        ok = false;
        thrown = ex.what();
        capture::close();
      }
      const hipError_t e = hipStreamEndCapture(s0_, &g);
      capture::abandon();
      ok = ok && e == hipSuccess && g != nullptr;
    }
    // (an error of the schedule itself is not a capture problem: report it instead of retrying eagerly on streams the
    // aborted capture may have left unusable)
    if (!thrown.empty()) {
      if (g) (void)hipGraphDestroy(g);
      fail("solve schedule failed while being captured: " + thrown);
    }
    if (ok) ok = hipGraphInstantiate(&gx, g, nullptr, nullptr, 0) == hipSuccess;
    // (upload now rather than at the first replay; the copy-engine runs still show one 9-12 ms solve among their first
    // 2-7 — never later — with or without it: profiles/r4/sdma_streams.md. bench.py warms copy-engine runs up longer)
    if (ok && hipGraphUpload(gx, s0_) != hipSuccess) {
      (void)hipGraphExecDestroy(gx);  // (instantiated but not uploadable: release it, run eagerly)
      ok = false;
    }
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    if (!ok) {
      gx = nullptr;
      opt_.graph = false;
    }
  }
  const double t0 = now_s();
  if (gx && opt_.graph && !opt_.timers && resume_n_ == 0)
    W3D_HIP(hipGraphLaunch(gx, s0_));
  else
    enqueue_solve();
  ++xsolves_;
  gather_errors(r);
  r.solve_s = now_s() - t0;
  collect_phases(r);
  ++runs_;
  return r;
}

std::vector<RunResult> GpuSolver::run_batch(int n) {
  std::vector<RunResult> out;
  if (n <= 0) return out;
  // Graph-captured solves are enqueued back to back, each followed by its error-log gather (RCCL ranks: the all-gather
  // run() issues, on the same stream), and the host synchronises once: no host round trip between solves. Every rank
  // enqueues the same sequence, so the collectives match. (Copy-engine and push ranks carry per-solve flag epochs and
  // host-side checks between solves: one run() each.)
  const bool gathered = world_ > 1 && comm_ && !opt_.fake_comm;
  const bool pipelined = !sdma_ && !push_ && opt_.graph && graph_exec_ && !opt_.timers && resume_n_ == 0 &&
                         (world_ == 1 || opt_.fake_comm || gathered);
  if (!pipelined) {
    for (int i = 0; i < n; ++i) out.push_back(run());
    return out;
  }
  const size_t per = static_cast<size_t>(prob_.K + 1);
  const int nsrc = gathered ? world_ : 1;
  const size_t slot = per * static_cast<size_t>(nsrc);
  if (hbatch_n_ < n * nsrc) {
    if (hbatch_) W3D_HIP(hipHostFree(hbatch_));
    hbatch_ = nullptr;
    W3D_HIP(hipHostMalloc(reinterpret_cast<void**>(&hbatch_), static_cast<size_t>(n) * slot * sizeof(Partial),
                          hipHostMallocDefault));
    hbatch_n_ = n * nsrc;
  }
  cur_unit_ = -1;
  const double t0 = now_s();
  for (int i = 0; i < n; ++i) {
    W3D_HIP(hipGraphLaunch(graph_exec_, s0_));
    // (stream order: this solve's log is gathered and copied out before the next replay's reductions overwrite it)
    if (gathered)
      W3D_NCCL(ncclAllGather(errlog_, errall_, 2 * per, ncclFloat64, static_cast<ncclComm_t>(comm_->raw()), s0_));
    W3D_HIP(hipMemcpyAsync(hbatch_ + static_cast<size_t>(i) * slot, gathered ? errall_ : errlog_,
                           slot * sizeof(Partial), hipMemcpyDeviceToHost, s0_));
  }
  // (the per-solve bound, per replay: a long timed block is not a hang)
  wait_stream(s0_, comm_.get(), gpu_timeout_s() * n);
  const double dt = (now_s() - t0) / n;
  xsolves_ += static_cast<unsigned>(n);
  runs_ += n;
  for (int i = 0; i < n; ++i) {
    RunResult r;
    decode_log(hbatch_ + static_cast<size_t>(i) * slot, nsrc, r);
    r.solve_s = dt;
    r.batched = true;
    out.push_back(std::move(r));
  }
  return out;
}

// ------------------------------------------------------------------------------------------------------------------
// push transport (slab LDS passes): peers, IPC, end of solve
// ------------------------------------------------------------------------------------------------------------------
// Pass j (1-based) of npass forwards its faces into the neighbours' staging of parity j % 2, reads its ghosts from its
// own staging of parity (j − 1) % 2 (pass 1: from the field, filled by the init / the loaded state), waits for both
// neighbours' pass j − 1 and signals its own. Epochs: in-kernel waits (graph-replayable) use the pass index j, every
// pass but the last signals (nobody waits for that one) and the flags are reset at the end of the solve, before its
// closing collective (which every multi-process run with in-kernel waits has: the error all-gather). Without a closing
// collective (push_no_collective) or with command-processor waits the epochs run on over the solves, every pass
// signals and pass 1 waits for the neighbours' last pass of the previous solve (no reset needed).
TbPush GpuSolver::make_push(int j, int npass) const {
  W3D_REQUIRE(peer_flags_[0] || !nb_lo_, "push transport: lower neighbour not connected");
  W3D_REQUIRE(peer_flags_[1] || !nb_hi_, "push transport: upper neighbour not connected");
  TbPush q;
  q.on = 1;
  q.faces_first = opt_.overlap ? 1 : 0;
  q.T = static_cast<int>(lay_.xg);
  q.nx = static_cast<int>(lay_.nx);
  q.flags = flags_;
  q.status = flags_ + 4;
  q.done = flags_ + 8;
  const bool mono = opt_.push_cp_wait || opt_.push_no_collective;
  const unsigned G = static_cast<unsigned>(mono ? push_epoch_ + j : j);
  const unsigned wait = mono ? G - 1 : (j > 1 ? G - 1 : 0u);
  q.wait_epoch = opt_.push_cp_wait ? 0u : wait;
  q.cp_wait = opt_.push_cp_wait ? wait : 0u;
  q.signal_epoch = (mono || j < npass) ? G : 0u;
  q.done_target = q.signal_epoch ? static_cast<unsigned>(j * n_tb_) : 0u;
  static const unsigned long long ticks = [] {
    int khz = 100000;
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
    return static_cast<unsigned long long>(std::min(gpu_timeout_s(), 60.0) * 1e3 * khz);
  }();
  q.spin_ticks = ticks;
  // (tag: unique per solver instance, rank, solve and pass, so a table entry left by another solver never matches)
  static unsigned instances = 0;
  if (push_uid_ == 0) push_uid_ = ++instances;
  // (disjoint fields: the pass index in the low 16 bits, the solve epoch in the high 16, XORed with a hash of the
  // instance and rank — distinct (epoch, pass) pairs never share a tag within 65536 epochs)
  q.tag = ((push_uid_ * 2654435761u) ^ (static_cast<unsigned>(rank_) * 40503u)) ^
          ((static_cast<unsigned>(push_epoch_) & 0xFFFFu) << 16) ^ (static_cast<unsigned>(j) & 0xFFFFu);
  const int par = j % 2, rpar = (j - 1) % 2;
  // (perf attribution of the transport with --fake-rank only: W3D_PUSH_ATTRIB=nofwd / noghost drop the forwarded
  // stores / the staging reads — the results are then wrong)
  const char* attrib = opt_.fake_comm ? std::getenv("W3D_PUSH_ATTRIB") : nullptr;
  const bool nofwd = attrib && std::strstr(attrib, "nofwd"), noghost = attrib && std::strstr(attrib, "noghost");
  if (attrib && std::strstr(attrib, "noacq")) q.acquire = 0;
  if (attrib && std::strstr(attrib, "nosync")) q.wait_epoch = q.signal_epoch = q.done_target = 0;
  for (int side = 0; side < 2; ++side) {
    if (!(side == 0 ? nb_lo_ : nb_hi_)) continue;
    q.fwd1[side] = nofwd ? nullptr : peer_stg_[side] + stg_off(par, 0, 1 - side);  // the neighbour's ghosts facing us
    q.fwd2[side] = nofwd ? nullptr : peer_stg_[side] + stg_off(par, 1, 1 - side);
    if (j > 1 && !noghost) {
      q.gprev[side] = stg_ + stg_off(rpar, 0, side);
      q.gcur[side] = stg_ + stg_off(rpar, 1, side);
    }
    q.rflag[side] = peer_flags_[side] + (1 - side);  // our slot in the neighbour's flags
    q.wait_side[side] = 1;
  }
  return q;
}

std::string GpuSolver::push_handles() const {
  W3D_REQUIRE(push_, "push_handles: this solver does not use the push transport");
  hipIpcMemHandle_t h[2];
  W3D_HIP(hipIpcGetMemHandle(&h[0], stg_));
  W3D_HIP(hipIpcGetMemHandle(&h[1], flags_));
  int dv[2] = {0, 0};  // this rank's device and the visible device count (peer-access check on the other side)
  W3D_HIP(hipGetDevice(&dv[0]));
  W3D_HIP(hipGetDeviceCount(&dv[1]));
  return std::string(reinterpret_cast<const char*>(h), sizeof h) + std::string(reinterpret_cast<const char*>(dv), sizeof dv);
}

void GpuSolver::connect_push_peer(int side, double* stg, unsigned* flags, bool ipc) {
  peer_stg_[side] = stg;
  peer_flags_[side] = flags;
  peer_ipc_[side] = ipc;
}

void GpuSolver::connect_push(const std::vector<std::string>& all) {
  W3D_REQUIRE(push_, "connect_push: this solver does not use the push transport");
  W3D_REQUIRE(static_cast<int>(all.size()) == world_, "connect_push: one handle set per rank expected");
  for (int side = 0; side < 2; ++side) {
    const int peer = neighbor_rank(dims_, rank_, 0, side);
    if (peer < 0) continue;
    const std::string& b = all[static_cast<size_t>(peer)];
    hipIpcMemHandle_t h[2];
    int dv[2] = {0, 0};
    W3D_REQUIRE(b.size() == sizeof h + sizeof dv, "connect_push: bad handle size from rank " + std::to_string(peer));
    std::memcpy(h, b.data(), sizeof h);
    std::memcpy(dv, b.data() + sizeof h, sizeof dv);
    // a neighbour on another GPU must be reachable by this GPU's stores (xGMI peer access), else the passes would
    // fault: refuse here, where the autotune can still drop the candidate
    int me = 0, nd = 0;
    W3D_HIP(hipGetDevice(&me));
    W3D_HIP(hipGetDeviceCount(&nd));
    if (dv[1] == nd && dv[0] != me) {
      int can = 0;
      W3D_HIP(hipDeviceCanAccessPeer(&can, me, dv[0]));
      W3D_REQUIRE(can, "push transport: GPU " + std::to_string(me) + " cannot access peer GPU " + std::to_string(dv[0]));
    }
    void* stg = nullptr;
    void* fl = nullptr;
    W3D_HIP(hipIpcOpenMemHandle(&stg, h[0], hipIpcMemLazyEnablePeerAccess));
    W3D_HIP(hipIpcOpenMemHandle(&fl, h[1], hipIpcMemLazyEnablePeerAccess));
    connect_push_peer(side, static_cast<double*>(stg), static_cast<unsigned*>(fl), true);
  }
}

void GpuSolver::connect_push_self() {
  W3D_REQUIRE(push_, "connect_push_self: this solver does not use the push transport");
  for (int side = 0; side < 2; ++side)
    // (the signal raises peer_flags_[side] + (1 − side): aim it at flags_[side], the slot this side waits on)
    if (neighbor_rank(dims_, rank_, 0, side) >= 0) connect_push_peer(side, stg_, flags_ + (2 * side - 1), false);
}

// After the last pass of a solve (which waited for both neighbours' last signals, the final values of this solve's
// flags) the flags go back to 0, before this rank's end-of-solve collective: no neighbour can signal the next solve's
// first pass before that collective has completed everywhere.
void GpuSolver::push_finish(hipStream_t st) {
  if (!opt_.push_cp_wait && !opt_.push_no_collective) W3D_HIP(hipMemsetAsync(flags_, 0, 2 * sizeof(unsigned), st));
}

void GpuSolver::push_check() {
  if (!push_) return;
  unsigned st = 0;
  W3D_HIP(hipMemcpy(&st, flags_ + 4, sizeof st, hipMemcpyDeviceToHost));
  W3D_REQUIRE(st != 2, "push transport: a pass read a stale parameter table (rank " + std::to_string(rank_) + ")");
  W3D_REQUIRE(st == 0, "push transport: a pass timed out waiting for a neighbour's signal (rank " +
                           std::to_string(rank_) + ")");
}

std::vector<double> GpuSolver::download(int which) const {
  std::vector<double> h(static_cast<size_t>(lay_.total));
  const double* src = u_[which == 0 ? final_buf_ : prev_buf_];
  int cur = 0;
  W3D_HIP(hipGetDevice(&cur));
  W3D_HIP(hipSetDevice(dev_));
  W3D_HIP(hipDeviceSynchronize());
  W3D_HIP(hipMemcpy(h.data(), src, h.size() * sizeof(double), hipMemcpyDeviceToHost));
  W3D_HIP(hipSetDevice(cur));
  return h;
}

unsigned long long GpuSolver::field_hash(int which) const {
  int cur = 0;
  W3D_HIP(hipGetDevice(&cur));
  W3D_HIP(hipSetDevice(dev_));
  W3D_HIP(hipDeviceSynchronize());
  unsigned long long* d = nullptr;
  W3D_HIP(hipMalloc(&d, sizeof(unsigned long long)));
  W3D_HIP(hipMemset(d, 0, sizeof(unsigned long long)));
  launch_field_hash(lay_, u_[which == 0 ? final_buf_ : prev_buf_], d, nullptr);
  unsigned long long h = 0;
  W3D_HIP(hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost));
  W3D_HIP(hipFree(d));
  W3D_HIP(hipSetDevice(cur));
  return h;
}

}  // namespace wave3d

namespace wave3d {

double comm_allreduce(const Comm& c, double v, bool max_op) {
  static thread_local hipStream_t st = nullptr;
  static thread_local double* buf = nullptr;
  if (!st) {
    W3D_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    W3D_HIP(hipMalloc(&buf, sizeof(double)));
  }
  W3D_HIP(hipMemcpyAsync(buf, &v, sizeof(double), hipMemcpyHostToDevice, st));
  W3D_NCCL(ncclAllReduce(buf, buf, 1, ncclFloat64, max_op ? ncclMax : ncclSum, static_cast<ncclComm_t>(c.raw()), st));
  double out = 0.0;
  W3D_HIP(hipMemcpyAsync(&out, buf, sizeof(double), hipMemcpyDeviceToHost, st));
  wait_stream(st, &c, gpu_timeout_s());
  return out;
}

void comm_barrier(const Comm& c) { (void)comm_allreduce(c, 0.0, false); }

std::vector<std::string> comm_allgather_bytes(const Comm& c, const std::string& mine) {
  const size_t n = mine.size(), w = static_cast<size_t>(c.world());
  hipStream_t st = nullptr;
  W3D_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  char* d = nullptr;
  W3D_HIP(hipMalloc(&d, n * (w + 1)));
  std::string all(n * w, '\0');
  W3D_HIP(hipMemcpyAsync(d, mine.data(), n, hipMemcpyHostToDevice, st));
  W3D_NCCL(ncclAllGather(d, d + n, n, ncclChar, static_cast<ncclComm_t>(c.raw()), st));
  W3D_HIP(hipMemcpyAsync(all.data(), d + n, n * w, hipMemcpyDeviceToHost, st));
  wait_stream(st, &c, gpu_timeout_s());
  (void)hipFree(d);
  (void)hipStreamDestroy(st);
  std::vector<std::string> v;
  for (size_t r = 0; r < w; ++r) v.push_back(all.substr(r * n, n));
  return v;
}

int rccl_version() {
  int v = 0;
  (void)ncclGetVersion(&v);
  return v;
}

}  // namespace wave3d

namespace wave3d {

GpuGroup::GpuGroup(const Problem& prob, const SolverOptions& opt, int world, const std::string& transport)
    : transport_(transport) {
  W3D_REQUIRE(world >= 1, "world must be >= 1");
  W3D_REQUIRE(transport == "loopback" || transport == "rccl-self" || transport == "push" || transport == "sdma" ||
                  transport == "multi-device",
              "group transport must be loopback, rccl-self, push, sdma or multi-device, not " + transport);
  SolverOptions o = opt;
  if (transport == "multi-device") {
    // one rank per visible device, each with its rank of one communicator; the production GpuSolver (not a group
    // member): its own graph, RCCL exchanges and error-log all-gather; opt.sdma selects the copy engines between the
    // devices (peer pointers, peer access enabled), else RCCL
    multi_ = true;
    int ndev = 0, dev0 = 0;
    W3D_HIP(hipGetDeviceCount(&ndev));
    W3D_HIP(hipGetDevice(&dev0));
    W3D_REQUIRE(world <= ndev, "multi-device group: " + std::to_string(world) + " ranks but " + std::to_string(ndev) +
                                   " visible GPU(s)");
    const auto comms = Comm::init_all(world);
    for (int r = 0; r < world; ++r) {
      W3D_HIP(hipSetDevice(r));
      for (int q = 0; q < world && o.sdma; ++q)
        if (q != r) {
          int can = 0;
          W3D_HIP(hipDeviceCanAccessPeer(&can, r, q));
          W3D_REQUIRE(can, "multi-device sdma: GPU " + std::to_string(r) + " cannot access GPU " + std::to_string(q));
          const hipError_t e = hipDeviceEnablePeerAccess(q, 0);
          if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) W3D_HIP(e);
          (void)hipGetLastError();
        }
      ranks_.push_back(std::make_unique<GpuSolver>(prob, o, r, world, comms[static_cast<size_t>(r)], false));
    }
    if (o.sdma && world > 1)
      for (auto& sp : ranks_)
        for (GpuSolver::XLink& l : sp->xlinks_) {
          GpuSolver* q = ranks_[static_cast<size_t>(l.peer)].get();
          l.flags = q->xflags_;
          for (int b = 0; b < q->nbuf_; ++b) l.u[b] = q->u_[b];
          l.recv = q->recv_buf_;
        }
    W3D_HIP(hipSetDevice(dev0));
    return;
  }
  o.push = transport == "push";
  o.sdma = transport == "sdma";
  for (int r = 0; r < world; ++r) {
    std::shared_ptr<Comm> c;
    if (transport == "rccl-self") c = std::make_shared<Comm>(0, 1, Comm::make_unique_id());
    ranks_.push_back(std::make_unique<GpuSolver>(prob, o, r, world, c, true));
  }
  if (o.push && world > 1) {
    // the ranks' passes wait for each other in the kernel: on ONE GPU they must not run concurrently (a waiting pass
    // could hold every CU while the pass it waits for cannot start), so every rank launches on rank 0's compute stream
    // in schedule order (rank 0 unit i, rank 1 unit i, ...) and each wait is already satisfied when it is reached.
    // The data path (forwarded faces in the neighbours' staging, ghosts read from the own staging, flags, counters,
    // epochs, flag reset) is the multi-process one; peers are the other ranks' buffers instead of IPC mappings.
    for (int r = 0; r < world; ++r) {
      GpuSolver* s = ranks_[static_cast<size_t>(r)].get();
      W3D_REQUIRE(s->push_, "push group: every rank must run the slab LDS passes (deep-tb)");
      if (r > 0) {
        (void)hipStreamDestroy(s->s0_);
        s->s0_ = ranks_[0]->s0_;
        s->own_s0_ = false;
      }
      for (int side = 0; side < 2; ++side) {
        const int peer = neighbor_rank(s->dims_, r, 0, side);
        if (peer < 0) continue;
        GpuSolver* q = ranks_[static_cast<size_t>(peer)].get();
        s->connect_push_peer(side, q->stg_, q->flags_, false);
      }
    }
  }
  if (o.sdma && world > 1) {
    // copy-engine ranks in one process: every link points at the peer rank's own buffers and flag words (no IPC)
    for (auto& sp : ranks_) {
      GpuSolver* s = sp.get();
      W3D_REQUIRE(s->sdma_, "sdma group: every rank must run the LDS multi-step passes (deep-tb)");
      for (GpuSolver::XLink& l : s->xlinks_) {
        GpuSolver* q = ranks_[static_cast<size_t>(l.peer)].get();
        l.flags = q->xflags_;
        for (int b = 0; b < q->nbuf_; ++b) l.u[b] = q->u_[b];
        l.recv = q->recv_buf_;
      }
    }
  }
  // (sdma: the flag waits of one rank's stream are released by other ranks' streams, so the group enqueues eagerly in
  // an order where every wait is issued after the write it waits for — see enqueue)
  graph_ = opt.graph && !opt.timers && !opt.debug_sync && (world == 1 || multistream_capture_safe()) && !o.sdma;
  W3D_HIP(hipStreamCreateWithFlags(&gs_, hipStreamNonBlocking));
  W3D_HIP(hipEventCreateWithFlags(&fork_, hipEventDisableTiming));
  W3D_HIP(hipEventCreateWithFlags(&all_packed_, hipEventDisableTiming));
  W3D_HIP(hipEventCreateWithFlags(&all_pulled_, hipEventDisableTiming));
  join_.resize(2 * static_cast<size_t>(world));
  for (hipEvent_t& e : join_) W3D_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
}

GpuGroup::~GpuGroup() {
  if (multi_) {  // (each rank's resources on its own device)
    for (auto& r : ranks_) {
      (void)hipSetDevice(r->device());
      r.reset();
    }
    return;
  }
  if (exec_) (void)hipGraphExecDestroy(exec_);
  for (hipEvent_t e : join_) (void)hipEventDestroy(e);
  for (hipEvent_t e : {fork_, all_packed_, all_pulled_})
    if (e) (void)hipEventDestroy(e);
  if (gs_) (void)hipStreamDestroy(gs_);
}

void GpuGroup::set_state(const double* prev, const double* cur, int n0) {
  for (auto& r : ranks_) r->set_state(prev, cur, n0);
  graph_ = false;  // (the state upload is a pageable host copy: eager runs)
}

std::vector<int> GpuGroup::comm_counts() const {
  std::vector<int> v;
  for (const auto& r : ranks_)
    if (r->comm_) v.push_back(r->comm_->count());
  return v;
}

// Every rank's schedule, interleaved unit by unit exactly as the ranks of a multi-process run would issue them.
void GpuGroup::enqueue() {
  std::vector<GpuSolver*> rs;
  for (auto& p : ranks_) rs.push_back(p.get());
  const bool dbg = std::getenv("W3D_DEBUG") != nullptr;
  auto step = [&](const char* what, int i) {
    if (dbg) std::fprintf(stderr, "[group] unit %d %s\n", i, what);
  };
  for (auto* s : rs) {
    s->xpar_ = static_cast<int>(s->xsolves_ & 1);
    s->phase_init();
    s->tb_region_ = 0;
    s->pending_.clear();
  }
  step("init", -1);
  const int nu = static_cast<int>(rs[0]->units_.size());
  const bool late = rs[0]->late_exchange();
  if (rs[0]->sdma_) {
    // copy-engine group: each rank runs its own production schedule; the phases are issued rank by rank so that every
    // flag wait reaches its HIP queue after the write that releases it (streams of one process may share a hardware
    // queue, where a wait issued first would block the write behind it): all receives (done(i − 1) writes) of unit i
    // before any exchange i (which waits for them), every exchange i − 1 ("arrived" writes) before the receives of unit i
    for (int i = 0; i < nu; ++i) {
      for (auto* s : rs) s->sdma_receive(i);
      for (auto* s : rs) {
        s->unit_shell(i);
        if (!late) s->unit_exchange_sdma(i);
        s->unit_interior(i);
        if (late) s->unit_exchange_sdma(i);
      }
      step("unit", i);
    }
    for (auto* s : rs) {
      s->flush_reduces();
      s->sdma_finish();
      ++s->xsolves_;
    }
    return;
  }
  for (int i = 0; i < nu; ++i) {
    for (auto* s : rs) s->unit_shell(i);
    step("shell", i);
    if (late)
      for (auto* s : rs) s->unit_interior(i);
    // Cross-rank ordering goes through the group stream: it joins every rank's "packed" event, and every puller
    // waits on the join (likewise "pulled" before anyone overwrites its send regions). Direct waits of one rank's
    // stream on a PEER's side-stream event are avoided on purpose: HIP 7.2 crashes in hipStreamEndCapture on such
    // sibling-to-sibling waits (tools/probes/capture_probe2.hip, flag 1); fork/join through the origin captures fine.
    for (auto* s : rs) s->lb_pack(i);
    step("pack", i);
    bool any = false;
    for (auto* s : rs)
      if (s->needs_exchange(i)) {
        capture::wait(gs_, s->ev_packed_);
        any = true;
      }
    if (any) capture::record(all_packed_, gs_);
    for (auto* s : rs) s->lb_pull(i, rs, all_packed_);
    step("pull", i);
    for (auto* s : rs)
      if (s->needs_exchange(i)) capture::wait(gs_, s->ev_halo_);
    if (any) capture::record(all_pulled_, gs_);
    for (auto* s : rs) s->lb_fence(i, all_pulled_);
    step("fence", i);
    if (!late)
      for (auto* s : rs) s->unit_interior(i);
    step("interior", i);
  }
  for (auto* s : rs) s->flush_reduces();
  for (auto* s : rs)
    if (s->push_) {
      s->push_finish(s->s0_);
      s->push_epoch_ += nu;
    }
  step("flush", nu);
}

// the group stream waits for every stream the ranks used
void GpuGroup::join() {
  for (size_t q = 0; q < ranks_.size(); ++q) {
    GpuSolver* s = ranks_[q].get();
    capture::record(join_[2 * q], s->s0_);
    capture::wait(gs_, join_[2 * q]);
    if (s->xstream() != s->s0_) {
      capture::record(join_[2 * q + 1], s->s1_);
      capture::wait(gs_, join_[2 * q + 1]);
    }
  }
}

RunResult GpuGroup::run() {
  if (multi_) {
    // every rank's production solve on its own thread and device, concurrently (RCCL's collectives and send/recv
    // pairs need every rank's call in flight); each rank's log is the global one (all-gathered), rank 0's is returned
    std::vector<RunResult> out(ranks_.size());
    std::vector<std::string> err(ranks_.size());
    std::vector<std::thread> th;
    const double t0 = now_s();
    for (size_t r = 0; r < ranks_.size(); ++r)
      th.emplace_back([&, r] {
        try {
          W3D_HIP(hipSetDevice(ranks_[r]->device()));
          out[r] = ranks_[r]->run();
        } catch (const std::exception& e) {
          err[r] = e.what();
        }
      });
    for (auto& t : th) t.join();
    for (size_t r = 0; r < ranks_.size(); ++r)
      W3D_REQUIRE(err[r].empty(), "multi-device rank " + std::to_string(r) + ": " + err[r]);
    for (size_t r = 1; r < ranks_.size(); ++r)
      W3D_REQUIRE(out[r].max_err == out[0].max_err, "multi-device: ranks gathered different error logs");
    RunResult r = out[0];
    r.solve_s = now_s() - t0;
    ++runs_;
    return r;
  }
  std::vector<GpuSolver*> rs;
  for (auto& p : ranks_) rs.push_back(p.get());
  const int K = rs[0]->prob_.K;
  // capture on the second run (RCCL connects its peers eagerly on the first send/recv, never inside a capture): the
  // group stream forks into every rank's two streams and joins them back, so the graph holds all ranks' work
  const bool dbg = std::getenv("W3D_DEBUG") != nullptr;
  auto trace = [&](const char* what) {
    if (dbg) {
      (void)hipDeviceSynchronize();
      std::fprintf(stderr, "[group] %s: %s\n", what, hipGetErrorString(hipGetLastError()));
    }
  };
  if (graph_ && !exec_ && runs_ >= 1) {
    hipGraph_t g = nullptr;
    bool ok = hipStreamBeginCapture(gs_, hipStreamCaptureModeThreadLocal) == hipSuccess;
    if (dbg) std::fprintf(stderr, "[group] begin capture ok=%d\n", ok ? 1 : 0);
    if (ok) {
      capture::begin(gs_);
      try {
        capture::record(fork_, gs_);
        for (auto* s : rs) {
          capture::wait(s->s0_, fork_);
          if (s->xstream() != s->s0_) capture::wait(s->s1_, fork_);
        }
        enqueue();
        join();
        capture::finish();
      } catch (const std::exception& ex) {
        if (dbg) std::fprintf(stderr, "[group] capture enqueue failed: %s\n", ex.what());
        ok = false;
        capture::close();
      }
      const hipError_t e = hipStreamEndCapture(gs_, &g);
      capture::abandon();
      if (dbg) std::fprintf(stderr, "[group] end capture: %s graph=%p\n", hipGetErrorString(e), (void*)g);
      ok = ok && e == hipSuccess && g != nullptr;
    }
    if (ok) {
      const hipError_t e = hipGraphInstantiate(&exec_, g, nullptr, nullptr, 0);
      if (dbg) std::fprintf(stderr, "[group] instantiate: %s\n", hipGetErrorString(e));
      ok = e == hipSuccess;
      if (ok && hipGraphUpload(exec_, gs_) != hipSuccess) {  // (see GpuSolver::run)
        (void)hipGraphExecDestroy(exec_);
        ok = false;
      }
    }
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    if (!ok) {
      exec_ = nullptr;
      graph_ = false;
    }
  }
  const double t0 = now_s();
  if (exec_ && graph_) {
    W3D_HIP(hipGraphLaunch(exec_, gs_));
    trace("graph launch");
  } else {
    enqueue();
    join();  // the gathers below run on the group stream
  }
  // per-rank error logs to the host: through ncclAllGather on each rank's communicator (rccl-self; one rank each, so
  // the gathered log is the rank's own) or straight from errlog_; combined in rank order as the multi-process
  // all-gather is
  const size_t per = static_cast<size_t>(K + 1);
  std::vector<Partial> all(per * rs.size());
  for (size_t q = 0; q < rs.size(); ++q) {
    GpuSolver* s = rs[q];
    const Partial* src = s->errlog_;
    if (s->comm_) {
      W3D_NCCL(ncclAllGather(s->errlog_, s->errall_, 2 * per, ncclFloat64, static_cast<ncclComm_t>(s->comm_->raw()),
                             gs_));
      src = s->errall_;
    }
    W3D_HIP(hipMemcpyAsync(all.data() + q * per, src, per * sizeof(Partial), hipMemcpyDeviceToHost, gs_));
  }
  trace("gathers");
  wait_stream(gs_, rs[0]->comm_.get(), gpu_timeout_s());
  for (auto* s : rs) {
    if (s->comm_) s->comm_->check_async();
    s->push_check();
  }
  RunResult r;
  for (size_t q = 0; q < rs.size(); ++q)
    W3D_REQUIRE(!rs[q]->sdma_ || all[q * per].x == 0.0,
                "sdma transport: a flag wait timed out on rank " + std::to_string(q));
  const double n_int = static_cast<double>(rs[0]->prob_.N - 1);
  for (int n : rs[0]->check_steps()) {
    double m = 0.0, sum = 0.0;
    for (size_t q = 0; q < rs.size(); ++q) {
      const Partial& v = all[q * per + static_cast<size_t>(n)];
      m = v.x > m || std::isnan(v.x) ? v.x : m;
      sum += v.y;
    }
    r.steps.push_back(n);
    r.max_err.push_back(m);
    r.rms_err.push_back(std::sqrt(sum / (n_int * n_int * n_int)));
    if (!std::isfinite(m) || !std::isfinite(sum)) r.finite = false;
  }
  r.solve_s = now_s() - t0;
  rs[0]->collect_phases(r);  // (timers: rank 0's phases, as the CLI reports)
  ++runs_;
  return r;
}

}  // namespace wave3d
