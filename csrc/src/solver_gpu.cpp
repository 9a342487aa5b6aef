// GPU solver runtime. See wave3d/solver.hpp.
#include "wave3d/solver.hpp"

#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
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

GpuSolver::GpuSolver(const Problem& prob, const SolverOptions& opt, int rank, int world, std::shared_ptr<Comm> comm,
                     bool loopback)
    : prob_(prob), opt_(opt), coef_(Coeffs::from(prob)), rank_(rank), world_(world), comm_(std::move(comm)),
      loopback_(loopback) {
  prob_.validate();
  W3D_REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad rank/world");
  W3D_REQUIRE(world == 1 || comm_ || loopback_, "world > 1 needs an RCCL communicator (or the loopback group)");
  dims_ = parse_dims(opt_.decomp, world, prob_.N);
  const Box box = rank_box(prob_, dims_, rank);
  W3D_REQUIRE(box.nx() >= 1 && box.ny() >= 1 && box.nz() >= 1,
              "decomposition leaves a rank without nodes; use fewer ranks or a larger N");
  lay_ = make_layout(prob_, box);
  plan_ = make_halo_plan(lay_, dims_, rank);
  full_ = compute_box(lay_);

  // interior = compute box minus one layer on every side that has a neighbour; shell = the rest, in ≤6 disjoint boxes
  bool nb[3][2];
  for (int a = 0; a < 3; ++a)
    for (int s = 0; s < 2; ++s) nb[a][s] = neighbor_rank(dims_, rank, a, s) >= 0;
  interior_ = full_;
  if (nb[0][0]) interior_.x0 += 1;
  if (nb[0][1]) interior_.x1 -= 1;
  if (nb[1][0]) interior_.y0 += 1;
  if (nb[1][1]) interior_.y1 -= 1;
  if (nb[2][0]) interior_.z0 += 1;
  if (nb[2][1]) interior_.z1 -= 1;
  auto push = [&](LBox b) {
    if (!b.empty()) shell_.push_back(b);
  };
  if (!full_.empty()) {
    const i64 ix0 = imin(imax(interior_.x0, full_.x0), full_.x1), ix1 = imax(interior_.x1, ix0);
    const i64 iy0 = imin(imax(interior_.y0, full_.y0), full_.y1), iy1 = imax(interior_.y1, iy0);
    if (nb[0][0]) push(LBox{full_.x0, full_.x0 + 1, full_.y0, full_.y1, full_.z0, full_.z1});
    if (nb[0][1]) push(LBox{imax(full_.x1 - 1, full_.x0 + (nb[0][0] ? 1 : 0)), full_.x1, full_.y0, full_.y1, full_.z0, full_.z1});
    if (nb[1][0]) push(LBox{ix0, ix1, full_.y0, full_.y0 + 1, full_.z0, full_.z1});
    if (nb[1][1]) push(LBox{ix0, ix1, imax(full_.y1 - 1, full_.y0 + (nb[1][0] ? 1 : 0)), full_.y1, full_.z0, full_.z1});
    if (nb[2][0]) push(LBox{ix0, ix1, iy0, iy1, full_.z0, full_.z0 + 1});
    if (nb[2][1]) push(LBox{ix0, ix1, iy0, iy1, imax(full_.z1 - 1, full_.z0 + (nb[2][0] ? 1 : 0)), full_.z1});
  }
  if (interior_.x1 < interior_.x0 || interior_.y1 < interior_.y0 || interior_.z1 < interior_.z0) interior_ = LBox{};

  // device memory
  W3D_HIP(hipStreamCreateWithFlags(&s0_, hipStreamNonBlocking));
  W3D_HIP(hipStreamCreateWithFlags(&s1_, hipStreamNonBlocking));
  W3D_HIP(hipEventCreateWithFlags(&ev_shell_, hipEventDisableTiming));
  W3D_HIP(hipEventCreateWithFlags(&ev_halo_, hipEventDisableTiming));
  W3D_HIP(hipEventCreateWithFlags(&ev_packed_, hipEventDisableTiming));
  // memory plan: temporal blocking needs four field buffers; fall back to the two-buffer in-place scheme when four
  // do not fit next to the other allocations (2049³ fp64 is 68.8 GB per buffer)
  nbuf_ = (opt_.temporal == 2 && !plan_.any() && world_ == 1) ? 4 : 2;
  {
    size_t free_b = 0, total_b = 0;
    W3D_HIP(hipMemGetInfo(&free_b, &total_b));
    const double need2 = 2.0 * static_cast<double>(lay_.bytes()), headroom = 2.0e9;
    W3D_REQUIRE(need2 + 1.0e8 < static_cast<double>(free_b),
                "not enough device memory for two field buffers of " + std::to_string(lay_.bytes()) + " bytes");
    if (nbuf_ == 4 && 2.0 * need2 + headroom > static_cast<double>(free_b)) nbuf_ = 2;
  }
  for (int b = 0; b < nbuf_; ++b) {
    W3D_HIP(hipMalloc(&u_[b], static_cast<size_t>(lay_.bytes())));
    W3D_HIP(hipMemset(u_[b], 0, static_cast<size_t>(lay_.bytes())));
  }
  const std::vector<double> s = sin_table_ext(prob_);
  W3D_HIP(hipMalloc(&d_s_, s.size() * sizeof(double)));
  W3D_HIP(hipMemcpy(d_s_, s.data(), s.size() * sizeof(double), hipMemcpyHostToDevice));
  if (plan_.packed_doubles > 0) {
    W3D_HIP(hipMalloc(&send_buf_, static_cast<size_t>(plan_.packed_doubles) * sizeof(double)));
    W3D_HIP(hipMalloc(&recv_buf_, static_cast<size_t>(plan_.packed_doubles) * sizeof(double)));
  }
  n_full_ = leapfrog_blocks(lay_, &full_, 1, opt_.tiling);
  n_shell_ = leapfrog_blocks(lay_, shell_.data(), static_cast<int>(shell_.size()), opt_.tiling);
  n_int_ = leapfrog_blocks(lay_, &interior_, 1, opt_.tiling);
  n_fused_ = (nbuf_ == 4 && !full_.empty()) ? leapfrog2_partials(lay_, full_, opt_.tiling2) : 0;
  n_partials_ = std::max({n_full_, n_shell_ + n_int_, error_blocks(lay_, full_), n_fused_,
                          opt_.init2 ? init_two_partials(lay_) : 0, 1});
  W3D_HIP(hipMalloc(&partials_, static_cast<size_t>(n_partials_) * sizeof(Partial)));
  W3D_HIP(hipMalloc(&errlog_, static_cast<size_t>(prob_.K + 1) * sizeof(Partial)));
  W3D_HIP(hipMalloc(&errall_, static_cast<size_t>(world_) * (prob_.K + 1) * sizeof(Partial)));
  ct_.resize(static_cast<size_t>(prob_.K + 1));
  for (int n = 0; n <= prob_.K; ++n) ct_[static_cast<size_t>(n)] = time_factor(prob_, n);
  if (opt_.timers || opt_.debug_sync || loopback_) opt_.graph = false;
}

GpuSolver::~GpuSolver() {
  if (graph_exec_) hipGraphExecDestroy(graph_exec_);
  for (double* p : {u_[0], u_[1], u_[2], u_[3], d_s_, send_buf_, recv_buf_})
    if (p) hipFree(p);
  if (partials_) hipFree(partials_);
  if (errlog_) hipFree(errlog_);
  if (errall_) hipFree(errall_);
  for (hipEvent_t e : ev_pool_) hipEventDestroy(e);
  if (ev_shell_) hipEventDestroy(ev_shell_);
  if (ev_halo_) hipEventDestroy(ev_halo_);
  if (ev_packed_) hipEventDestroy(ev_packed_);
  if (s0_) hipStreamDestroy(s0_);
  if (s1_) hipStreamDestroy(s1_);
}

size_t GpuSolver::device_bytes() const {
  return static_cast<size_t>(nbuf_) * static_cast<size_t>(lay_.bytes()) + 2 * static_cast<size_t>(plan_.packed_doubles) * sizeof(double) +
         static_cast<size_t>(n_partials_) * sizeof(Partial) + static_cast<size_t>(prob_.N + 3) * sizeof(double);
}

std::vector<int> GpuSolver::check_steps() const {
  std::vector<int> v;
  const int ce = opt_.check_every;
  for (int n = 1; n <= prob_.K; ++n)
    if ((ce > 0 && n % ce == 0) || n == prob_.K) v.push_back(n);
  return v;
}

void GpuSolver::exchange(double* field, hipStream_t st) {
  if (!plan_.any()) return;
  if (plan_.packed_doubles > 0) launch_pack(lay_, plan_, field, send_buf_, st);
  ncclComm_t c = static_cast<ncclComm_t>(comm_->raw());
  W3D_NCCL(ncclGroupStart());
  for (const Face& f : plan_.faces) {
    const double* sp = f.contiguous ? field + f.send_off : send_buf_ + f.pack_off;
    double* rp = f.contiguous ? field + f.recv_off : recv_buf_ + f.pack_off;
    W3D_NCCL(ncclSend(sp, static_cast<size_t>(f.count), ncclFloat64, f.peer, c, st));
    W3D_NCCL(ncclRecv(rp, static_cast<size_t>(f.count), ncclFloat64, f.peer, c, st));
  }
  W3D_NCCL(ncclGroupEnd());
  if (plan_.packed_doubles > 0) launch_unpack(lay_, plan_, recv_buf_, field, st);
}

// ------------------------------------------------------------------------------------------------------------------
// step phases. One step n (u^{n+1} from u^n, u^{n−1}) is: shell → exchange → interior. With overlap the exchange
// carries the NEW field's shell faces on the side stream s1 while the interior runs on s0; without overlap the
// exchange carries the CURRENT field's faces on s0 before the whole-box update.
// ------------------------------------------------------------------------------------------------------------------
bool GpuSolver::split() const { return opt_.overlap && plan_.any(); }

bool GpuSolver::needs_exchange(int n) const {
  if (!plan_.any()) return false;
  return split() ? n < prob_.K - 1 : n > start_n_;
}

double* GpuSolver::xfield() const { return split() ? u_[old_] : u_[cur_]; }
hipStream_t GpuSolver::xstream() const { return split() ? s1_ : s0_; }

// Per-phase device timers (SolverOptions::timers, eager launches only): every timed launch group is bracketed by two
// events on its stream; after the solve the intervals are summed per phase. The reference reports its GPU time as
// compute / H2D-D2H copies / MPI exchange (report.pdf p.16 §4.4); here: init, compute (shell + interior / fused),
// exchange (pack + RCCL + unpack, overlapped with compute on the side stream) and error check (reductions).
template <class F>
void GpuSolver::timed(int phase, hipStream_t st, F&& f) {
  if (!opt_.timers) {
    f();
    return;
  }
  auto take = [&]() {
    if (ev_next_ == ev_pool_.size()) {
      hipEvent_t e;
      W3D_HIP(hipEventCreate(&e));
      ev_pool_.push_back(e);
    }
    return ev_pool_[ev_next_++];
  };
  hipEvent_t a = take(), b = take();
  W3D_HIP(hipEventRecord(a, st));
  f();
  W3D_HIP(hipEventRecord(b, st));
  marks_.push_back({phase, a, b});
}

void GpuSolver::phase_init() {
  const int K = prob_.K;
  const double* s = d_s_ + 1;
  is_check_.assign(static_cast<size_t>(K + 1), 0);
  for (int n : check_steps()) is_check_[static_cast<size_t>(n)] = 1;
  ev_next_ = 0;
  marks_.clear();
  W3D_HIP(hipMemsetAsync(errlog_, 0, static_cast<size_t>(K + 1) * sizeof(Partial), s0_));
  if (opt_.init2 && K >= 2) {
    // u¹ -> buf 0, u² -> buf 1 analytically (no read pass); the first leapfrog step is n = 2
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
}

void GpuSolver::phase_shell(int n) {
  const bool chk = is_check_[static_cast<size_t>(n + 1)] != 0;
  if (split()) {
    timed(kPhaseShell, s0_, [&] {
      launch_leapfrog(lay_, coef_, u_[cur_], u_[old_], shell_.data(), static_cast<int>(shell_.size()), d_s_ + 1,
                      ct_[static_cast<size_t>(n + 1)], chk ? partials_ : nullptr, opt_.tiling, s0_);
    });
  }
  if (needs_exchange(n)) W3D_HIP(hipEventRecord(ev_shell_, s0_));
}

void GpuSolver::phase_exchange_rccl(int n) {
  if (!needs_exchange(n)) return;
  hipStream_t xs = xstream();
  if (xs != s0_) W3D_HIP(hipStreamWaitEvent(xs, ev_shell_, 0));
  if (opt_.poison_ghosts) poison(xfield(), xs);
  timed(kPhaseComm, xs, [&] { exchange(xfield(), xs); });
  if (split()) W3D_HIP(hipEventRecord(ev_halo_, xs));
}

void GpuSolver::phase_interior(int n) {
  const bool chk = is_check_[static_cast<size_t>(n + 1)] != 0;
  const double ct = ct_[static_cast<size_t>(n + 1)];
  if (split()) {
    timed(kPhaseCompute, s0_, [&] {
      launch_leapfrog(lay_, coef_, u_[cur_], u_[old_], &interior_, 1, d_s_ + 1, ct,
                      chk ? partials_ + n_shell_ : nullptr, opt_.tiling, s0_);
    });
    if (needs_exchange(n)) W3D_HIP(hipStreamWaitEvent(s0_, ev_halo_, 0));
    if (chk) timed(kPhaseCheck, s0_, [&] { launch_reduce(partials_, n_shell_ + n_int_, errlog_ + n + 1, s0_); });
  } else {
    timed(kPhaseCompute, s0_, [&] {
      launch_leapfrog(lay_, coef_, u_[cur_], u_[old_], &full_, 1, d_s_ + 1, ct, chk ? partials_ : nullptr,
                      opt_.tiling, s0_);
    });
    if (chk) timed(kPhaseCheck, s0_, [&] { launch_reduce(partials_, n_full_, errlog_ + n + 1, s0_); });
  }
  if (opt_.debug_sync) W3D_HIP(hipDeviceSynchronize());
  std::swap(cur_, old_);
  if (n == prob_.K - 1) final_buf_ = cur_;
}

void GpuSolver::enqueue_solve() {
  if (fused()) {
    enqueue_solve_fused();
    return;
  }
  phase_init();
  for (int n = start_n_; n <= prob_.K - 1; ++n) {
    phase_shell(n);
    phase_exchange_rccl(n);
    phase_interior(n);
  }
  final_buf_ = cur_;
  prev_buf_ = old_;
}

bool GpuSolver::fused() const { return opt_.temporal == 2 && !plan_.any() && nbuf_ == 4 && !full_.empty(); }

// Single rank with temporal blocking: steps are taken two at a time (u^{n+1}, u^{n+2} in one HBM pass) whenever the
// intermediate step n+1 needs no error check; otherwise one in-place step. Four buffers rotate (see kernels.hpp).
void GpuSolver::enqueue_solve_fused() {
  phase_init();  // (u0, u1) or (u1, u2) -> bufs (0, 1); cur_ = 1, old_ = 0
  const int K = prob_.K;
  const double* s = d_s_ + 1;
  int n = start_n_;  // u^n is current
  while (n <= K - 1) {
    if (n + 2 <= K && !is_check_[static_cast<size_t>(n + 1)]) {
      int f[2], k = 0;
      for (int b = 0; b < 4; ++b)
        if (b != cur_ && b != old_) f[k++] = b;
      const bool chk = is_check_[static_cast<size_t>(n + 2)] != 0;
      timed(kPhaseCompute, s0_, [&] {
        launch_leapfrog2(lay_, coef_, u_[old_], u_[cur_], u_[f[0]], u_[f[1]], full_, s,
                         ct_[static_cast<size_t>(n + 2)], chk ? partials_ : nullptr, opt_.tiling2, s0_);
      });
      if (chk) timed(kPhaseCheck, s0_, [&] { launch_reduce(partials_, n_fused_, errlog_ + n + 2, s0_); });
      old_ = f[0];
      cur_ = f[1];
      n += 2;
    } else {
      const bool chk = is_check_[static_cast<size_t>(n + 1)] != 0;
      timed(kPhaseCompute, s0_, [&] {
        launch_leapfrog(lay_, coef_, u_[cur_], u_[old_], &full_, 1, s, ct_[static_cast<size_t>(n + 1)],
                        chk ? partials_ : nullptr, opt_.tiling, s0_);
      });
      if (chk) timed(kPhaseCheck, s0_, [&] { launch_reduce(partials_, n_full_, errlog_ + n + 1, s0_); });
      std::swap(cur_, old_);
      n += 1;
    }
    if (opt_.debug_sync) W3D_HIP(hipDeviceSynchronize());
  }
  final_buf_ = cur_;
  prev_buf_ = old_;
}

// Debug aid: fill the ghost layers that the next exchange must overwrite with NaN, so a halo that
// is not delivered shows up in the error norms at once instead of silently reusing stale values.
void GpuSolver::poison(double* field, hipStream_t st) {
  for (const Face& f : plan_.faces) {
    if (f.contiguous) {
      W3D_HIP(hipMemsetAsync(field + f.recv_off, 0xFF, static_cast<size_t>(f.count) * sizeof(double), st));
    }
  }
  if (plan_.packed_doubles > 0)
    W3D_HIP(hipMemsetAsync(recv_buf_, 0xFF, static_cast<size_t>(plan_.packed_doubles) * sizeof(double), st));
}

void GpuSolver::collect_phases(RunResult& r) {
  if (!opt_.timers) return;
  double acc[kNumPhases] = {0, 0, 0, 0, 0};
  for (const auto& m : marks_) {
    float ms = 0.0f;
    W3D_HIP(hipEventElapsedTime(&ms, m.b, m.e));
    acc[m.phase] += ms;
  }
  r.phases.init_ms = acc[kPhaseInit];
  r.phases.shell_ms = acc[kPhaseShell];
  r.phases.interior_ms = acc[kPhaseCompute];
  r.phases.comm_ms = acc[kPhaseComm];
  r.phases.check_ms = acc[kPhaseCheck];
}

// ------------------------------------------------------------------------------------------------------------------
// loopback transport (GpuGroup): P ranks in one process on one device, halos moved by device copies. Test-only
// stand-in for RCCL that exercises the identical shell/interior split, halo plans, pack/unpack and stream/event
// ordering of the production path on a single GPU (RCCL refuses two ranks on one device).
// ------------------------------------------------------------------------------------------------------------------
void GpuSolver::lb_pack(int n) {
  if (!needs_exchange(n)) return;
  hipStream_t xs = xstream();
  if (xs != s0_) W3D_HIP(hipStreamWaitEvent(xs, ev_shell_, 0));
  if (plan_.packed_doubles > 0) launch_pack(lay_, plan_, xfield(), send_buf_, xs);
  W3D_HIP(hipEventRecord(ev_packed_, xs));
}

void GpuSolver::lb_pull(int n, const std::vector<GpuSolver*>& ranks) {
  if (!needs_exchange(n)) return;
  hipStream_t xs = xstream();
  const int b = split() ? old_ : cur_;
  if (opt_.poison_ghosts) poison(u_[b], xs);
  for (const Face& f : plan_.faces) {
    const GpuSolver* q = ranks[static_cast<size_t>(f.peer)];
    const Face* g = nullptr;
    for (const Face& h : q->plan_.faces)
      if (h.peer == rank_) g = &h;
    W3D_REQUIRE(g && g->count == f.count, "loopback: mismatched faces");
    W3D_HIP(hipStreamWaitEvent(xs, q->ev_packed_, 0));
    const double* src = g->contiguous ? q->u_[b] + g->send_off : q->send_buf_ + g->pack_off;
    double* dst = f.contiguous ? u_[b] + f.recv_off : recv_buf_ + f.pack_off;
    W3D_HIP(hipMemcpyAsync(dst, src, static_cast<size_t>(f.count) * sizeof(double), hipMemcpyDeviceToDevice, xs));
  }
  if (plan_.packed_doubles > 0) launch_unpack(lay_, plan_, recv_buf_, u_[b], xs);
  W3D_HIP(hipEventRecord(ev_halo_, xs));
}

void GpuSolver::lb_fence(int n, const std::vector<GpuSolver*>& ranks) {
  // the peers have read this rank's send regions once their pulls are done: keep both streams behind them
  if (!needs_exchange(n)) return;
  for (const Face& f : plan_.faces) {
    const GpuSolver* q = ranks[static_cast<size_t>(f.peer)];
    W3D_HIP(hipStreamWaitEvent(s0_, q->ev_halo_, 0));
    if (s1_ != s0_) W3D_HIP(hipStreamWaitEvent(s1_, q->ev_halo_, 0));
  }
}

RunResult GpuSolver::collect_local() {
  RunResult r;
  gather_errors(r);
  return r;
}

void GpuSolver::gather_errors(RunResult& r) {
  const int K = prob_.K;
  const size_t per = static_cast<size_t>(K + 1);
  std::vector<Partial> host(per * static_cast<size_t>(world_));
  if (world_ > 1 && comm_) {
    W3D_NCCL(ncclAllGather(errlog_, errall_, 2 * per, ncclFloat64, static_cast<ncclComm_t>(comm_->raw()), s0_));
    W3D_HIP(hipMemcpyAsync(host.data(), errall_, host.size() * sizeof(Partial), hipMemcpyDeviceToHost, s0_));
  } else {
    host.resize(per);
    W3D_HIP(hipMemcpyAsync(host.data(), errlog_, per * sizeof(Partial), hipMemcpyDeviceToHost, s0_));
  }
  wait_stream(s0_, comm_.get(), gpu_timeout_s());
  const int nsrc = static_cast<int>(host.size() / per);
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
  if (opt_.graph && !graph_exec_) {
    // capture once (outside the timed region of later runs); fall back to eager launches if capture is refused
    hipGraph_t g = nullptr;
    bool ok = hipStreamBeginCapture(s0_, hipStreamCaptureModeThreadLocal) == hipSuccess;
    if (ok) {
      try {
        enqueue_solve();
      } catch (...) {
        ok = false;
      }
      const hipError_t e = hipStreamEndCapture(s0_, &g);
      ok = ok && e == hipSuccess && g != nullptr;
    }
    if (ok) ok = hipGraphInstantiate(&graph_exec_, g, nullptr, nullptr, 0) == hipSuccess;
    if (g) hipGraphDestroy(g);
    (void)hipGetLastError();
    if (!ok) {
      graph_exec_ = nullptr;
      opt_.graph = false;
    }
  }
  const double t0 = now_s();
  if (graph_exec_)
    W3D_HIP(hipGraphLaunch(graph_exec_, s0_));
  else
    enqueue_solve();
  const double tg = now_s();
  gather_errors(r);
  r.solve_s = now_s() - t0;
  collect_phases(r);
  r.phases.gather_ms = (now_s() - tg) * 1e3;  // host: waits for the device, then all-gathers the error log
  return r;
}

std::vector<double> GpuSolver::download(int which) const {
  std::vector<double> h(static_cast<size_t>(lay_.total));
  const double* src = u_[which == 0 ? final_buf_ : prev_buf_];
  W3D_HIP(hipDeviceSynchronize());
  W3D_HIP(hipMemcpy(h.data(), src, h.size() * sizeof(double), hipMemcpyDeviceToHost));
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

}  // namespace wave3d

namespace wave3d {

GpuGroup::GpuGroup(const Problem& prob, const SolverOptions& opt, int world) {
  W3D_REQUIRE(world >= 1, "world must be >= 1");
  for (int r = 0; r < world; ++r) ranks_.push_back(std::make_unique<GpuSolver>(prob, opt, r, world, nullptr, true));
}

RunResult GpuGroup::run() {
  std::vector<GpuSolver*> rs;
  for (auto& p : ranks_) rs.push_back(p.get());
  const int K = rs[0]->prob_.K;
  const double t0 = now_s();
  for (auto* s : rs) s->phase_init();
  for (int n = rs[0]->start_n_; n <= K - 1; ++n) {
    for (auto* s : rs) s->phase_shell(n);
    for (auto* s : rs) s->lb_pack(n);
    for (auto* s : rs) s->lb_pull(n, rs);
    for (auto* s : rs) s->lb_fence(n, rs);
    for (auto* s : rs) s->phase_interior(n);
  }
  // combine the per-rank error logs in rank order (what the RCCL all-gather does across processes)
  const size_t per = static_cast<size_t>(K + 1);
  std::vector<Partial> all(per * rs.size());
  for (size_t q = 0; q < rs.size(); ++q) {
    rs[q]->final_buf_ = rs[q]->cur_;
    rs[q]->prev_buf_ = rs[q]->old_;
    W3D_HIP(hipMemcpyAsync(all.data() + q * per, rs[q]->errlog_, per * sizeof(Partial), hipMemcpyDeviceToHost,
                           rs[q]->s0_));
  }
  for (auto* s : rs) wait_stream(s->s0_, nullptr, gpu_timeout_s());
  RunResult r;
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
  return r;
}

}  // namespace wave3d
