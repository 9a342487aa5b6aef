// Native multi-process CPU solver over a shared-memory segment. See wave3d/cpu_dist.hpp.
#include "wave3d/cpu_dist.hpp"

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <thread>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <new>

namespace wave3d {

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

constexpr size_t kAlign = 64;  // doubles: every outbox starts on its own 512-byte boundary

size_t round_up_sz(size_t a, size_t b) { return (a + b - 1) / b * b; }

}  // namespace

void ShmGroup::layout(const Problem& p) {
  W3D_REQUIRE(world_ >= 1 && dims_.size() == world_, "ShmGroup: dims do not match the world size");
  static_assert(std::atomic<int>::is_always_lock_free, "process-shared atomics must be lock-free");
  const Dims& d = dims_;
  const int world = world_;
  size_t off = 0;
  face_off_.resize(static_cast<size_t>(world));
  for (int r = 0; r < world; ++r) {
    const Layout l = make_layout(p, rank_box(p, d, r));
    const HaloPlan h = make_halo_plan(l, d, r);
    for (const Face& f : h.faces) {
      face_off_[static_cast<size_t>(r)].push_back(off);
      off = round_up_sz(off + static_cast<size_t>(f.count), kAlign);
    }
  }
  // per rank: error log (max, Σe²) for steps 0..K, then 8 timer slots
  slot_doubles_ = round_up_sz(2 * static_cast<size_t>(p.K + 1) + 8, kAlign);
  slot_off_ = off;
  off += slot_doubles_ * static_cast<size_t>(world);
  bytes_ = 4096 + off * sizeof(double);
}

ShmGroup::ShmGroup(const Problem& p, const Dims& d, int world) : world_(world), dims_(d) {
  layout(p);
  base_ = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (base_ == MAP_FAILED) {
    base_ = nullptr;
    fail("ShmGroup: mmap of " + std::to_string(bytes_) + " bytes failed");
  }
  hdr_ = new (base_) Header;
  hdr_->count.store(0);
  hdr_->sense.store(0);
  hdr_->failed.store(0);
  hdr_->ready.store(1);
}

ShmGroup::ShmGroup(const Problem& p, const Dims& d, int world, const std::string& name, int rank, double timeout_s)
    : world_(world), dims_(d), name_(name), owner_(rank == 0) {
  layout(p);
  W3D_REQUIRE(!name.empty() && name[0] == '/', "ShmGroup: segment names start with '/'");
  const double t0 = now_s();
  int fd = -1;
  if (owner_) {
    shm_unlink(name.c_str());  // a stale segment of an aborted run with the same job id
    fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) fail("ShmGroup: shm_open(" + name + ") failed: " + std::strerror(errno));
    if (ftruncate(fd, static_cast<off_t>(bytes_)) != 0) {
      close(fd);
      shm_unlink(name.c_str());
      fail("ShmGroup: ftruncate failed");
    }
  } else {
    for (;;) {  // rank 0 creates the segment: wait for it with its full size
      fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd >= 0) {
        struct stat st {};
        if (fstat(fd, &st) == 0 && static_cast<size_t>(st.st_size) >= bytes_) break;
        close(fd);
        fd = -1;
      }
      if (now_s() - t0 > timeout_s) fail("ShmGroup: rank 0 did not create " + name + " in time");
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
  }
  base_ = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (base_ == MAP_FAILED) {
    base_ = nullptr;
    if (owner_) shm_unlink(name.c_str());
    fail("ShmGroup: mmap of " + name + " failed");
  }
  hdr_ = static_cast<Header*>(base_);
  if (owner_) {
    new (base_) Header;
    hdr_->count.store(0);
    hdr_->sense.store(0);
    hdr_->failed.store(0);
    hdr_->ready.store(1, std::memory_order_release);
  } else {
    while (hdr_->ready.load(std::memory_order_acquire) != 1) {
      if (now_s() - t0 > timeout_s) fail("ShmGroup: " + name + " never became ready");
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  }
}

ShmGroup::~ShmGroup() {
  if (base_) munmap(base_, bytes_);
  if (owner_ && !name_.empty()) shm_unlink(name_.c_str());
}

double* ShmGroup::data() const { return reinterpret_cast<double*>(static_cast<char*>(base_) + 4096); }

double* ShmGroup::outbox(int rank, int f) const {
  return data() + face_off_[static_cast<size_t>(rank)][static_cast<size_t>(f)];
}

double* ShmGroup::slot(int rank) const { return data() + slot_off_ + slot_doubles_ * static_cast<size_t>(rank); }

void ShmGroup::abort() { hdr_->failed.store(1, std::memory_order_release); }

// Sense-reversing central barrier. The acq_rel arrival and the acquire spin order every rank's plain stores before
// the barrier (outboxes, slots) with every rank's loads after it.
void ShmGroup::barrier(double timeout_s) {
  if (world_ == 1) return;
  const int my = local_sense_ ^= 1;
  if (hdr_->count.fetch_add(1, std::memory_order_acq_rel) == world_ - 1) {
    hdr_->count.store(0, std::memory_order_relaxed);
    hdr_->sense.store(my, std::memory_order_release);
    return;
  }
  const double t0 = now_s();
  for (unsigned spin = 0; hdr_->sense.load(std::memory_order_acquire) != my; ++spin) {
    if (hdr_->failed.load(std::memory_order_acquire)) fail("another rank failed");
    if (spin > 1024) {
      sched_yield();
      if ((spin & 1023) == 0 && now_s() - t0 > timeout_s) {
        abort();
        fail("barrier timed out (a rank died or hangs)");
      }
    }
  }
}

CpuRankSolver::CpuRankSolver(const Problem& p, ShmGroup& g, int rank, int check_every, int threads)
    : prob_(p), g_(g), rank_(rank), check_every_(check_every) {
  prob_.validate();
  cpu_set_threads(threads);
  lay_ = make_layout(prob_, rank_box(prob_, g.dims(), rank));
  plan_ = make_halo_plan(lay_, g.dims(), rank);
  u_[0].assign(static_cast<size_t>(lay_.total), 0.0);
  u_[1].assign(static_cast<size_t>(lay_.total), 0.0);
  s_ = sin_table_ext(prob_);
  for (const Face& f : plan_.faces) {
    const HaloPlan hq = make_halo_plan(make_layout(prob_, rank_box(prob_, g.dims(), f.peer)), g.dims(), f.peer);
    int idx = -1;
    for (size_t k = 0; k < hq.faces.size(); ++k)
      if (hq.faces[k].peer == rank_ && hq.faces[k].axis == f.axis && hq.faces[k].side == 1 - f.side)
        idx = static_cast<int>(k);
    W3D_REQUIRE(idx >= 0 && hq.faces[static_cast<size_t>(idx)].count == f.count, "exchange: peer face mismatch");
    peer_face_.push_back(idx);
  }
}

std::vector<int> CpuRankSolver::check_steps() const {
  std::vector<int> v;
  for (int n = 1; n <= prob_.K; ++n)
    if ((check_every_ > 0 && n % check_every_ == 0) || n == prob_.K) v.push_back(n);
  return v;
}

// Every rank publishes its faces of u, waits, copies each neighbour's matching face into its ghost layer, and waits
// again before the outboxes may be overwritten (the MPI_Sendrecv of the reference's exchange, report.pdf p.16).
void CpuRankSolver::exchange(double* u) {
  if (!plan_.any()) return;
  const double t0 = now_s();
  for (size_t f = 0; f < plan_.faces.size(); ++f)
    cpu_pack_face(lay_, plan_.faces[f], u, g_.outbox(rank_, static_cast<int>(f)));
  const double t1 = now_s();
  g_.barrier();
  const double t2 = now_s();
  for (size_t f = 0; f < plan_.faces.size(); ++f)
    cpu_unpack_face(lay_, plan_.faces[f], g_.outbox(plan_.faces[f].peer, peer_face_[f]), u);
  const double t3 = now_s();
  g_.barrier();
  boundary_s_ += (t1 - t0) + (t3 - t2);  // face packing ("boundary processing")
  exchange_s_ += (t2 - t1) + (now_s() - t3);  // waiting for the neighbours
}

CpuResult CpuRankSolver::run() {
  CpuResult r;
  const Coeffs c = Coeffs::from(prob_);
  const double* s = s_.data() + 1;
  const LBox box = compute_box(lay_);
  const int K = prob_.K;
  std::vector<char> is_check(static_cast<size_t>(K + 1), 0);
  for (int n : check_steps()) is_check[static_cast<size_t>(n)] = 1;
  double* mine = g_.slot(rank_);
  for (size_t q = 0; q < 2 * static_cast<size_t>(K + 1); ++q) mine[q] = 0.0;
  exchange_s_ = boundary_s_ = 0.0;
  g_.barrier();
  const double t0 = now_s();
  cpu_init_first(lay_, c, s, u_[0].data(), u_[1].data());  // ghosts analytic: no exchange before step 2
  const double t1 = now_s();
  r.init_s = t1 - t0;
  auto record = [&](int n, const ErrAcc& a) {
    mine[2 * n] = a.max;
    mine[2 * n + 1] = a.sum;
  };
  if (is_check[1]) {
    ErrAcc a;
    cpu_error(lay_, u_[1].data(), box, s, time_factor(prob_, 1), &a);
    record(1, a);
  }
  int cur = 1, old = 0;
  for (int n = 1; n <= K - 1; ++n) {
    if (n > 1) exchange(u_[cur].data());
    const double tc = now_s();
    if (is_check[static_cast<size_t>(n + 1)]) {
      ErrAcc a;
      if (!box.empty()) cpu_leapfrog(lay_, c, u_[cur].data(), u_[old].data(), box, s, time_factor(prob_, n + 1), &a);
      record(n + 1, a);
    } else if (!box.empty()) {
      cpu_leapfrog(lay_, c, u_[cur].data(), u_[old].data(), box, s, 0.0, nullptr);
    }
    r.compute_s += now_s() - tc;
    std::swap(cur, old);
  }
  final_ = cur;
  const size_t tslot = 2 * static_cast<size_t>(K + 1);
  mine[tslot] = now_s() - t0;
  mine[tslot + 1] = exchange_s_;
  mine[tslot + 2] = boundary_s_;
  mine[tslot + 3] = r.init_s;
  mine[tslot + 4] = r.compute_s;
  g_.barrier();  // every rank's partials and timers are in its slot
  const double n_int = static_cast<double>(prob_.N - 1);
  const double denom = n_int * n_int * n_int;
  for (int n : check_steps()) {
    double m = 0.0, sum = 0.0;
    for (int q = 0; q < g_.world(); ++q) {  // fixed rank order: the same log on every rank and every run
      const double* v = g_.slot(q);
      m = v[2 * n] > m || std::isnan(v[2 * n]) ? v[2 * n] : m;
      sum += v[2 * n + 1];
    }
    r.steps.push_back(n);
    r.max_err.push_back(m);
    r.rms_err.push_back(std::sqrt(sum / denom));
    if (!std::isfinite(m) || !std::isfinite(sum)) r.finite = false;
  }
  r.solve_s = 0.0;
  for (int q = 0; q < g_.world(); ++q) {  // the reference reports the slowest rank (max over ranks), per phase too
    const double* v = g_.slot(q);
    if (v[tslot] >= r.solve_s) {
      r.slow_phases[0] = v[tslot + 3];
      r.slow_phases[1] = v[tslot + 4];
      r.slow_phases[2] = v[tslot + 2];
      r.slow_phases[3] = v[tslot + 1];
    }
    r.solve_s = std::max(r.solve_s, v[tslot]);
    exchange_s_ = std::max(exchange_s_, v[tslot + 1]);
    boundary_s_ = std::max(boundary_s_, v[tslot + 2]);
    r.init_s = std::max(r.init_s, v[tslot + 3]);
    r.compute_s = std::max(r.compute_s, v[tslot + 4]);
  }
  r.exchange_s = exchange_s_;
  r.boundary_s = boundary_s_;
  g_.barrier();  // the slots may be reused by the next run
  return r;
}

}  // namespace wave3d
