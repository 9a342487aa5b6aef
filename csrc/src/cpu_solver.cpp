// Whole-domain CPU solver (sequential / OpenMP). See wave3d/cpu.hpp.
//
// Reference programs: `wave` (sequential, readme.md:33-36) and `openmpwave`/`wave3dOMP` (report.pdf p.21 §5.2). Phase
// timers follow the reference's CPU breakdown columns init / compute / (check) (report.pdf p.16 §4.4).
#include <algorithm>
#include <chrono>
#include <cmath>

#include "wave3d/cpu.hpp"

namespace wave3d {

namespace {
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

CpuSolver::CpuSolver(const Problem& p, int check_every, int threads) : prob_(p), check_every_(check_every) {
  prob_.validate();
  cpu_set_threads(threads);
  Box b{0, p.N + 1, 0, p.N + 1, 0, p.N + 1};
  lay_ = make_layout(prob_, b);
  u_[0].assign(static_cast<size_t>(lay_.total), 0.0);
  u_[1].assign(static_cast<size_t>(lay_.total), 0.0);
  s_ = sin_table_ext(prob_);
}

void global_to_local(const Layout& l, const double* g, double* out) {
  const i64 n1 = l.N + 1;
  std::fill(out, out + l.total, 0.0);
#pragma omp parallel for schedule(static)
  for (i64 x = -l.xg; x < l.nx + l.xg; ++x) {
    const i64 gx = l.gx0 + x;
    if (gx < 0 || gx > l.N) continue;
    for (i64 y = -l.yg; y < l.ny + l.yg; ++y) {
      const i64 gy = l.gy0 + y;
      if (gy < 0 || gy > l.N) continue;
      const i64 z0 = imax(-l.zg, -l.gz0), z1 = imin(l.nz + l.zg, n1 - l.gz0);
      if (z1 <= z0) continue;
      std::copy(g + (gx * n1 + gy) * n1 + l.gz0 + z0, g + (gx * n1 + gy) * n1 + l.gz0 + z1, out + l.off(x, y, z0));
    }
  }
}

void CpuSolver::set_state(const double* prev, const double* cur, int n0) {
  W3D_REQUIRE(n0 >= 1 && n0 < prob_.K, "resume step must be in [1, K)");
  for (int k = 0; k < 2; ++k) {
    resume_[k].assign(static_cast<size_t>(lay_.total), 0.0);
    global_to_local(lay_, k == 0 ? prev : cur, resume_[k].data());
  }
  resume_n_ = n0;
}

std::vector<int> CpuSolver::check_steps() const {
  std::vector<int> v;
  for (int n = 1; n <= prob_.K; ++n)
    if ((check_every_ > 0 && n % check_every_ == 0) || n == prob_.K) v.push_back(n);
  return v;
}

CpuResult CpuSolver::run() {
  CpuResult r;
  const Coeffs c = Coeffs::from(prob_);
  const double* s = s_.data() + 1;
  const LBox box = compute_box(lay_);
  const double n_int = static_cast<double>(prob_.N - 1);
  const double denom = n_int * n_int * n_int;
  std::vector<char> is_check(static_cast<size_t>(prob_.K + 1), 0);
  for (int n : check_steps()) is_check[static_cast<size_t>(n)] = 1;
  auto record = [&](int n, const ErrAcc& a) {
    r.steps.push_back(n);
    r.max_err.push_back(a.max);
    r.rms_err.push_back(std::sqrt(a.sum / denom));
    if (!std::isfinite(a.max) || !std::isfinite(a.sum)) r.finite = false;
  };
  const double t0 = now_s();
  const int n_start = resume_n_ > 0 ? resume_n_ : 1;
  if (resume_n_ > 0) {
    u_[0] = resume_[0];
    u_[1] = resume_[1];
  } else {
    cpu_init_first(lay_, c, s, u_[0].data(), u_[1].data());
  }
  const double t1 = now_s();
  r.init_s = t1 - t0;
  if (is_check[1] && resume_n_ == 0) {
    ErrAcc a;
    cpu_error(lay_, u_[1].data(), box, s, time_factor(prob_, 1), &a);
    record(1, a);
  }
  int cur = 1, old = 0;
  for (int n = n_start; n <= prob_.K - 1; ++n) {
    const double tc = now_s();
    if (is_check[static_cast<size_t>(n + 1)]) {
      ErrAcc a;
      cpu_leapfrog(lay_, c, u_[cur].data(), u_[old].data(), box, s, time_factor(prob_, n + 1), &a);
      record(n + 1, a);
    } else {
      cpu_leapfrog(lay_, c, u_[cur].data(), u_[old].data(), box, s, 0.0, nullptr);
    }
    r.compute_s += now_s() - tc;
    std::swap(cur, old);
  }
  final_ = cur;
  r.solve_s = now_s() - t0;
  r.slow_phases[0] = r.init_s;
  r.slow_phases[1] = r.compute_s;
  return r;
}

}  // namespace wave3d
