// Problem specification: PDE, grid, scheme coefficients, analytic solution, CFL guard.
//
// Reference behaviour (AICCer1/MPI-CUDA, documents only — see SURVEY.md §1):
//   * u_tt = Δu on [0,L]^3, homogeneous Dirichlet on all faces        (report.pdf p.4 §1)
//   * grid x_i = i*h, h = L/N, nodes 0..N (N = number of intervals)   (report.pdf p.5 §2; SURVEY §1.2 VERIFIED)
//   * u^0 = φ, u^1 = u^0 + τ²/2 Δ_h u^0, u^{n+1} = 2u^n − u^{n−1} + τ² Δ_h u^n   (report.pdf p.5 §2.2)
//   * analytic u_a = sin(πx/L) sin(πy/L) sin(πz/L) cos(a_t t), a_t = π√3/L        (report.pdf p.4 §1)
//   * CLI positional "N tau K [L]"                                   (report.pdf p.15 §4.2.4)
#pragma once

#include <cmath>
#include <vector>

#include "wave3d/common.hpp"

namespace wave3d {

struct Problem {
  i64 N = 512;        // number of intervals per axis → (N+1)^3 nodes
  double tau = 1e-3;  // time step
  int K = 20;         // number of time steps
  double L = 1.0;     // cube edge length (Lx = Ly = Lz = L)

  double h() const { return L / static_cast<double>(N); }
  i64 nodes() const { return N + 1; }
  // a_t = π·sqrt(1/Lx² + 1/Ly² + 1/Lz²)
  double a_t() const { return M_PI * std::sqrt(3.0 / (L * L)); }
  // Courant number for the 3D 7-point leapfrog: stable iff τ·sqrt(3)/h ≤ 1.
  double courant() const { return tau * std::sqrt(3.0) / h(); }
  bool cfl_ok() const { return courant() <= 1.0; }
  // Largest stable τ for this grid.
  double tau_max() const { return h() / std::sqrt(3.0); }
  // Cell updates of one full solve (reference convention for GCell/s: N³·K).
  double cell_updates() const { return static_cast<double>(N) * N * N * K; }

  void validate() const {
    W3D_REQUIRE(N >= 2, "N must be >= 2");
    W3D_REQUIRE(tau > 0.0 && std::isfinite(tau), "tau must be > 0");
    W3D_REQUIRE(K >= 1, "K must be >= 1");
    W3D_REQUIRE(L > 0.0 && std::isfinite(L), "L must be > 0");
  }
};

// Scheme coefficients shared by every kernel (CPU and GPU use the same values → same bits).
struct Coeffs {
  double ihx2, ihy2, ihz2;  // 1/h_d²
  double tau2;              // τ²
  double half_tau2;         // τ²/2
  double lam;               // τ²/h²: the update coefficient of d2sum (stencil.hpp)
  double half_lam;          // (τ²/2)/h²

  static Coeffs from(const Problem& p) {
    Coeffs c;
    const double h = p.h();
    c.ihx2 = 1.0 / (h * h);
    c.ihy2 = c.ihx2;
    c.ihz2 = c.ihx2;
    c.tau2 = p.tau * p.tau;
    c.half_tau2 = 0.5 * c.tau2;
    c.lam = c.tau2 * c.ihx2;
    c.half_lam = c.half_tau2 * c.ihx2;
    return c;
  }
};

// 1-D factor of the initial condition, sin(π x_i / L) for i = 0..N, with the two boundary entries forced to an exact 0.
// u^0(i,j,k) = (s[i]·s[j])·s[k]; because the boundary entries are 0 the same product also yields the Dirichlet zeros,
// so every kernel (init, first step, error check) evaluates φ by the identical expression.
//
// The returned table is EXTENDED by one zero entry on each side: element [g+1] holds node g for g = -1..N+1, so ghost
// nodes just outside the domain (which some ranks allocate) evaluate to 0 without a branch. Kernels receive &t[1].
inline std::vector<double> sin_table_ext(const Problem& p) {
  std::vector<double> s(static_cast<size_t>(p.N + 3), 0.0);
  const double h = p.h();
  for (i64 i = 1; i < p.N; ++i) {
    const double x = static_cast<double>(i) * h;
    s[static_cast<size_t>(i + 1)] = std::sin(M_PI * x / p.L);
  }
  return s;  // s[1] (node 0) and s[N+1] (node N) stay exact zeros
}

// cos(a_t · n · τ): the time factor of the analytic solution at step n.
inline double time_factor(const Problem& p, int n) { return std::cos(p.a_t() * (static_cast<double>(n) * p.tau)); }

}  // namespace wave3d
