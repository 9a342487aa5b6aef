// The numerical core shared verbatim by the CPU path and every HIP kernel.
//
// Every translation unit is compiled with -ffp-contract=off, so these expressions are evaluated with the same rounding
// sequence on host and device: this is what makes the GPU field bit-identical to the CPU path and to itself under every
// domain decomposition (the reference's "1-GPU log == 2-GPU log" property, report.pdf p.15-16 §4.3.1-4.3.2).
#pragma once

#include <cmath>

#include "wave3d/common.hpp"

namespace wave3d {

// h²·Δ_h u: the sum of the three second differences of the 7-point Laplacian at a node with centre value c
// (report.pdf p.5 §2.1). The domain is a cube with the same N on every axis, so the differences share one 1/h² factor,
// which the update formulas fold into their coefficient (Coeffs::lam = τ²/h², half_lam = τ²/(2h²)): 12 instead of 15
// f64 operations per node and step in the hot kernels. The differences keep the reference's form
// (u_{i+1} − 2u_i + u_{i−1}): the 512³ log stays identical to the reference's printed digits, which a neighbour-sum
// form (Σ − 6c) does not (it moves the 7th digit of the L∞ lines).
//
// On the device each difference's first half is one v_fma_f64: 2c is exact (a power-of-two scale), so
// fma(−2, c, xp) rounds the same exact value xp − 2c once, as xp − (2c) does — bit-identical to the host form, one
// f64 operation per node and step fewer (no separate 2c; the leapfrog's 2c − old is fma(2, c, −old) likewise).
W3D_HD double d2sum(double c, double xm, double xp, double ym, double yp, double zm, double zp) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (__builtin_fma(-2.0, c, xp) + xm) + (__builtin_fma(-2.0, c, yp) + ym) + (__builtin_fma(-2.0, c, zp) + zm);
#else
  const double c2 = 2.0 * c;
  return (xp - c2 + xm) + (yp - c2 + ym) + (zp - c2 + zm);
#endif
}

// Leapfrog update u^{n+1} = 2u^n − u^{n−1} + τ² Δ_h u^n (report.pdf p.5 §2.2(3)), with s = d2sum and lam = τ²/h².
// The τ²-term is fused: (2c − old) + lam·s rounded once (one v_fma_f64: 10 instead of 11 f64 operations per node and
// step). Host and device round identically (std::fma is the IEEE fused operation); the printed 128³ / 512³ logs keep
// every digit of the reference's (checked for N = 128, 256, 512 and L = 1, π: profiles/r3/fma_forms.md).
W3D_HD double leapfrog(double c, double old, double s, double lam) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_fma(lam, s, __builtin_fma(2.0, c, -old));
#else
  return std::fma(lam, s, 2.0 * c - old);
#endif
}

// Second-order first step u^1 = u^0 + τ²/2 Δ_h u^0, using ∂u/∂t = 0 (report.pdf p.5 §2.2(2)); half_lam = τ²/(2h²).
// (fused like leapfrog)
W3D_HD double first_step(double c, double s, double half_lam) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_fma(half_lam, s, c);
#else
  return std::fma(half_lam, s, c);
#endif
}

// IEEE fused multiply-add on the host (bindings: the numpy emulators' rounding primitive)
inline double fma_exact(double a, double b, double c) { return std::fma(a, b, c); }

// The error check's analytic value u_a = φ·cos(a_t t) at a node: ((s_x·s_y)·ct)·s_z. The row factor (s_x·s_y)·ct is
// shared by a whole z row (one product per node), and the squared error is accumulated with one fma (err_acc).
W3D_HD double analytic_row(double sx, double sy, double ct) { return (sx * sy) * ct; }
W3D_HD double err_sq_acc(double e, double acc) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_fma(e, e, acc);
#else
  return std::fma(e, e, acc);
#endif
}

// φ at a global node from the separable table (boundary entries are exact zeros, see problem.hpp::sin_table).
W3D_HD double phi(const double* s, i64 gi, i64 gj, i64 gk) { return (s[gi] * s[gj]) * s[gk]; }

}  // namespace wave3d
