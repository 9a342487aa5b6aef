// The numerical core shared verbatim by the CPU path and every HIP kernel.
//
// Every translation unit is compiled with -ffp-contract=off, so these expressions are evaluated with the same rounding
// sequence on host and device: this is what makes the GPU field bit-identical to the CPU path and to itself under every
// domain decomposition (the reference's "1-GPU log == 2-GPU log" property, report.pdf p.15-16 §4.3.1-4.3.2).
#pragma once

#include "wave3d/common.hpp"

namespace wave3d {

// 7-point Laplacian Δ_h u at a node with centre value c (report.pdf p.5 §2.1). The domain is a cube with the same N
// on every axis (Coeffs::from: ihx2 = ihy2 = ihz2), so the three second differences share one 1/h² factor: one
// multiply instead of three (13 instead of 15 f64 operations per node and step in the hot kernels). The second
// differences keep the reference's form (u_{i+1} − 2u_i + u_{i−1}): the 512³ log stays identical to the reference's
// printed digits, which a neighbour-sum form (Σ − 6c) does not (it moves the 7th digit of the L∞ lines).
W3D_HD double lap7(double c, double xm, double xp, double ym, double yp, double zm, double zp, double ihx2, double ihy2,
                   double ihz2) {
  (void)ihy2;
  (void)ihz2;
  const double c2 = 2.0 * c;
  return ((xp - c2 + xm) + (yp - c2 + ym) + (zp - c2 + zm)) * ihx2;
}

// Leapfrog update u^{n+1} = 2u^n − u^{n−1} + τ² Δ_h u^n (report.pdf p.5 §2.2(3)).
W3D_HD double leapfrog(double c, double old, double lap, double tau2) { return (2.0 * c - old) + tau2 * lap; }

// Second-order first step u^1 = u^0 + τ²/2 Δ_h u^0, using ∂u/∂t = 0 (report.pdf p.5 §2.2(2)).
W3D_HD double first_step(double c, double lap, double half_tau2) { return c + half_tau2 * lap; }

// φ at a global node from the separable table (boundary entries are exact zeros, see problem.hpp::sin_table).
W3D_HD double phi(const double* s, i64 gi, i64 gj, i64 gk) { return (s[gi] * s[gj]) * s[gk]; }

}  // namespace wave3d
