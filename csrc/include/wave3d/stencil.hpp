// The numerical core shared verbatim by the CPU path and every HIP kernel.
//
// Every translation unit is compiled with -ffp-contract=off, so these expressions are evaluated with the same rounding
// sequence on host and device: this is what makes the GPU field bit-identical to the CPU path and to itself under every
// domain decomposition (the reference's "1-GPU log == 2-GPU log" property, report.pdf p.15-16 §4.3.1-4.3.2).
#pragma once

#include "wave3d/common.hpp"

namespace wave3d {

// 7-point Laplacian Δ_h u at a node with centre value c (report.pdf p.5 §2.1).
W3D_HD double lap7(double c, double xm, double xp, double ym, double yp, double zm, double zp, double ihx2, double ihy2,
                   double ihz2) {
  const double c2 = 2.0 * c;
  return (xp - c2 + xm) * ihx2 + (yp - c2 + ym) * ihy2 + (zp - c2 + zm) * ihz2;
}

// Leapfrog update u^{n+1} = 2u^n − u^{n−1} + τ² Δ_h u^n (report.pdf p.5 §2.2(3)).
W3D_HD double leapfrog(double c, double old, double lap, double tau2) { return (2.0 * c - old) + tau2 * lap; }

// Second-order first step u^1 = u^0 + τ²/2 Δ_h u^0, using ∂u/∂t = 0 (report.pdf p.5 §2.2(2)).
W3D_HD double first_step(double c, double lap, double half_tau2) { return c + half_tau2 * lap; }

// φ at a global node from the separable table (boundary entries are exact zeros, see problem.hpp::sin_table).
W3D_HD double phi(const double* s, i64 gi, i64 gj, i64 gk) { return (s[gi] * s[gj]) * s[gk]; }

}  // namespace wave3d
