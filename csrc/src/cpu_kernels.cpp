// CPU solver kernels (sequential + OpenMP). See wave3d/cpu.hpp.
//
// Parallelisation is over x-planes. The error reduction keeps one partial per plane and combines the partials in plane
// order, so the result does not depend on the thread count (the reference's tables show identical δ for every thread
// and rank count, report.pdf p.7-11).
#include <omp.h>

#include <cmath>
#include <vector>

#include "wave3d/cpu.hpp"
#include "wave3d/stencil.hpp"

namespace wave3d {

int cpu_set_threads(int n) {
  if (n > 0) omp_set_num_threads(n);
  return omp_get_max_threads();
}
int cpu_max_threads() { return omp_get_max_threads(); }

void cpu_init_first(const Layout& l, const Coeffs& c, const double* s, double* u0, double* u1) {
  const i64 N = l.N;
#pragma omp parallel for schedule(static)
  for (i64 ix = -1; ix <= l.nx; ++ix) {
    const i64 gx = l.gx0 + ix;
    // zero the whole plane first: padding and out-of-domain ghosts stay 0
    double* p0 = u0 + (ix + 1) * l.plane;
    double* p1 = u1 + (ix + 1) * l.plane;
    for (i64 q = 0; q < l.plane; ++q) {
      p0[q] = 0.0;
      p1[q] = 0.0;
    }
    for (i64 iy = -1; iy <= l.ny; ++iy) {
      const i64 gy = l.gy0 + iy;
      for (i64 iz = -1; iz <= l.nz; ++iz) {
        const i64 gz = l.gz0 + iz;
        const i64 o = l.off(ix, iy, iz);
        const double v = phi(s, gx, gy, gz);
        u0[o] = v;
        const bool interior = gx > 0 && gx < N && gy > 0 && gy < N && gz > 0 && gz < N;
        if (interior) {
          const double lap = d2sum(v, phi(s, gx - 1, gy, gz), phi(s, gx + 1, gy, gz), phi(s, gx, gy - 1, gz),
                                  phi(s, gx, gy + 1, gz), phi(s, gx, gy, gz - 1), phi(s, gx, gy, gz + 1));
          u1[o] = first_step(v, lap, c.half_lam);
        } else {
          u1[o] = 0.0;
        }
      }
    }
  }
}

namespace {

template <bool CHECK>
void leapfrog_impl(const Layout& l, const Coeffs& c, const double* cur, double* out, const LBox& b, const double* s,
                   double ct, ErrAcc* acc) {
  const i64 nxp = b.x1 - b.x0;
  std::vector<ErrAcc> part(CHECK ? static_cast<size_t>(nxp) : 0);
  const i64 P = l.plane, R = l.pitch;
#pragma omp parallel for schedule(static)
  for (i64 ix = b.x0; ix < b.x1; ++ix) {
    double emax = 0.0, esum = 0.0;
    const double sx = s[l.gx0 + ix];
    for (i64 iy = b.y0; iy < b.y1; ++iy) {
      const double sxy = analytic_row(sx, s[l.gy0 + iy], ct);
      const i64 row = l.off(ix, iy, 0);
      const double* cr = cur + row;
      double* orow = out + row;
      for (i64 iz = b.z0; iz < b.z1; ++iz) {
        const double u = cr[iz];
        const double lap =
            d2sum(u, cr[iz - P], cr[iz + P], cr[iz - R], cr[iz + R], cr[iz - 1], cr[iz + 1]);
        const double v = leapfrog(u, orow[iz], lap, c.lam);
        orow[iz] = v;
        if (CHECK) {
          const double e = std::fabs(v - sxy * s[l.gz0 + iz]);
          emax = e > emax ? e : emax;
          esum = err_sq_acc(e, esum);
        }
      }
    }
    if (CHECK) part[static_cast<size_t>(ix - b.x0)] = ErrAcc{emax, esum};
  }
  if (CHECK) {
    for (const auto& p : part) {
      acc->max = p.max > acc->max ? p.max : acc->max;
      acc->sum += p.sum;
    }
  }
}

}  // namespace

void cpu_leapfrog(const Layout& l, const Coeffs& c, const double* cur, double* old_out, const LBox& box,
                  const double* s, double ct, ErrAcc* acc) {
  if (box.empty()) return;
  if (acc)
    leapfrog_impl<true>(l, c, cur, old_out, box, s, ct, acc);
  else
    leapfrog_impl<false>(l, c, cur, old_out, box, s, ct, nullptr);
}

void cpu_error(const Layout& l, const double* u, const LBox& b, const double* s, double ct, ErrAcc* acc) {
  if (b.empty()) return;
  const i64 nxp = b.x1 - b.x0;
  std::vector<ErrAcc> part(static_cast<size_t>(nxp));
#pragma omp parallel for schedule(static)
  for (i64 ix = b.x0; ix < b.x1; ++ix) {
    double emax = 0.0, esum = 0.0;
    const double sx = s[l.gx0 + ix];
    for (i64 iy = b.y0; iy < b.y1; ++iy) {
      const double sxy = analytic_row(sx, s[l.gy0 + iy], ct);
      for (i64 iz = b.z0; iz < b.z1; ++iz) {
        const double e = std::fabs(u[l.off(ix, iy, iz)] - sxy * s[l.gz0 + iz]);
        emax = e > emax ? e : emax;
        esum = err_sq_acc(e, esum);
      }
    }
    part[static_cast<size_t>(ix - b.x0)] = ErrAcc{emax, esum};
  }
  for (const auto& p : part) {
    acc->max = p.max > acc->max ? p.max : acc->max;
    acc->sum += p.sum;
  }
}

void cpu_pack_face(const Layout& l, const Face& f, const double* u, double* buf) {
  if (f.axis == 1) {
#pragma omp parallel for schedule(static)
    for (i64 ix = 0; ix < l.nx; ++ix)
      for (i64 iz = 0; iz < l.nz; ++iz) buf[ix * l.nz + iz] = u[l.off(ix, f.send_layer, iz)];
  } else if (f.axis == 2) {
#pragma omp parallel for schedule(static)
    for (i64 ix = 0; ix < l.nx; ++ix)
      for (i64 iy = 0; iy < l.ny; ++iy) buf[ix * l.ny + iy] = u[l.off(ix, iy, f.send_layer)];
  } else {
    const double* src = u + f.send_off;
    for (i64 q = 0; q < f.count; ++q) buf[q] = src[q];
  }
}

void cpu_unpack_face(const Layout& l, const Face& f, const double* buf, double* u) {
  if (f.axis == 1) {
#pragma omp parallel for schedule(static)
    for (i64 ix = 0; ix < l.nx; ++ix)
      for (i64 iz = 0; iz < l.nz; ++iz) u[l.off(ix, f.recv_layer, iz)] = buf[ix * l.nz + iz];
  } else if (f.axis == 2) {
#pragma omp parallel for schedule(static)
    for (i64 ix = 0; ix < l.nx; ++ix)
      for (i64 iy = 0; iy < l.ny; ++iy) u[l.off(ix, iy, f.recv_layer)] = buf[ix * l.ny + iy];
  } else {
    double* dst = u + f.recv_off;
    for (i64 q = 0; q < f.count; ++q) dst[q] = buf[q];
  }
}

}  // namespace wave3d
