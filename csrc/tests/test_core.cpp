// Native unit tests of the host-side core (no GPU): decomposition, layout, halo plans, scheme, CPU solver.
//
// SURVEY.md §4.2 "unit (C++/ctest)": exact-arithmetic checks of the pieces every backend shares. Built and run by
// CMake/ctest (CMakeLists.txt) and, with host AddressSanitizer + UBSan, by tests/test_native_unit.py.
// Exit status 0 = all checks passed; every failure prints its location.
#include <cmath>
#include <cstdio>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "wave3d/cpu.hpp"
#include "wave3d/decomp.hpp"
#include "wave3d/problem.hpp"
#include "wave3d/stencil.hpp"

using namespace wave3d;

namespace {

int g_fail = 0, g_checks = 0;

#define CHECK(cond)                                                          \
  do {                                                                       \
    ++g_checks;                                                              \
    if (!(cond)) {                                                           \
      ++g_fail;                                                              \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
    }                                                                        \
  } while (0)

template <class F>
bool throws(F&& f) {
  try {
    f();
  } catch (const std::exception&) {
    return true;
  }
  return false;
}

// split_axis: the parts tile 0..N exactly once, interior work differs by at most one node between parts
void test_split_axis() {
  for (i64 N : {2, 3, 7, 64, 127, 512, 2048}) {
    for (int p = 1; p <= 32; ++p) {
      if (p > N - 1) continue;
      i64 expect = 0, mn = 1 << 30, mx = 0;
      for (int c = 0; c < p; ++c) {
        i64 b = 0, e = 0;
        split_axis(N, p, c, &b, &e);
        CHECK(b == expect);
        CHECK(e > b);
        expect = e;
        const i64 work = std::min(e, N) - std::max<i64>(b, 1);
        mn = std::min(mn, work);
        mx = std::max(mx, work);
      }
      CHECK(expect == N + 1);
      CHECK(mx - mn <= 1);
    }
  }
}

// every decomposition: boxes partition the grid, neighbours are adjacent, x faces contiguous, y/z faces packed
void test_decompositions() {
  const std::vector<std::pair<std::string, int>> cases = {
      {"slab", 1}, {"slab", 2}, {"slab", 3}, {"slab", 8}, {"slab", 16}, {"block", 4}, {"block", 7},
      {"block", 8}, {"block", 10}, {"block", 20}, {"block", 32}, {"2x2x2", 8}, {"1x2x3", 6}, {"4x1x2", 8}};
  for (const auto& [spec, P] : cases) {
    for (i64 N : {40, 65}) {
      Problem pr;
      pr.N = N;
      const Dims d = parse_dims(spec, P, N);
      CHECK(d.size() == P);
      i64 total = 0;
      for (int r = 0; r < P; ++r) {
        const Box b = rank_box(pr, d, r);
        total += b.count();
        for (int axis = 0; axis < 3; ++axis)
          for (int side = 0; side < 2; ++side) {
            const int q = neighbor_rank(d, r, axis, side);
            if (q < 0) continue;
            CHECK(neighbor_rank(d, q, axis, 1 - side) == r);
            const Box c = rank_box(pr, d, q);
            const i64 lo[3] = {b.x0, b.y0, b.z0}, hi[3] = {b.x1, b.y1, b.z1};
            const i64 clo[3] = {c.x0, c.y0, c.z0}, chi[3] = {c.x1, c.y1, c.z1};
            CHECK(side ? chi[axis] > hi[axis] && clo[axis] == hi[axis] : chi[axis] == lo[axis]);
          }
        // halo plan: message sizes agree with the peer's matching face
        const Layout l = make_layout(pr, b);
        const HaloPlan h = make_halo_plan(l, d, r);
        for (const Face& f : h.faces) {
          const Layout lq = make_layout(pr, rank_box(pr, d, f.peer));
          const HaloPlan hq = make_halo_plan(lq, d, f.peer);
          int matches = 0;
          for (const Face& g : hq.faces)
            if (g.peer == r && g.axis == f.axis && g.side == 1 - f.side) {
              ++matches;
              CHECK(g.count == f.count);
            }
          CHECK(matches == 1);
          CHECK(f.contiguous == (f.axis == 0));
        }
      }
      CHECK(total == (N + 1) * (N + 1) * (N + 1));
    }
  }
  CHECK(throws([] { parse_dims("2x2x3", 8, 64); }));
  CHECK(throws([] { parse_dims("pencil", 8, 64); }));
  const Dims b8 = block_dims(8, 512);
  CHECK(b8.px == 2 && b8.py == 2 && b8.pz == 2);
}

// layout: 64-bit offsets at 2049³, 128-byte aligned rows, first updated node of a row on a line boundary
void test_layout() {
  Problem pr;
  pr.N = 2048;
  const Layout l = make_layout(pr, rank_box(pr, Dims{1, 1, 1}, 0));
  CHECK(l.total > (i64{1} << 33));  // > 8.6e9 doubles: needs 64-bit indexing
  CHECK(l.off(l.nx, l.ny, l.nz) < l.total);
  CHECK(l.off(-1, -1, -1) >= 0);
  CHECK(l.pitch % 16 == 0);
  CHECK((l.cz0 + 1 + l.zs) % 16 == 0);
  for (i64 xg : {1, 2, 4}) {
    pr.N = 70;
    const Layout m = make_layout(pr, rank_box(pr, Dims{3, 1, 1}, 1), 16, xg);
    CHECK(m.plane_off(-xg) == 0);
    CHECK(m.plane_off(m.nx + xg) == m.total);
    CHECK(m.off(0, 0, 0) == m.plane_off(0) + m.pitch + 1 + m.zs);
    for (i64 x = -xg; x <= m.nx + xg - 1; ++x) CHECK(m.kbase() + (x + 1) * m.plane == m.plane_off(x));  // kernel base
  }
}

// Δ_h is exact on quadratics when h is a power of two: u = x² + 2y² + 3z² → Δu = 12
void test_lap7_quadratic() {  // d2sum · 1/h²
  const double h = 1.0 / 64.0, ih2 = 1.0 / (h * h);
  auto u = [&](int i, int j, int k) {
    const double x = i * h, y = j * h, z = k * h;
    return x * x + 2.0 * y * y + 3.0 * z * z;
  };
  for (int i = 1; i < 10; ++i)
    for (int j = 1; j < 10; ++j)
      for (int k = 1; k < 10; ++k) {
        const double v = d2sum(u(i, j, k), u(i - 1, j, k), u(i + 1, j, k), u(i, j - 1, k), u(i, j + 1, k),
                              u(i, j, k - 1), u(i, j, k + 1));
        CHECK(v * ih2 == 12.0);
      }
  // the leapfrog and first-step formulas
  CHECK(leapfrog(1.5, 0.5, 2.0, 0.25) == 3.0);
  CHECK(first_step(1.0, 4.0, 0.125) == 1.5);
}

void test_problem() {
  Problem p;
  p.N = 512;
  p.tau = 1e-3;
  CHECK(p.cfl_ok());
  CHECK(std::fabs(p.courant() - 0.001 * std::sqrt(3.0) * 512) < 1e-12);
  p.N = 1024;
  CHECK(!p.cfl_ok());  // τ = 1e-3 diverges from N ≈ 578 up
  p.N = 2048;
  p.tau = 2.5e-4;
  CHECK(p.cfl_ok());
  CHECK(p.cell_updates() == 2048.0 * 2048.0 * 2048.0 * 20.0);
  const std::vector<double> s = sin_table_ext(p);
  CHECK(s.size() == static_cast<size_t>(p.N + 3));
  CHECK(s[0] == 0.0 && s[1] == 0.0 && s[static_cast<size_t>(p.N + 1)] == 0.0 && s[static_cast<size_t>(p.N + 2)] == 0.0);
  CHECK(std::fabs(s[static_cast<size_t>(p.N / 2 + 1)] - 1.0) < 1e-15);
  Problem bad;
  bad.N = 1;
  CHECK(throws([&] { bad.validate(); }));
  bad.N = 8;
  bad.tau = -1.0;
  CHECK(throws([&] { bad.validate(); }));
}

// pack → unpack moves a y/z face into the peer's ghost layer and nothing else
void test_pack_unpack() {
  Problem pr;
  pr.N = 20;
  const Dims d{1, 2, 2};
  const Box b = rank_box(pr, d, 0);
  const Layout l = make_layout(pr, b);
  const HaloPlan h = make_halo_plan(l, d, 0);
  std::vector<double> u(static_cast<size_t>(l.total));
  for (size_t i = 0; i < u.size(); ++i) u[i] = static_cast<double>(i);
  for (const Face& f : h.faces) {
    std::vector<double> buf(static_cast<size_t>(f.count));
    cpu_pack_face(l, f, u.data(), buf.data());
    std::vector<double> v(static_cast<size_t>(l.total), -1.0);
    cpu_unpack_face(l, f, buf.data(), v.data());
    i64 written = 0;
    for (size_t i = 0; i < v.size(); ++i) written += v[i] != -1.0;
    CHECK(written == f.count);
    // the value at ghost (x, recv_layer, z) came from (x, send_layer, z)
    if (f.axis == 1) CHECK(v[static_cast<size_t>(l.off(3, f.recv_layer, 4))] == u[static_cast<size_t>(l.off(3, f.send_layer, 4))]);
    if (f.axis == 2) CHECK(v[static_cast<size_t>(l.off(3, 4, f.recv_layer))] == u[static_cast<size_t>(l.off(3, 4, f.send_layer))]);
  }
}

// CPU solver at the reference's sequential config (128³, τ = 1e-3, K = 20): the closed-form oracle values that the
// golden tests pin, all printed digits
void test_cpu_solver_golden() {
  Problem p;
  p.N = 128;
  p.tau = 1e-3;
  p.K = 20;
  CpuSolver s(p, 2, 0);
  const CpuResult r = s.run();
  CHECK(r.steps.size() == 10 && r.steps.back() == 20);
  char buf[64];
  std::snprintf(buf, sizeof buf, "%.6e %.6e", r.max_err.back(), r.rms_err.back());
  CHECK(std::string(buf) == "2.820954e-07 1.009161e-07");
  CHECK(r.finite);
  // boundary nodes are never written: the Dirichlet faces stay exact zeros
  const Layout& l = s.layout();
  const std::vector<double>& u = s.field(0);
  for (i64 j = 0; j <= p.N; j += 7)
    for (i64 k = 0; k <= p.N; k += 5) {
      CHECK(u[static_cast<size_t>(l.off(0, j, k))] == 0.0);
      CHECK(u[static_cast<size_t>(l.off(p.N, j, k))] == 0.0);
    }
}

}  // namespace

int main() {
  test_split_axis();
  test_decompositions();
  test_layout();
  test_lap7_quadratic();
  test_problem();
  test_pack_unpack();
  test_cpu_solver_golden();
  std::printf("test_core: %d checks, %d failed\n", g_checks, g_fail);
  return g_fail == 0 ? 0 : 1;
}
