// wave3d — MI355X-native 3D wave-equation solver.
// Shared basic definitions usable from host C++ (g++) and HIP (hipcc) translation units.
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define W3D_HD __host__ __device__ __forceinline__
#else
#define W3D_HD inline
#endif

namespace wave3d {

using i64 = std::int64_t;

// Throwing check used by host-side planning code (surfaces as Python exceptions through the bindings).
[[noreturn]] inline void fail(const std::string& msg) { throw std::runtime_error("wave3d: " + msg); }

#define W3D_REQUIRE(cond, msg)                         \
  do {                                                 \
    if (!(cond)) ::wave3d::fail(std::string(msg));     \
  } while (0)

W3D_HD i64 ceil_div(i64 a, i64 b) { return (a + b - 1) / b; }
W3D_HD i64 round_up(i64 a, i64 b) { return ceil_div(a, b) * b; }
W3D_HD i64 imin(i64 a, i64 b) { return a < b ? a : b; }
W3D_HD i64 imax(i64 a, i64 b) { return a > b ? a : b; }

}  // namespace wave3d
