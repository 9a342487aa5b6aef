// Launch helpers of the pair-tiled S-step pass (k_leapfrog_p2), shared by its instantiation translation units
// (kernels_leapfrog_p2*.hip: one per stage count, compiled in parallel).
#pragma once

#include "wave3d/leapfrog_p2_kernel.hpp"

namespace wave3d {
namespace p2k {

// instantiated check supersets per S: none, even levels, odd levels, all (checks every 2nd step hit one parity)
template <int S>
constexpr int kFull = (1 << S) - 1;
template <int S>
constexpr int kEven = 0b01010 & kFull<S>;
template <int S>
constexpr int kOdd = 0b10101 & kFull<S>;

// the kernel's static LDS (the reduction arrays) as laid out, and the dynamic limit it leaves
template <int S, int CM, bool INIT, bool CH>
size_t prepare_cfg() {
  static const size_t limit = [] {
    const void* fn = reinterpret_cast<const void*>(k_leapfrog_p2<S, CM, INIT, CH>);
    hipFuncAttributes fa{};
    hipError_t e = hipFuncGetAttributes(&fa, fn);
    if (e != hipSuccess) fail(std::string("leapfrog_p2 attributes: ") + hipGetErrorString(e));
    const size_t lim = 160 * 1024 - fa.sharedSizeBytes;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lim));
    if (e != hipSuccess) fail(std::string("leapfrog_p2 LDS attribute: ") + hipGetErrorString(e));
    return lim;
  }();
  return limit;
}

template <int S, int CM, bool INIT>
void launch_cfg(const P2Params& p, int nblocks, hipStream_t st) {
  const size_t shmem = p2_lds_bytes<S>((p.check_mask || INIT) ? p2_nxt<S>(p.xlen_max) : 0);
  if (p.chunked) {
    const size_t lim = prepare_cfg<S, CM, INIT, true>();
    W3D_REQUIRE(shmem <= lim, "leapfrog_p2: too many planes for the LDS sin table");
    hipLaunchKernelGGL((k_leapfrog_p2<S, CM, INIT, true>), dim3(nblocks), dim3(kNT), shmem, st, p);
  } else {
    const size_t lim = prepare_cfg<S, CM, INIT, false>();
    W3D_REQUIRE(shmem <= lim, "leapfrog_p2: too many planes for the LDS sin table");
    hipLaunchKernelGGL((k_leapfrog_p2<S, CM, INIT, false>), dim3(nblocks), dim3(kNT), shmem, st, p);
  }
}

template <int S, bool INIT>
void launch_cm(const P2Params& p, int nblocks, hipStream_t st) {
  const int m = p.check_mask;
  if (m == 0)
    launch_cfg<S, 0, INIT>(p, nblocks, st);
  else if ((m & ~kEven<S>) == 0)
    launch_cfg<S, kEven<S>, INIT>(p, nblocks, st);
  else if ((m & ~kOdd<S>) == 0)
    launch_cfg<S, kOdd<S>, INIT>(p, nblocks, st);
  else
    launch_cfg<S, kFull<S>, INIT>(p, nblocks, st);
}

template <int S, bool INIT>
void prepare_all() {
  prepare_cfg<S, 0, INIT, false>();
  prepare_cfg<S, kEven<S>, INIT, false>();
  prepare_cfg<S, kOdd<S>, INIT, false>();
  prepare_cfg<S, kFull<S>, INIT, false>();
  prepare_cfg<S, 0, INIT, true>();
  prepare_cfg<S, kEven<S>, INIT, true>();
  prepare_cfg<S, kOdd<S>, INIT, true>();
  prepare_cfg<S, kFull<S>, INIT, true>();
}

// per-S entry points (one translation unit each)
void launch_p2_s2(const P2Params& p, int nblocks, bool init, hipStream_t st);
void launch_p2_s3(const P2Params& p, int nblocks, bool init, hipStream_t st);
void launch_p2_s4(const P2Params& p, int nblocks, bool init, hipStream_t st);
void launch_p2_s5(const P2Params& p, int nblocks, bool init, hipStream_t st);
void prepare_p2_s2();
void prepare_p2_s3();
void prepare_p2_s4();
void prepare_p2_s5();

}  // namespace p2k
}  // namespace wave3d
