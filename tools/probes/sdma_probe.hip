// Runtime probe: can halo copies run on the copy engines (SDMA) while an LDS-bound kernel holds every CU, and which
// stream operations around them survive graph capture on this HIP runtime?
//
//   hipcc --offload-arch=gfx950 -O2 tools/probes/sdma_probe.hip -o build/sdma_probe && build/sdma_probe
//
// Prints one line per measurement:
//   copy-alone   kind, MB, µs, GB/s            hipMemcpyAsync D2D (default kind = blit kernel) vs NoCU (copy engine)
//   busy-alone   µs                            a kernel with one 1024-thread / 128 KiB-LDS workgroup per CU
//   overlap      kind, kernel µs, copy µs      both at once on two streams (copy on a high-priority stream)
//   rect         kind, ok, µs                  hipMemcpy3DAsync of a sub-box between two pitched arrays
//   capture      what, hipError                memops / NoCU copies inside hipStreamBeginCapture .. EndCapture + launch
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      std::printf("FAIL %s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);             \
      std::exit(1);                                                                           \
    }                                                                                         \
  } while (0)

// streams through a buffer repeatedly, one workgroup per CU (128 KiB of LDS keeps a second one off the CU)
__global__ __launch_bounds__(1024) void k_busy(const double* __restrict__ a, double* __restrict__ b, long n, int reps) {
  extern __shared__ double lds[];
  double acc = 0.0;
  for (int r = 0; r < reps; ++r)
    for (long i = blockIdx.x * 1024L + threadIdx.x; i < n; i += gridDim.x * 1024L) {
      const double v = a[i];
      lds[threadIdx.x] = v;
      __syncthreads();
      acc += lds[(threadIdx.x + 1) & 1023];
      __syncthreads();
    }
  b[blockIdx.x * 1024L + threadIdx.x] = acc;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  int rtv = 0;
  CK(hipRuntimeGetVersion(&rtv));
  std::printf("device CUs %d, HIP runtime %d\n", ncu, rtv);
  const size_t big = 512ull << 20;  // busy kernel's buffer
  double *a = nullptr, *b = nullptr, *src = nullptr, *dst = nullptr;
  CK(hipMalloc(&a, big));
  CK(hipMalloc(&b, 64ull << 20));
  CK(hipMemset(a, 0, big));
  const size_t cmax = 64ull << 20;
  CK(hipMalloc(&src, cmax));
  CK(hipMalloc(&dst, cmax));
  CK(hipMemset(src, 1, cmax));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_busy), hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  hipStream_t sk, sc;
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  CK(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking));
  CK(hipStreamCreateWithPriority(&sc, hipStreamNonBlocking, hi));
  hipEvent_t e0, e1, e2, e3;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  CK(hipEventCreate(&e3));

  auto time_copy = [&](hipMemcpyKind kind, size_t bytes, int reps) {
    CK(hipMemcpyAsync(dst, src, bytes, kind, sc));
    CK(hipStreamSynchronize(sc));
    CK(hipEventRecord(e0, sc));
    for (int r = 0; r < reps; ++r) CK(hipMemcpyAsync(dst, src, bytes, kind, sc));
    CK(hipEventRecord(e1, sc));
    CK(hipStreamSynchronize(sc));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return 1e3 * ms / reps;
  };
  const hipMemcpyKind kinds[2] = {hipMemcpyDeviceToDevice, hipMemcpyDeviceToDeviceNoCU};
  const char* kname[2] = {"D2D", "D2D-NoCU"};
  for (int k = 0; k < 2; ++k)
    for (size_t mb : {1, 2, 4, 8, 16, 32}) {
      const double us = time_copy(kinds[k], mb << 20, 20);
      std::printf("copy-alone %s %zu MB %.1f us %.1f GB/s\n", kname[k], mb, us, (mb << 20) / us * 1e-3);
    }

  const long n = static_cast<long>(big / sizeof(double));
  const int reps = 4;
  auto busy = [&](hipStream_t s) {
    hipLaunchKernelGGL(k_busy, dim3(ncu), dim3(1024), 131072, s, a, b, n, reps);
  };
  busy(sk);
  CK(hipStreamSynchronize(sk));
  CK(hipEventRecord(e0, sk));
  busy(sk);
  CK(hipEventRecord(e1, sk));
  CK(hipStreamSynchronize(sk));
  float kms = 0;
  CK(hipEventElapsedTime(&kms, e0, e1));
  std::printf("busy-alone %.1f us (%.2f TB/s)\n", kms * 1e3, reps * big / (kms * 1e-3) * 1e-12);

  for (int k = 0; k < 2; ++k)
    for (size_t mb : {2, 8, 16}) {
      const size_t bytes = mb << 20;
      const int nc = 8;
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, sk));
      busy(sk);
      CK(hipEventRecord(e1, sk));
      // the copies start once the kernel is resident
      CK(hipEventRecord(e2, sc));
      for (int r = 0; r < nc; ++r) CK(hipMemcpyAsync(dst, src, bytes, kinds[k], sc));
      CK(hipEventRecord(e3, sc));
      CK(hipDeviceSynchronize());
      float km = 0, cm = 0, span = 0;
      CK(hipEventElapsedTime(&km, e0, e1));
      CK(hipEventElapsedTime(&cm, e2, e3));
      CK(hipEventElapsedTime(&span, e0, e3));
      std::printf("overlap %s %zu MB x%d: kernel %.1f us (alone %.1f), copies %.1f us (%.1f GB/s), copies end %.1f us "
                  "after kernel start\n",
                  kname[k], mb, nc, km * 1e3, kms * 1e3, cm * 1e3, nc * bytes / (cm * 1e-3) * 1e-9, span * 1e3);
    }

  // sub-box copy between two pitched 3-D arrays (a y-face slab of a block rank: rows of 256 doubles, and a z-face:
  // rows of 4 doubles)
  for (int k = 0; k < 2; ++k)
    for (int zrow : {256, 4}) {
      const size_t pitch = 272 * sizeof(double), ny = 264, nx = 260;
      hipMemcpy3DParms p{};
      p.srcPtr = make_hipPitchedPtr(src, pitch, pitch, ny);
      p.dstPtr = make_hipPitchedPtr(dst, pitch, pitch, ny);
      p.srcPos = make_hipPos(8 * sizeof(double), 4, 4);
      p.dstPos = make_hipPos(8 * sizeof(double), 0, 4);
      p.extent = make_hipExtent(zrow * sizeof(double), zrow == 256 ? 4 : 256, 256);
      p.kind = kinds[k];
      (void)nx;
      hipError_t e = hipMemcpy3DAsync(&p, sc);
      hipError_t e2s = hipStreamSynchronize(sc);
      float ms = 0;
      if (e == hipSuccess && e2s == hipSuccess) {
        CK(hipEventRecord(e0, sc));
        for (int r = 0; r < 10; ++r) (void)hipMemcpy3DAsync(&p, sc);
        CK(hipEventRecord(e1, sc));
        CK(hipStreamSynchronize(sc));
        CK(hipEventElapsedTime(&ms, e0, e1));
      }
      const double bytes = double(p.extent.width) * p.extent.height * p.extent.depth;
      std::printf("rect %s row %d doubles: %s / %s, %.1f us, %.2f GB/s\n", kname[k], zrow, hipGetErrorString(e),
                  hipGetErrorString(e2s), ms * 100.0, bytes / (ms * 1e-4) * 1e-9);
      (void)hipGetLastError();
    }

  // graph capture of stream memops and NoCU copies
  unsigned* flag = nullptr;
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&flag), 64, hipDeviceMallocUncached));
  CK(hipMemset(flag, 0, 64));
  auto try_capture = [&](const char* what, auto body) {
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    hipError_t eb = hipStreamBeginCapture(sc, hipStreamCaptureModeThreadLocal);
    hipError_t ei = hipSuccess;
    if (eb == hipSuccess) ei = body();
    hipError_t ee = hipStreamEndCapture(sc, &g);
    hipError_t en = g ? hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) : hipErrorUnknown;
    hipError_t el = ge ? hipGraphLaunch(ge, sc) : hipErrorUnknown;
    hipError_t es = hipStreamSynchronize(sc);
    std::printf("capture %s: begin %s, op %s, end %s, instantiate %s, launch %s, sync %s\n", what,
                hipGetErrorString(eb), hipGetErrorString(ei), hipGetErrorString(ee), hipGetErrorString(en),
                hipGetErrorString(el), hipGetErrorString(es));
    if (ge) (void)hipGraphExecDestroy(ge);
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
  };
  try_capture("write-value32", [&] { return hipStreamWriteValue32(sc, flag, 7, 0); });
  unsigned hv = 0;
  CK(hipMemcpy(&hv, flag, 4, hipMemcpyDeviceToHost));
  std::printf("flag after captured write: %u\n", hv);
  try_capture("wait-value32 (satisfied)", [&] { return hipStreamWaitValue32(sc, flag, 7, hipStreamWaitValueGte, 0xFFFFFFFFu); });
  try_capture("memcpy NoCU", [&] { return hipMemcpyAsync(dst, src, 8 << 20, hipMemcpyDeviceToDeviceNoCU, sc); });
  {  // stream memops eager: write then wait on one stream, and cross-stream wait released by a write
    CK(hipMemset(flag, 0, 64));
    const double t0 = now_us();
    CK(hipStreamWaitValue32(sk, flag + 1, 5, hipStreamWaitValueGte, 0xFFFFFFFFu));
    busy(sk);
    CK(hipMemcpyAsync(dst, src, 8 << 20, hipMemcpyDeviceToDeviceNoCU, sc));
    CK(hipStreamWriteValue32(sc, flag + 1, 5, 0));
    CK(hipStreamSynchronize(sk));
    std::printf("eager wait released by a write on another stream after a NoCU copy: %.1f us\n", now_us() - t0);
  }
  // a timed memop round trip: write on one stream, wait on another, event around
  {
    CK(hipMemset(flag, 0, 64));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, sc));
    for (unsigned v = 1; v <= 100; ++v) {
      CK(hipStreamWriteValue32(sc, flag + 2, v, 0));
      CK(hipStreamWaitValue32(sk, flag + 2, v, hipStreamWaitValueGte, 0xFFFFFFFFu));
      CK(hipStreamWaitValue32(sc, flag + 2, v, hipStreamWaitValueGte, 0xFFFFFFFFu));
    }
    CK(hipEventRecord(e1, sc));
    CK(hipDeviceSynchronize());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("memop write+wait pair: %.2f us each\n", ms * 10.0);
  }
  // copy engines in parallel: 32 MB split into k chunks on k streams (does each stream get its own engine?)
  {
    std::vector<hipStream_t> ss(8);
    for (auto& s : ss) CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi));
    for (int k : {1, 2, 4, 8}) {
      const size_t total = 32ull << 20, chunk = total / k;
      for (int warm = 0; warm < 2; ++warm) {
        CK(hipDeviceSynchronize());
        const double t0 = now_us();
        for (int r = 0; r < 4; ++r)
          for (int c = 0; c < k; ++c)
            CK(hipMemcpyAsync(reinterpret_cast<char*>(dst) + c * chunk, reinterpret_cast<char*>(src) + c * chunk, chunk,
                              hipMemcpyDeviceToDeviceNoCU, ss[c]));
        CK(hipDeviceSynchronize());
        const double us = now_us() - t0;
        if (warm) std::printf("parallel NoCU %d streams: 4 x 32 MB in %.1f us = %.1f GB/s\n", k, us, 4 * total / us * 1e-3);
      }
    }
    for (auto& s : ss) CK(hipStreamDestroy(s));
  }
  // a captured NoCU copy: still on the copy engine (time ~ the eager NoCU copy) or turned into a blit kernel?
  {
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    CK(hipStreamBeginCapture(sc, hipStreamCaptureModeThreadLocal));
    for (int r = 0; r < 4; ++r) CK(hipMemcpyAsync(dst, src, 8 << 20, hipMemcpyDeviceToDeviceNoCU, sc));
    CK(hipStreamEndCapture(sc, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, sc));
    CK(hipStreamSynchronize(sc));
    CK(hipEventRecord(e0, sc));
    CK(hipGraphLaunch(ge, sc));
    CK(hipEventRecord(e1, sc));
    CK(hipStreamSynchronize(sc));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("captured NoCU 4 x 8 MB: %.1f us (%.1f GB/s)\n", ms * 1e3, 4 * (8 << 20) / (ms * 1e-3) * 1e-9);
    // same graph while the busy kernel holds the CUs
    CK(hipEventRecord(e0, sk));
    busy(sk);
    CK(hipEventRecord(e1, sk));
    CK(hipEventRecord(e2, sc));
    CK(hipGraphLaunch(ge, sc));
    CK(hipEventRecord(e3, sc));
    CK(hipDeviceSynchronize());
    float km = 0, cm = 0;
    CK(hipEventElapsedTime(&km, e0, e1));
    CK(hipEventElapsedTime(&cm, e2, e3));
    std::printf("captured NoCU under busy kernel: kernel %.1f us, copies %.1f us\n", km * 1e3, cm * 1e3);
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
  }
  std::printf("done\n");
  return 0;
}
