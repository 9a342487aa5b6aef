// Stream-capture probe: which multi-stream capture shapes does this HIP runtime accept?
//   hipcc --offload-arch=gfx950 -O2 tools/capture_probe.hip -o build/capture_probe && build/capture_probe P
// Each pattern captures a small multi-stream DAG into a graph, instantiates it, launches it and checks the sums.
//   0  origin g, fork one stream a (normal priority), kernel, join
//   1  as 0 with a high-priority forked stream
//   2  production shape: origin a; b (high priority) waits an event of a, kernel on b, a waits b's event; end on a
//   3  as 2 with b at normal priority
//   4  origin g, fork a and b, kernels on both, join both
//   5  as 4, three units of a→b→a event ping-pong before the join
//   6  production shape over three units: origin a; per unit b waits a's event, kernel on b, a waits b's event
//   7  as 6 with the same two events re-recorded every unit (what GpuSolver does with ev_shell_ / ev_halo_)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                    \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) {                                                                      \
      std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
      std::exit(1);                                                                              \
    }                                                                                            \
  } while (0)

__global__ void k_add(double* p, int n, double v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += v;
}

int main(int argc, char** argv) {
  const int pat = argc > 1 ? std::atoi(argv[1]) : 0;
  const int n = 1024;
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t g, a, b;
  CK(hipStreamCreateWithFlags(&g, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  if (pat == 1 || pat == 2)
    CK(hipStreamCreateWithPriority(&b, hipStreamNonBlocking, hi));
  else
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  hipEvent_t e1, e2, e3, e4;
  for (hipEvent_t* e : {&e1, &e2, &e3, &e4}) CK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  double* d;
  CK(hipMalloc(&d, 2 * n * sizeof(double)));
  CK(hipMemset(d, 0, 2 * n * sizeof(double)));
  auto kern = [&](hipStream_t s, int w) { hipLaunchKernelGGL(k_add, dim3(n / 256), dim3(256), 0, s, d + w * n, n, 1.0); };

  hipGraph_t graph = nullptr;
  hipStream_t origin = g;
  double expect0 = 0, expect1 = 0;
  if (pat == 0 || pat == 1) {
    hipStream_t f = pat == 0 ? a : b;
    CK(hipStreamBeginCapture(g, hipStreamCaptureModeThreadLocal));
    CK(hipEventRecord(e1, g));
    CK(hipStreamWaitEvent(f, e1, 0));
    kern(f, 0);
    expect0 = 1;
    CK(hipEventRecord(e2, f));
    CK(hipStreamWaitEvent(g, e2, 0));
  } else if (pat == 6 || pat == 7) {
    origin = a;
    CK(hipStreamBeginCapture(a, hipStreamCaptureModeThreadLocal));
    hipEvent_t ev[6] = {e1, e2, e3, e4, e1, e2};
    for (int u = 0; u < 3; ++u) {
      hipEvent_t es = pat == 7 ? e1 : ev[2 * u], eh = pat == 7 ? e2 : ev[2 * u + 1];
      if (pat == 6 && u == 2) {
        CK(hipEventCreateWithFlags(&es, hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&eh, hipEventDisableTiming));
      }
      kern(a, 0);
      CK(hipEventRecord(es, a));
      CK(hipStreamWaitEvent(b, es, 0));
      kern(b, 1);
      CK(hipEventRecord(eh, b));
      kern(a, 0);
      CK(hipStreamWaitEvent(a, eh, 0));
      expect0 += 2;
      expect1 += 1;
    }
  } else if (pat == 2 || pat == 3) {
    origin = a;
    CK(hipStreamBeginCapture(a, hipStreamCaptureModeThreadLocal));
    kern(a, 0);
    CK(hipEventRecord(e1, a));
    CK(hipStreamWaitEvent(b, e1, 0));
    kern(b, 1);
    CK(hipEventRecord(e2, b));
    kern(a, 0);
    CK(hipStreamWaitEvent(a, e2, 0));
    kern(a, 1);
    expect0 = 2;
    expect1 = 2;
  } else {
    CK(hipStreamBeginCapture(g, hipStreamCaptureModeThreadLocal));
    CK(hipEventRecord(e1, g));
    CK(hipStreamWaitEvent(a, e1, 0));
    CK(hipStreamWaitEvent(b, e1, 0));
    const int units = pat == 5 ? 3 : 1;
    for (int u = 0; u < units; ++u) {
      kern(a, 0);
      CK(hipEventRecord(e2, a));
      CK(hipStreamWaitEvent(b, e2, 0));
      kern(b, 1);
      CK(hipEventRecord(e3, b));
      CK(hipStreamWaitEvent(a, e3, 0));
      expect0 += 1;
      expect1 += 1;
    }
    CK(hipEventRecord(e3, a));
    CK(hipEventRecord(e4, b));
    CK(hipStreamWaitEvent(g, e3, 0));
    CK(hipStreamWaitEvent(g, e4, 0));
  }
  std::fprintf(stderr, "pattern %d: ending capture\n", pat);
  CK(hipStreamEndCapture(origin, &graph));
  std::fprintf(stderr, "pattern %d: captured\n", pat);
  hipGraphExec_t ex;
  CK(hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ex, origin));
  CK(hipStreamSynchronize(origin));
  double h[2];
  CK(hipMemcpy(&h[0], d, sizeof(double), hipMemcpyDeviceToHost));
  CK(hipMemcpy(&h[1], d + n, sizeof(double), hipMemcpyDeviceToHost));
  std::printf("pattern %d: %s (%g %g, expected %g %g)\n", pat, h[0] == expect0 && h[1] == expect1 ? "ok" : "WRONG", h[0],
              h[1], expect0, expect1);
  return 0;
}
