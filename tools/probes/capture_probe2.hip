// Stream-capture probe 2: the in-process group shape (R ranks × two streams forked from one origin), with the
// cross-stream event waits selected by bit flags:
//   bit0 fence: s0[r] waits the peer's halo event   bit1 fence: s1[r] waits the peer's halo event
//   bit2 interior: s0[r] waits its own halo event    bit3 one rank (the peer is the rank itself)
//   bit4 no explicit s1 fork (s1 joins through the shell event)
//   bit5 fence through the origin: g joins every halo event, s0/s1 of every rank wait g's event
//   bit6 pull through the origin: g joins every shell event, every s1 waits g's event
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

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
  const int f = argc > 1 ? std::atoi(argv[1]) : 0;
  const int n = 1024, R = (f & 8) ? 1 : 2;
  hipStream_t g;
  CK(hipStreamCreateWithFlags(&g, hipStreamNonBlocking));
  std::vector<hipStream_t> s0(R), s1(R);
  std::vector<hipEvent_t> ea(R), eb(R), ej(2 * R);
  for (int r = 0; r < R; ++r) {
    CK(hipStreamCreateWithFlags(&s0[r], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1[r], hipStreamNonBlocking));
    for (hipEvent_t* e : {&ea[r], &eb[r], &ej[2 * r], &ej[2 * r + 1]}) CK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  hipEvent_t fork, allp, allh;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&allp, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&allh, hipEventDisableTiming));
  double* d;
  CK(hipMalloc(&d, 4 * n * sizeof(double)));
  CK(hipMemset(d, 0, 4 * n * sizeof(double)));
  auto kern = [&](hipStream_t s, int w) { hipLaunchKernelGGL(k_add, dim3(n / 256), dim3(256), 0, s, d + w * n, n, 1.0); };
  hipGraph_t graph = nullptr;
  CK(hipStreamBeginCapture(g, hipStreamCaptureModeThreadLocal));
  CK(hipEventRecord(fork, g));
  for (int r = 0; r < R; ++r) {
    CK(hipStreamWaitEvent(s0[r], fork, 0));
    if (!(f & 16)) CK(hipStreamWaitEvent(s1[r], fork, 0));
  }
  for (int r = 0; r < R; ++r) {
    kern(s0[r], r);
    CK(hipEventRecord(ea[r], s0[r]));
    CK(hipStreamWaitEvent(s1[r], ea[r], 0));
  }
  if (f & 64) {
    for (int r = 0; r < R; ++r) CK(hipStreamWaitEvent(g, ea[r], 0));
    CK(hipEventRecord(allp, g));
    for (int r = 0; r < R; ++r) CK(hipStreamWaitEvent(s1[r], allp, 0));
  }
  for (int r = 0; r < R; ++r) {
    kern(s1[r], 2 + r);
    CK(hipEventRecord(eb[r], s1[r]));
  }
  for (int r = 0; r < R; ++r) {
    const int q = (r + 1) % R;
    if (f & 1) CK(hipStreamWaitEvent(s0[r], eb[q], 0));
    if (f & 2) CK(hipStreamWaitEvent(s1[r], eb[q], 0));
  }
  if (f & 32) {
    for (int r = 0; r < R; ++r) CK(hipStreamWaitEvent(g, eb[r], 0));
    CK(hipEventRecord(allh, g));
    for (int r = 0; r < R; ++r) {
      CK(hipStreamWaitEvent(s0[r], allh, 0));
      CK(hipStreamWaitEvent(s1[r], allh, 0));
    }
  }
  for (int r = 0; r < R; ++r) {
    if (f & 4) CK(hipStreamWaitEvent(s0[r], eb[r], 0));
    kern(s0[r], r);
  }
  for (int r = 0; r < R; ++r) {
    CK(hipEventRecord(ej[2 * r], s0[r]));
    CK(hipEventRecord(ej[2 * r + 1], s1[r]));
    CK(hipStreamWaitEvent(g, ej[2 * r], 0));
    CK(hipStreamWaitEvent(g, ej[2 * r + 1], 0));
  }
  std::fprintf(stderr, "flags %d: ending capture\n", f);
  CK(hipStreamEndCapture(g, &graph));
  hipGraphExec_t ex;
  CK(hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ex, g));
  CK(hipStreamSynchronize(g));
  std::printf("flags %d: ok\n", f);
  return 0;
}
