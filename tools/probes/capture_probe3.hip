// Stream-capture probe 3: the copy-engine exchange topologies of GpuSolver::unit_exchange_sdma
// captured into one graph, to find which one crashed the HIP 7.2 runtime in round 4 (profiles/r4/sdma_split_attempt.log:
// "two copy streams per slab link" dumped core in graph capture).
//
// A solve = `units` passes; after each pass but the last, an overlapped exchange: s0 runs the shell kernel, the exchange
// stream xs waits for it, forks to the copy streams (each: a one-workgroup flag kernel, hipMemcpyDeviceToDeviceNoCU
// copies, a 4-byte "arrived" copy behind them), joins them back, and s0 waits for xs after its interior kernel.
//   mode 0  production slab: one copy stream per face (2), both field copies and the signal on it
//   mode 1  production block: 3 copy streams, 7 messages dealt round-robin
//   mode 2  round-4 split: two copy streams per face (4), the signal stream waits for its sibling's event first
//   mode 3  split, joined through the origin: both copy streams join xs, the signal goes out on xs itself
//   mode 4  split, second fork: both join xs, xs forks again to the signal stream (a fresh event)
//   mode 5  mode 2 (sibling wait) plus a direct join of the first copy stream into xs
//   mode 6  the in-process group's pattern: b waits on a once before its own work (a sibling event, then b's own work),
//           both join xs directly
// Prints the step before every capture-level call so a crash names it. Build:
//   hipcc --offload-arch=gfx950 -O2 tools/probes/capture_probe3.hip -o build/probes/capture_probe3
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

__global__ void k_touch(double* p, int n, double v) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] += v;
}
__global__ void k_flag(unsigned* f) {  // (stands in for k_flag_sync: one workgroup, a vector store)
  if (threadIdx.x == 0) f[0] = f[0] + 1u;
}

static void step(const char* what, int mode, int u) {
  std::fprintf(stderr, "mode %d unit %d: %s\n", mode, u, what);
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? std::atoi(argv[1]) : 0;
  const int units = argc > 2 ? std::atoi(argv[2]) : 4;
  const bool eager = argc > 3 && std::atoi(argv[3]) != 0;
  const int nc = mode == 0 ? 2 : mode == 1 ? 3 : 4;
  const size_t n = size_t{1} << 22, msg = size_t{1} << 20;  // (doubles: a 32 MB field, 8 MB messages)
  double *field, *ghost;
  unsigned* flags;
  CK(hipMalloc(&field, n * sizeof(double)));
  CK(hipMalloc(&ghost, n * sizeof(double)));
  CK(hipMalloc(&flags, 64 * sizeof(unsigned)));
  CK(hipMemset(field, 0, n * sizeof(double)));
  CK(hipMemset(flags, 0, 64 * sizeof(unsigned)));
  hipStream_t s0, xs;
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithPriority(&xs, hipStreamNonBlocking, hi));
  std::vector<hipStream_t> cs(static_cast<size_t>(nc));
  std::vector<hipEvent_t> cev(static_cast<size_t>(nc));
  for (int c = 0; c < nc; ++c) {
    CK(hipStreamCreateWithPriority(&cs[static_cast<size_t>(c)], hipStreamNonBlocking, hi));
    CK(hipEventCreateWithFlags(&cev[static_cast<size_t>(c)], hipEventDisableTiming));
  }
  hipEvent_t ev_shell, ev_halo, xfork, xfork2;
  for (hipEvent_t* e : {&ev_shell, &ev_halo, &xfork, &xfork2}) CK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  auto kern = [&](hipStream_t s, size_t off, size_t cnt) {
    hipLaunchKernelGGL(k_touch, dim3(256), dim3(256), 0, s, field + off, static_cast<int>(cnt), 1.0);
  };
  auto copy = [&](hipStream_t s, int k) {
    CK(hipMemcpyAsync(ghost + (static_cast<size_t>(k) % 4) * msg, field + (static_cast<size_t>(k) % 4) * msg,
                      msg * sizeof(double), hipMemcpyDeviceToDeviceNoCU, s));
  };
  auto signal = [&](hipStream_t s, int k) {
    CK(hipMemcpyAsync(flags + 32 + k, flags + k, sizeof(unsigned), hipMemcpyDeviceToDeviceNoCU, s));
  };
  auto exchange = [&](int u) {
    CK(hipEventRecord(xfork, xs));
    if (mode == 0 || mode == 1) {
      const int msgs = mode == 0 ? 2 : 7;
      for (int c = 0; c < nc; ++c) {
        hipStream_t s = cs[static_cast<size_t>(c)];
        CK(hipStreamWaitEvent(s, xfork, 0));
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s, flags + c);
        for (int k = c; k < msgs; k += nc) {
          copy(s, 2 * k);
          if (mode == 0) copy(s, 2 * k + 1);  // (slab: u^{n+S} and u^{n+S-1} to the same face)
        }
        for (int k = c; k < msgs; k += nc) signal(s, k);
        CK(hipEventRecord(cev[static_cast<size_t>(c)], s));
        CK(hipStreamWaitEvent(xs, cev[static_cast<size_t>(c)], 0));
      }
      return;
    }
    for (int face = 0; face < 2; ++face) {
      hipStream_t a = cs[static_cast<size_t>(2 * face)], b = cs[static_cast<size_t>(2 * face + 1)];
      hipEvent_t ea = cev[static_cast<size_t>(2 * face)], eb = cev[static_cast<size_t>(2 * face + 1)];
      CK(hipStreamWaitEvent(a, xfork, 0));
      CK(hipStreamWaitEvent(b, xfork, 0));
      hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, a, flags + face);
      copy(a, 2 * face);
      copy(b, 2 * face + 1);
      CK(hipEventRecord(ea, a));
      if (mode == 2 || mode == 5) {  // sibling-to-sibling: b waits for a, then raises the signal behind both
        step("sibling wait", mode, u);
        CK(hipStreamWaitEvent(b, ea, 0));
        signal(b, face);
        CK(hipEventRecord(eb, b));
        CK(hipStreamWaitEvent(xs, eb, 0));
        if (mode == 5) CK(hipStreamWaitEvent(xs, ea, 0));
      } else if (mode == 6) {
        CK(hipStreamWaitEvent(b, ea, 0));
        signal(b, face);
        CK(hipEventRecord(eb, b));
        CK(hipStreamWaitEvent(xs, ea, 0));
        CK(hipStreamWaitEvent(xs, eb, 0));
      } else {
        CK(hipEventRecord(eb, b));
        CK(hipStreamWaitEvent(xs, ea, 0));
        CK(hipStreamWaitEvent(xs, eb, 0));
        if (mode == 3) {
          signal(xs, face);
        } else {  // mode 4: a second fork from the origin to the signal stream
          CK(hipEventRecord(xfork2, xs));
          CK(hipStreamWaitEvent(b, xfork2, 0));
          signal(b, face);
          CK(hipEventRecord(eb, b));
          CK(hipStreamWaitEvent(xs, eb, 0));
        }
      }
    }
  };
  auto solve = [&] {
    for (int u = 0; u < units; ++u) {
      if (u + 1 < units) {
        kern(s0, 0, msg);  // shells
        CK(hipEventRecord(ev_shell, s0));
        CK(hipStreamWaitEvent(xs, ev_shell, 0));
        exchange(u);
        CK(hipEventRecord(ev_halo, xs));
        kern(s0, msg, n - msg);  // interior
        CK(hipStreamWaitEvent(s0, ev_halo, 0));
      } else {
        kern(s0, 0, n);
      }
    }
  };
  if (eager) {
    step("eager solve", mode, -1);
    solve();
    CK(hipStreamSynchronize(s0));
    std::printf("mode %d eager: ok\n", mode);
    return 0;
  }
  hipGraph_t graph = nullptr;
  step("hipStreamBeginCapture", mode, -1);
  CK(hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal));
  CK(hipEventRecord(xfork, s0));  // (xs joins the capture through s0)
  CK(hipStreamWaitEvent(xs, xfork, 0));
  solve();
  CK(hipEventRecord(ev_halo, xs));
  CK(hipStreamWaitEvent(s0, ev_halo, 0));
  step("hipStreamEndCapture", mode, -1);
  CK(hipStreamEndCapture(s0, &graph));
  size_t nodes = 0;
  CK(hipGraphGetNodes(graph, nullptr, &nodes));
  step("hipGraphInstantiate", mode, -1);
  hipGraphExec_t ex;
  CK(hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0));
  step("hipGraphUpload", mode, -1);
  CK(hipGraphUpload(ex, s0));
  for (int r = 0; r < 3; ++r) {
    step("hipGraphLaunch", mode, r);
    CK(hipGraphLaunch(ex, s0));
  }
  CK(hipStreamSynchronize(s0));
  std::printf("mode %d units %d: ok (%zu graph nodes)\n", mode, units, nodes);
  return 0;
}
