// Probe (one GPU): what the peer-push halo transport relies on.
//   1. hipStreamWaitValue32 / hipStreamWriteValue32 inside a stream capture (graph memop nodes)
//   2. hipIpcGetMemHandle on fine-grained and uncached device allocations
//   3. a kernel's system-scope flag store observed by hipStreamWaitValue32 on another stream
// Build: hipcc --offload-arch=gfx950 -O2 tools/push_probe.hip -o build/push_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    std::printf("%-70s -> %s\n", #x, hipGetErrorString(e_));                                   \
  } while (0)

__global__ void k_add(double* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1.0;
}

__global__ void k_signal(unsigned* flag, unsigned v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

int main() {
  int can = 0;
  CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0));
  std::printf("CanUseStreamWaitValue = %d\n", can);
  unsigned* flag = nullptr;
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&flag), 256, hipDeviceMallocUncached));
  CK(hipMemset(flag, 0, 256));
  double* fg = nullptr;
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&fg), 1 << 20, hipDeviceMallocFinegrained));
  double* cg = nullptr;
  CK(hipMalloc(&cg, 1 << 20));
  hipIpcMemHandle_t h;
  CK(hipIpcGetMemHandle(&h, fg));
  CK(hipIpcGetMemHandle(&h, flag));
  CK(hipIpcGetMemHandle(&h, cg));

  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  // eager: wait on s for a flag that a kernel on s2 sets
  CK(hipStreamWaitValue32(s, flag, 1, hipStreamWaitValueGte, 0xffffffffu));
  hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, s, cg, 64);
  hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, s2, flag, 1u);
  CK(hipStreamSynchronize(s));
  CK(hipStreamSynchronize(s2));

  // capture: wait value + kernel + write value
  hipGraph_t g = nullptr;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  CK(hipStreamWaitValue32(s, flag + 1, 2, hipStreamWaitValueGte, 0xffffffffu));
  hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, s, cg, 64);
  CK(hipStreamWriteValue32(s, flag + 2, 7, 0));
  CK(hipStreamEndCapture(s, &g));
  hipGraphExec_t ge = nullptr;
  if (g) {
    size_t n = 0;
    CK(hipGraphGetNodes(g, nullptr, &n));
    std::printf("graph nodes: %zu\n", n);
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  }
  if (ge) {
    CK(hipGraphLaunch(ge, s));
    hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, s2, flag + 1, 2u);
    CK(hipStreamSynchronize(s));
    unsigned host[4] = {};
    CK(hipMemcpy(host, flag, sizeof host, hipMemcpyDeviceToHost));
    std::printf("flags after graph: %u %u %u\n", host[0], host[1], host[2]);
  }
  (void)hipGetLastError();
  std::printf("probe done\n");
  return 0;
}
