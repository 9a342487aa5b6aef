// Runtime probe: does a hipStreamWaitValue32 captured into a hipGraph still WAIT when the graph is launched?
// (tools/probes/sdma_probe.hip only showed that capture + launch of an already-satisfied wait succeeds.)
//
//   hipcc --offload-arch=gfx950 -O2 tools/probes/memop_capture_probe.hip -o build/memop_capture_probe
//
// For each variant: a graph [wait flag == 5] -> [kernel: marker = 1] is launched on stream A, the host sleeps 50 ms and
// reads the marker (0 = the wait held), then stream B writes flag = 5 and the host reads the marker again (1 = released).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::printf("FAIL %s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

__global__ void k_mark(unsigned* m) { __hip_atomic_store(m, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }

int main() {
  unsigned *flag = nullptr, *mark = nullptr;
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&flag), 256, hipDeviceMallocUncached));
  CK(hipHostMalloc(reinterpret_cast<void**>(&mark), 64, hipHostMallocCoherent));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  auto variant = [&](const char* name, bool capture, unsigned wflags, bool batch) {
    CK(hipMemset(flag, 0, 256));
    CK(hipDeviceSynchronize());
    *reinterpret_cast<volatile unsigned*>(mark) = 0;
    hipGraphExec_t ge = nullptr;
    auto body = [&]() {
      if (batch) {
        hipStreamBatchMemOpParams p[1];
        std::memset(p, 0, sizeof p);
        p[0].operation = hipStreamMemOpWaitValue32;
        p[0].waitValue.address = flag;
        p[0].waitValue.value = 5;
        p[0].waitValue.flags = wflags;
        CK(hipStreamBatchMemOp(a, 1, p, 0));
      } else {
        CK(hipStreamWaitValue32(a, flag, 5, wflags, 0xFFFFFFFFu));
      }
      hipLaunchKernelGGL(k_mark, dim3(1), dim3(1), 0, a, mark);
    };
    if (capture) {
      hipGraph_t g = nullptr;
      CK(hipStreamBeginCapture(a, hipStreamCaptureModeThreadLocal));
      body();
      CK(hipStreamEndCapture(a, &g));
      size_t n = 0;
      CK(hipGraphGetNodes(g, nullptr, &n));
      hipGraphNode_t nodes[8];
      CK(hipGraphGetNodes(g, nodes, &n));
      std::printf("%s: graph nodes:", name);
      for (size_t i = 0; i < n; ++i) {
        hipGraphNodeType t;
        CK(hipGraphNodeGetType(nodes[i], &t));
        std::printf(" %d", static_cast<int>(t));
      }
      std::printf("\n");
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphDestroy(g));
      CK(hipGraphLaunch(ge, a));
    } else {
      body();
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    const unsigned before = *reinterpret_cast<volatile unsigned*>(mark);
    const hipError_t q = hipStreamQuery(a);
    CK(hipStreamWriteValue32(b, flag, 5, 0));
    CK(hipStreamSynchronize(b));
    CK(hipStreamSynchronize(a));
    const unsigned after = *reinterpret_cast<volatile unsigned*>(mark);
    std::printf("%s: marker before release %u (stream %s), after %u -> %s\n", name, before, hipGetErrorString(q), after,
                before == 0 && after == 1 ? "WAIT HELD" : "WAIT DID NOT HOLD");
    if (ge) CK(hipGraphExecDestroy(ge));
  };
  variant("eager Eq", false, hipStreamWaitValueEq, false);
  variant("eager Gte", false, hipStreamWaitValueGte, false);
  variant("captured Eq", true, hipStreamWaitValueEq, false);
  variant("captured Gte", true, hipStreamWaitValueGte, false);
  variant("eager batch Eq", false, hipStreamWaitValueEq, true);
  variant("captured batch Eq", true, hipStreamWaitValueEq, true);
  variant("captured batch Gte", true, hipStreamWaitValueGte, true);
  std::printf("done\n");
  return 0;
}
