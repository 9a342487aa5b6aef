// Stream-capture topology guard: see wave3d/capture_guard.hpp for the HIP 7.2 failure it prevents.
#include "wave3d/capture_guard.hpp"

#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

#include "wave3d/solver.hpp"  // W3D_HIP, fail

namespace wave3d::capture {
namespace {

struct State {
  bool on = false;
  hipStream_t origin = nullptr;
  std::map<hipStream_t, hipStream_t> parent;  // forked stream → the stream it forked from (its first dependency)
  std::map<hipEvent_t, hipStream_t> rec;      // event → the stream that last recorded it in this capture
  std::vector<hipEvent_t> temp;               // events close() created (released by abandon())
};
thread_local State st;

}  // namespace

bool active() { return st.on; }

void begin(hipStream_t origin) {
  abandon();
  st.on = true;
  st.origin = origin;
}

void abandon() {  // (after hipStreamEndCapture: the graph keeps the edges, not the events)
  for (hipEvent_t e : st.temp) (void)hipEventDestroy(e);
  st = State{};
}

void record(hipEvent_t e, hipStream_t s) {
  W3D_HIP(hipEventRecord(e, s));
  if (st.on) st.rec[e] = s;
}

void wait(hipStream_t s, hipEvent_t e) {
  if (st.on) {
    auto it = st.rec.find(e);
    if (it != st.rec.end() && it->second != s) {
      const hipStream_t src = it->second;
      auto ps = st.parent.find(s), pt = st.parent.find(src);
      if (ps == st.parent.end()) {
        if (s != st.origin) st.parent[s] = src;  // first dependency: the fork
      } else if (pt != st.parent.end() && pt->second == ps->second && ps->second != st.origin) {
        // two streams forked from the same non-origin stream, one waiting on the other: refused BEFORE it enters the
        // capture (the probe's modes 2 and 5 crash hipStreamEndCapture; siblings under the origin — a group's
        // per-rank streams — and joins into a parent are fine)
        char buf[240];
        std::snprintf(buf, sizeof buf,
                      "capture topology refused: stream %p waits on an event of its sibling %p (both forked from "
                      "%p); HIP 7.2 hipStreamEndCapture crashes on this (tools/probes/capture_probe3.hip modes 2, 5)",
                      static_cast<void*>(s), static_cast<void*>(src), static_cast<void*>(ps->second));
        fail(buf);
      }
    }
  }
  W3D_HIP(hipStreamWaitEvent(s, e, 0));
}

void close() {
  if (!st.on) return;
  // an aborted capture: every stream that joined it is joined into its parent, deepest first (the shape of the
  // probe's modes 3 / 4, which capture), so hipStreamEndCapture sees a joined (if useless) graph
  auto depth = [](hipStream_t s) {
    int d = 0;
    for (auto it = st.parent.find(s); it != st.parent.end() && d < 64; it = st.parent.find(it->second)) ++d;
    return d;
  };
  std::vector<std::pair<int, hipStream_t>> order;
  for (const auto& kv : st.parent) order.emplace_back(-depth(kv.first), kv.first);
  std::sort(order.begin(), order.end());
  for (const auto& od : order) {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) continue;
    st.temp.push_back(e);
    if (hipEventRecord(e, od.second) == hipSuccess) (void)hipStreamWaitEvent(st.parent[od.second], e, 0);
  }
  st.on = false;
}

void finish() { st.on = false; }

std::string selftest(int mode) {
  // (multi-stream captures need the ROCm 7.2 runtime: the HIP 7.0 one PyTorch bundles crashes on per-unit joins even
  // for the production topology — tools/probes/capture_probe.hip; the solver captures them only on 7.2, too)
  int v = 0;
  if (hipRuntimeGetVersion(&v) != hipSuccess || v < 70200000)
    return "skipped: HIP runtime " + std::to_string(v) + " < 7.2 does not capture multi-stream schedules";
  const size_t bytes = size_t{1} << 22;
  void *a = nullptr, *b = nullptr;
  W3D_HIP(hipMalloc(&a, 4 * bytes));
  W3D_HIP(hipMalloc(&b, 4 * bytes));
  hipStream_t s0, xs, c[4];
  hipEvent_t fork, ev[4], halo, shell;
  W3D_HIP(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  W3D_HIP(hipStreamCreateWithFlags(&xs, hipStreamNonBlocking));
  for (int i = 0; i < 4; ++i) {
    W3D_HIP(hipStreamCreateWithFlags(&c[i], hipStreamNonBlocking));
    W3D_HIP(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
  }
  for (hipEvent_t* e : {&fork, &halo, &shell}) W3D_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
  auto copy = [&](hipStream_t s, int k) {
    W3D_HIP(hipMemcpyAsync(static_cast<char*>(b) + k * bytes, static_cast<char*>(a) + k * bytes, bytes,
                           hipMemcpyDeviceToDeviceNoCU, s));
  };
  std::string refused;
  W3D_HIP(hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal));
  begin(s0);
  try {
    for (int u = 0; u < 3; ++u) {
      W3D_HIP(hipMemsetAsync(a, u, bytes, s0));
      record(shell, s0);
      wait(xs, shell);
      record(fork, xs);
      if (mode == 2) {  // the round-4 split: per face two copy streams, the second waits for its sibling
        for (int f = 0; f < 2; ++f) {
          wait(c[2 * f], fork);
          wait(c[2 * f + 1], fork);
          copy(c[2 * f], 2 * f);
          copy(c[2 * f + 1], 2 * f + 1);
          record(ev[2 * f], c[2 * f]);
          wait(c[2 * f + 1], ev[2 * f]);
          record(ev[2 * f + 1], c[2 * f + 1]);
          wait(xs, ev[2 * f + 1]);
        }
      } else {  // production: one copy stream per face
        for (int f = 0; f < 2; ++f) {
          wait(c[f], fork);
          copy(c[f], 2 * f);
          copy(c[f], 2 * f + 1);
          record(ev[f], c[f]);
          wait(xs, ev[f]);
        }
      }
      record(halo, xs);
      W3D_HIP(hipMemsetAsync(static_cast<char*>(a) + bytes, u, bytes, s0));
      wait(s0, halo);
    }
    finish();
  } catch (const std::exception& ex) {
    refused = ex.what();
    close();
  }
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(s0, &g);
  abandon();
  std::string out;
  if (!refused.empty()) {
    out = refused;
  } else if (e != hipSuccess || g == nullptr) {
    out = std::string("capture failed: ") + hipGetErrorString(e);
  } else {
    hipGraphExec_t x = nullptr;
    W3D_HIP(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    W3D_HIP(hipGraphLaunch(x, s0));
    W3D_HIP(hipStreamSynchronize(s0));
    W3D_HIP(hipGraphExecDestroy(x));
    out = "ok";
  }
  if (g) (void)hipGraphDestroy(g);
  (void)hipGetLastError();
  for (int i = 0; i < 4; ++i) {
    (void)hipStreamDestroy(c[i]);
    (void)hipEventDestroy(ev[i]);
  }
  for (hipEvent_t x : {fork, halo, shell}) (void)hipEventDestroy(x);
  (void)hipStreamDestroy(s0);
  (void)hipStreamDestroy(xs);
  (void)hipFree(a);
  (void)hipFree(b);
  return out;
}

}  // namespace wave3d::capture
