// Copy-engine ("sdma") halo transport of the LDS multi-step passes (slab and 3-D block ranks). See wave3d/solver.hpp.
//
// Why: the reference exchanges its ghost planes with MPI through host staging after every step (report.pdf p.16 §4.4:
// 2 GPUs spend 0.135 s copying + 0.054 s in MPI against 0.344 s of compute, nothing overlapped).
// RCCL point-to-point moves data with copy kernels that need compute units, and the LDS passes hold every CU (one
// 1024-thread workgroup per CU), so an RCCL "overlap" mostly queues behind the pass. The SDMA engines need no CU:
// hipMemcpyAsync(..., hipMemcpyDeviceToDeviceNoCU) runs beside a pass that owns the whole GPU (measured on MI355X,
// tools/probes/sdma_probe.hip: a pass-sized kernel 741 µs alone, 733-750 µs with 8 concurrent NoCU copies; ~60 GB/s
// per engine).
//
// Data path, exchange i (after unit i; the next pass reads S-deep ghosts of the two levels unit i wrote):
//   slab ranks   the face planes go straight into the neighbour's ghost planes of the same field buffers (IPC-mapped;
//                contiguous planes, no packing); with overlap they leave from the side stream as soon as the two
//                shell passes have written them, while the interior pass runs;
//   block ranks  k_box_copy packs every peer's faces/edges/corners into send_buf_ (one CU kernel), the copy engines move
//                each peer's message into the peer's receive staging, the receiver unpacks it (k_box_copy) before its
//                next pass.
// Cross-rank order (no host round trip, no RCCL): two flag words per link in uncached device memory, written and
// waited for by one-workgroup kernels (k_flag_sync, kernels_halo.hip; system-scope vector atomics, a bounded spin whose
// timeout lands in the rank's error log, word 0 of errlog_, so every rank learns of it through the end-of-solve
// gather). hipStreamWaitValue32 / hipStreamWriteValue32 would keep the compute units out of it entirely, but this HIP
// runtime executes a captured stream wait once at capture time instead of recording it into the graph
// (tools/probes/memop_capture_probe.hip), and the solve is replayed from a graph; the flag kernels are graph nodes.
//   "arrived" [2k]     link k's copies of exchange i are complete (the signal kernel follows the copies in stream
//                      order)                                              → receiver's s0 waits before unit i + 1
//   "done"    [2k + 1] link k finished unit i − 1 and consumed exchange i − 1 (the regions the next copy overwrites are
//                      free)                                               → sender's copy stream waits before exchange i
// Values: exchange i of a solve of parity p writes p·0x10000 + i + 1; the done word after the last pass of a solve
// holds p·0x10000 + 0xFFFF (the next solve's exchange 0 waits for it). Waits are for EQUALITY: a word is never written
// again before its reader has seen the previous value (the next write needs the reader's own signal), and consecutive
// values of a word always differ (they alternate between the two parity sets across solves), so no flag is ever reset
// and a captured graph (values baked in) is replayed for every solve of its parity: one graph per parity.
// Visibility: the copy engines read the sender's fields after the shell / pass kernels ended (their end-of-kernel
// release wrote the L2s back) and write HBM; the receiver's next kernel starts with an acquire that drops stale L2
// lines, and its ghost planes share no 128-B line with planes it writes (planes are whole lines).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "wave3d/capture_guard.hpp"
#include "wave3d/solver.hpp"

namespace wave3d {

namespace {
constexpr int kHandleBufs = 6;  // u[0..3], receive staging, flags
struct XInfo {                  // layout facts shipped with the handles (checked on the receiving side)
  int dev, ndev;
  long long nx, plane, xg, yg, zg;
  int has_recv, nbuf;
};
}  // namespace

std::vector<GpuSolver::XLink> GpuSolver::sdma_links() const {
  std::vector<XLink> v;
  if (!block_tb_) {
    for (int side = 0; side < 2; ++side) {
      const int peer = neighbor_rank(dims_, rank_, 0, side);
      if (peer < 0) continue;
      XLink l;
      l.peer = peer;
      l.side = side;
      // the peer's links are [its lower neighbour (if any), its upper]: this rank is the peer's upper neighbour when
      // the peer is below it
      l.slot = side == 0 ? (neighbor_rank(dims_, peer, 0, 0) >= 0 ? 1 : 0) : 0;
      l.peer_nx = rank_box(prob_, dims_, peer).nx();
      v.push_back(l);
    }
    return v;
  }
  const int s0 = 2;
  for (const DeepPeer& q : deep_[s0].peers) {
    XLink l;
    l.peer = q.peer;
    // the peer's plan (its layout has the same ghost depths): this rank's index among its peers, and where its message
    // lands in the peer's staging for every pass depth
    const Layout pl = make_layout(prob_, rank_box(prob_, dims_, q.peer), 16, lay_.xg, lay_.yg, lay_.zg);
    W3D_REQUIRE(opt_.temporal < static_cast<int>(sizeof(l.recv_off) / sizeof(l.recv_off[0])),
                "sdma: pass depth beyond the link's offset table");
    for (int st = 2; st <= opt_.temporal; ++st) {
      const DeepPlan pp = make_deep_plan(pl, dims_, q.peer, st);
      int idx = -1;
      for (size_t k = 0; k < pp.peers.size(); ++k)
        if (pp.peers[k].peer == rank_) idx = static_cast<int>(k);
      W3D_REQUIRE(idx >= 0, "sdma: peer plan does not list this rank");
      const DeepPeer& back = pp.peers[static_cast<size_t>(idx)];
      const DeepPeer* mine = nullptr;
      for (const DeepPeer& m : deep_[st].peers)
        if (m.peer == q.peer) mine = &m;
      W3D_REQUIRE(mine && mine->count == back.count, "sdma: message sizes differ between the two ends of a link");
      l.slot = idx;
      l.recv_off[st] = back.buf_off;
    }
    v.push_back(l);
  }
  return v;
}

void GpuSolver::sdma_alloc() {
  xlinks_ = sdma_links();
  const size_t n = std::max<size_t>(1, xlinks_.size());
  W3D_HIP(hipExtMallocWithFlags(reinterpret_cast<void**>(&xflags_), std::max<size_t>(256, 8 * n),
                                hipDeviceMallocUncached));
  l2_flush_all(nullptr);  // (no dirty line of a freed cached buffer may be evicted over the flags later: kernels.hpp)
  W3D_HIP(hipDeviceSynchronize());
  // "arrived" 0 (never waited for before it is written); "done" = the end of a solve of parity 1, so the first solve's
  // first exchange (parity 0) finds its peers' previous solve finished
  std::vector<unsigned> init(2 * n, 0u);
  for (size_t k = 0; k < n; ++k) init[2 * k + 1] = xend(1);
  W3D_HIP(hipMemcpy(xflags_, init.data(), init.size() * sizeof(unsigned), hipMemcpyHostToDevice));
  {
    const int K1 = prob_.K + 1;
    std::vector<unsigned> v(static_cast<size_t>(2 * K1));
    for (int par = 0; par < 2; ++par)
      for (int i = 0; i < K1; ++i) v[static_cast<size_t>(par * K1 + i)] = (par ? 0x10000u : 0u) + static_cast<unsigned>(i + 1);
    W3D_HIP(hipMalloc(&xvals_, v.size() * sizeof(unsigned)));
    W3D_HIP(hipMemcpy(xvals_, v.data(), v.size() * sizeof(unsigned), hipMemcpyHostToDevice));
  }
  // copy streams (SolverOptions::sdma_streams, env W3D_SDMA_STREAMS; at most one per link): each has its own engine,
  // and with s0 and s1 at most 4 streams fit the hardware queues a process gets (GPU_MAX_HW_QUEUES). Defaults: slab
  // ranks one per face; block ranks exchanging after the pass (s0 + 3 copy streams) three — the 512³ 2x2x2 rank 3/8
  // runs 1.51 / 1.70 ms best / mean of 60 solves with three against 2.14 / 2.29 with one (profiles/r4/sdma_streams.md);
  // overlapped block ranks one (with two, the graph executor queued the 2048³ core pass behind a copy branch, r3)
  int ns = opt_.sdma_streams > 0 ? opt_.sdma_streams : block_tb_ ? (opt_.overlap ? 1 : 3) : 2;
  if (const char* v = std::getenv("W3D_SDMA_STREAMS")) ns = std::max(1, std::atoi(v));
  ns = std::min<int>(ns, static_cast<int>(std::max<size_t>(1, xlinks_.size())));
  int lo = 0, hi = 0;
  W3D_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
  xcs_.resize(static_cast<size_t>(ns));
  xcev_.resize(static_cast<size_t>(ns));
  for (int c = 0; c < ns; ++c) {
    W3D_HIP(hipStreamCreateWithPriority(&xcs_[static_cast<size_t>(c)], hipStreamNonBlocking, hi));
    W3D_HIP(hipEventCreateWithFlags(&xcev_[static_cast<size_t>(c)], hipEventDisableTiming));
  }
  W3D_HIP(hipEventCreateWithFlags(&xfork_, hipEventDisableTiming));
}

std::string GpuSolver::sdma_handles() const {
  W3D_REQUIRE(sdma_, "sdma_handles: this solver does not use the copy-engine transport");
  hipIpcMemHandle_t h[kHandleBufs];
  std::memset(h, 0, sizeof h);
  for (int b = 0; b < nbuf_; ++b) W3D_HIP(hipIpcGetMemHandle(&h[b], u_[b]));
  if (recv_buf_) W3D_HIP(hipIpcGetMemHandle(&h[4], recv_buf_));
  W3D_HIP(hipIpcGetMemHandle(&h[5], xflags_));
  XInfo inf{};
  W3D_HIP(hipGetDevice(&inf.dev));
  W3D_HIP(hipGetDeviceCount(&inf.ndev));
  inf.nx = lay_.nx;
  inf.plane = lay_.plane;
  inf.xg = lay_.xg;
  inf.yg = lay_.yg;
  inf.zg = lay_.zg;
  inf.has_recv = recv_buf_ ? 1 : 0;
  inf.nbuf = nbuf_;
  return std::string(reinterpret_cast<const char*>(h), sizeof h) + std::string(reinterpret_cast<const char*>(&inf), sizeof inf);
}

void GpuSolver::connect_sdma(const std::vector<std::string>& all) {
  W3D_REQUIRE(sdma_, "connect_sdma: this solver does not use the copy-engine transport");
  W3D_REQUIRE(static_cast<int>(all.size()) == world_, "connect_sdma: one handle set per rank expected");
  int me = 0, nd = 0;
  W3D_HIP(hipGetDevice(&me));
  W3D_HIP(hipGetDeviceCount(&nd));
  for (XLink& l : xlinks_) {
    const std::string& b = all[static_cast<size_t>(l.peer)];
    hipIpcMemHandle_t h[kHandleBufs];
    XInfo inf{};
    W3D_REQUIRE(b.size() == sizeof h + sizeof inf, "connect_sdma: bad handle size from rank " + std::to_string(l.peer));
    std::memcpy(h, b.data(), sizeof h);
    std::memcpy(&inf, b.data() + sizeof h, sizeof inf);
    W3D_REQUIRE(inf.xg == lay_.xg && inf.yg == lay_.yg && inf.zg == lay_.zg && inf.nbuf == nbuf_,
                "connect_sdma: rank " + std::to_string(l.peer) + " runs another schedule (ghost depths differ)");
    W3D_REQUIRE(block_tb_ || (inf.plane == lay_.plane && inf.nx == l.peer_nx),
                "connect_sdma: slab neighbour " + std::to_string(l.peer) + " has another plane geometry");
    W3D_REQUIRE(!block_tb_ || inf.has_recv, "connect_sdma: block neighbour without a receive staging");
    // a neighbour on another GPU must be reachable by this GPU's copy engines over xGMI (peer access)
    if (inf.ndev == nd && inf.dev != me) {
      int can = 0;
      W3D_HIP(hipDeviceCanAccessPeer(&can, me, inf.dev));
      W3D_REQUIRE(can, "sdma transport: GPU " + std::to_string(me) + " cannot access peer GPU " + std::to_string(inf.dev));
    }
    auto open = [&](const hipIpcMemHandle_t& hh) {
      void* p = nullptr;
      W3D_HIP(hipIpcOpenMemHandle(&p, hh, hipIpcMemLazyEnablePeerAccess));
      return p;
    };
    l.ipc = true;
    l.flags = static_cast<unsigned*>(open(h[5]));
    if (block_tb_) {
      l.recv = static_cast<double*>(open(h[4]));
    } else {
      for (int k = 0; k < nbuf_; ++k) l.u[k] = static_cast<double*>(open(h[k]));
    }
  }
}

void GpuSolver::connect_sdma_self() {
  W3D_REQUIRE(sdma_, "connect_sdma_self: this solver does not use the copy-engine transport");
  // perf study (fake rank): every link is this rank itself — the copies land in its own ghosts / staging (wrong values,
  // same traffic), the flags are its own words at the link's own index
  for (size_t k = 0; k < xlinks_.size(); ++k) {
    XLink& l = xlinks_[k];
    l.slot = static_cast<int>(k);
    l.flags = xflags_;
    l.peer_nx = lay_.nx;
    for (int b = 0; b < nbuf_; ++b) l.u[b] = u_[b];
    l.recv = recv_buf_;
    if (block_tb_)
      for (int st = 2; st <= opt_.temporal; ++st) l.recv_off[st] = deep_[st].peers[k].buf_off;
    l.ipc = false;
  }
}

void GpuSolver::sdma_check_connected() const {
  for (const XLink& l : xlinks_) {
    bool ok = l.flags != nullptr;
    if (block_tb_)
      ok = ok && l.recv != nullptr;
    else
      for (int b = 0; b < nbuf_; ++b) ok = ok && l.u[b] != nullptr;
    W3D_REQUIRE(ok, "sdma transport: neighbour " + std::to_string(l.peer) +
                        " not connected (connect_sdma / connect_sdma_self before the first solve)");
  }
}

// Bound of one flag wait in wall-clock ticks: SolverOptions::flag_timeout_s, else min(W3D_TIMEOUT_S (default 300) / 2,
// 60) s — below the host's own wait bound (wait_stream), so a lost peer is reported by the device ("a flag wait timed
// out") rather than by the host timer, and with k_flag_sync's early exit the whole solve then ends within one bound.
unsigned long long GpuSolver::flag_ticks() const {
  static const int khz = [] {
    int k = 100000;
    (void)hipDeviceGetAttribute(&k, hipDeviceAttributeWallClockRate, 0);
    return k;
  }();
  double sec = opt_.flag_timeout_s;
  if (sec <= 0.0) {
    const char* v = std::getenv("W3D_TIMEOUT_S");
    const double host = v && std::atof(v) > 0.0 ? std::atof(v) : 300.0;
    sec = std::min(0.5 * host, 60.0);
  }
  return static_cast<unsigned long long>(sec * 1e3 * khz);
}

// Exchange i: on the side stream once the shells are written (overlap), else on s0 after the pass.
void GpuSolver::unit_exchange_sdma(int i) {
  if (!needs_exchange(i)) return;
  hipStream_t xs = xstream();  // (overlap: the shells already ran on xs, after its wait for the unit's inputs)
  timed(kPhaseComm, xs, [&] {
    const int s = units_[static_cast<size_t>(i) + 1].steps;
    if (block_tb_) pack_halo(xs);  // (build_msgs set deep_s_ = s)
    // per copy stream: wait until its links' receivers have finished with the regions the copies overwrite, copy,
    // then raise the links' "arrived" words with 4-byte copy-engine writes behind the data (stream order: after the
    // copies have completed; no compute queue is held while the copies run)
    capture::record(xfork_, xs);
    const size_t P = static_cast<size_t>(lay_.plane), nc = xcs_.size();
    for (size_t c = 0; c < nc; ++c) {
      hipStream_t cs = xcs_[c];
      capture::wait(cs, xfork_);
      FlagOp w, none;
      w.value = i == 0 ? xend(1 - xpar_) : xval(i - 1);
      w.status = reinterpret_cast<unsigned*>(errlog_);
      w.ticks = flag_ticks();
      for (size_t k = c; k < xlinks_.size(); k += nc) w.addr[w.n++] = xflags_ + 2 * k + 1;
      launch_flag_sync(w, none, cs);
      for (size_t k = c; k < xlinks_.size(); k += nc) {
        const XLink& l = xlinks_[k];
        if (block_tb_) {
          const DeepPeer& q = deep_[s].peers[k];
          W3D_HIP(hipMemcpyAsync(l.recv + l.recv_off[s], send_buf_ + sbase_[s] + q.buf_off,
                                 static_cast<size_t>(q.count) * sizeof(double), hipMemcpyDeviceToDeviceNoCU, cs));
        } else {
          // u^{n+S} s planes deep and u^{n+S−1} s − 1 deep: this rank's planes next to the face → the peer's ghost
          // planes beyond its facing side (the peer's plane p sits at (p + xg)·plane in its buffers, same geometry)
          // (ghost_bits: both ends stored u^{n+S−1}'s first ghost plane themselves — its part starts one plane in)
          for (int f = 0; f < 2; ++f) {
            const i64 g = f == 1 ? (ghost_bits(i) >> l.side) & 1 : 0;
            const i64 d = (f == 0 ? s : s - 1) - g;
            if (d <= 0) continue;
            const int b = uf_[f == 0 ? 1 : 0];
            const i64 src = l.side == 0 ? g : lay_.nx - d - g;
            const i64 dst = l.side == 0 ? l.peer_nx + g : -d - g;
            W3D_HIP(hipMemcpyAsync(l.u[b] + (dst + lay_.xg) * static_cast<i64>(P), u_[b] + lay_.plane_off(src),
                                   static_cast<size_t>(d) * P * sizeof(double), hipMemcpyDeviceToDeviceNoCU, cs));
          }
        }
      }
      const unsigned* val = xvals_ + xpar_ * (prob_.K + 1) + i;  // (= xval(i))
      for (size_t k = c; k < xlinks_.size(); k += nc)
        W3D_HIP(hipMemcpyAsync(xsig(xlinks_[k], 0), val, sizeof(unsigned), hipMemcpyDeviceToDeviceNoCU, cs));
      capture::record(xcev_[c], cs);
      capture::wait(xs, xcev_[c]);
    }
  });
  if (xs != s0_) capture::record(ev_halo_, xs);
}

// s0, before unit i: the ghosts of exchange i − 1 have arrived (block: unpack them), then the regions exchange i
// overwrites are released to the neighbours.
void GpuSolver::sdma_receive(int i) {
  if (!plan_.any()) return;
  FlagOp w, sig;
  if (i >= 1 && needs_exchange(i - 1)) {
    w.value = xval(i - 1);
    w.status = reinterpret_cast<unsigned*>(errlog_);
    w.ticks = flag_ticks();
    for (size_t k = 0; k < xlinks_.size(); ++k) w.addr[w.n++] = xflags_ + 2 * k;
  }
  if (i >= 1 && needs_exchange(i)) {
    sig.value = xval(i - 1);
    for (const XLink& l : xlinks_) sig.addr[sig.n++] = xsig(l, 1);
  }
  // slab ranks need nothing between the two: one launch waits and signals
  const bool between = block_tb_ || (opt_.poison_ghosts && i >= 1 && needs_exchange(i));
  if (!between) {
    timed(kPhaseComm, s0_, [&] { launch_flag_sync(w, sig, s0_); });
    return;
  }
  timed(kPhaseComm, s0_, [&] {
    launch_flag_sync(w, FlagOp{}, s0_);
    if (block_tb_ && w.n > 0) unpack_halo(s0_);
  });
  if (opt_.poison_ghosts && i >= 1 && needs_exchange(i)) {
    int uf[2], k = 0;  // (the two buffers unit i writes)
    for (int b = 0; b < 4; ++b)
      if (b != cur_ && b != old_) uf[k++] = b;
    sdma_poison(i, uf);
  }
  launch_flag_sync(FlagOp{}, sig, s0_);
}

// --poison-ghosts: NaN into the ghost regions exchange i fills, in the two buffers unit i writes (uf[0]: u^{n+S−1},
// uf[1]: u^{n+S}), until the neighbours' copies land. Issued right before the "done" signal that lets those copies start
// (exchange 0: at the end of the previous solve, before its last "done").
void GpuSolver::sdma_poison(int i, const int uf[2]) {
  const int s = units_[static_cast<size_t>(i) + 1].steps;
  if (block_tb_) {
    launch_box_copy(lay_, unpack_tab_[s], 2, u_[uf[1]], u_[uf[0]], nullptr, s0_);
    return;
  }
  const size_t P = static_cast<size_t>(lay_.plane);
  for (const XLink& l : xlinks_)
    for (int f = 0; f < 2; ++f) {
      const i64 g1 = f == 1 ? (ghost_bits(i) >> l.side) & 1 : 0;  // (the plane unit i stores itself: not poisoned)
      const i64 d = (f == 0 ? s : s - 1) - g1;
      if (d <= 0) continue;
      const i64 g = l.side == 0 ? -d - g1 : lay_.nx + g1;
      W3D_HIP(hipMemsetAsync(u_[uf[f == 0 ? 1 : 0]] + lay_.plane_off(g), 0xFF, static_cast<size_t>(d) * P * sizeof(double),
                             s0_));
    }
}

void GpuSolver::sdma_finish() {
  if (!plan_.any() || units_.size() < 2) return;
  if (opt_.poison_ghosts) {
    const int uf[2] = {2, 3};  // (every solve starts with cur = 1, old = 0: its first unit writes buffers 2 and 3)
    sdma_poison(0, uf);
  }
  FlagOp sig;
  sig.value = xend(xpar_);
  for (const XLink& l : xlinks_) sig.addr[sig.n++] = xsig(l, 1);
  launch_flag_sync(FlagOp{}, sig, s0_);
}

}  // namespace wave3d
