// Multi-rank schedule autotune of the native runtime (bench.py's --autotune on every rank; Python Solver(autotune=True)).
// See wave3d/runtime.hpp.
//
// Why a runtime choice: the halo volume of S-deep passes against the per-step exchanges of single steps, overlap against
// whole passes, slabs against blocks and RCCL copy kernels against the copy engines trade xGMI bandwidth and latency
// against HBM traffic and compute units, and the balance depends on the node. So every
// candidate is timed on the real interconnect and all ranks adopt the one whose slowest rank was fastest.
#include <algorithm>
#include <cstdio>

#include "wave3d/runtime.hpp"

namespace wave3d {

std::vector<Candidate> autotune_candidates(int world, bool with_push) {
  std::vector<Candidate> v;
  auto add = [&](const char* name, const char* decomp, const char* transport, int temporal, bool overlap,
                 int streams = 0, bool conc = false) {
    v.push_back(Candidate{name, decomp, transport, temporal, overlap, streams, conc});
  };
  if (world <= 1) {  // one rank: only the pass depth matters
    add("slab-S4", "slab", "rccl", 4, true);
    add("slab-S3", "slab", "rccl", 3, true);
    add("slab-S2", "slab", "rccl", 2, true);
    add("slab-S1", "slab", "rccl", 1, true);
    return v;
  }
  // simplest first: sequential before overlapped, RCCL before the copy engines, deep passes before shallow ones
  add("slab-S4-seq", "slab", "rccl", 4, false);
  add("slab-S4", "slab", "rccl", 4, true);
  add("slab-S4-sdma-seq", "slab", "sdma", 4, false);
  add("slab-S4-sdma", "slab", "sdma", 4, true);
  if (with_push) {  // (opt-in: not yet run across two GPUs)
    add("slab-S4-push-seq", "slab", "push", 4, false);
    add("slab-S4-push", "slab", "push", 4, true);
  }
  add("slab-S3", "slab", "rccl", 3, true);
  add("slab-S2", "slab", "rccl", 2, true);
  add("slab-S1", "slab", "rccl", 1, true);
  if (world >= 4) {  // (2 ranks: "block" is the slab)
    add("block-S4-seq", "block", "rccl", 4, false);
    add("block-S4", "block", "rccl", 4, true);
    add("block-S4-conc", "block", "rccl", 4, true, 0, true);  // (shells beside the interior)
    add("block-S4-sdma-seq", "block", "sdma", 4, false);
    add("block-S4-sdma", "block", "sdma", 4, true);            // (one copy stream)
    add("block-S4-sdma-x2", "block", "sdma", 4, true, 2);     // (two copy streams: two engines)
    add("block-S3", "block", "rccl", 3, true);
    add("block-S1", "block", "rccl", 1, true);
  }
  return v;
}

void connect_transport(GpuSolver& s, const HostColl& hc, bool fake) {
  if (s.sdma()) {
    if (fake)
      s.connect_sdma_self();
    else
      s.connect_sdma(hc.allgather(s.sdma_handles()));
  } else if (s.push()) {
    if (fake)
      s.connect_push_self();
    else
      s.connect_push(hc.allgather(s.push_handles()));
  }
}

namespace {
// what actually runs (two candidates with the same signature are one schedule timed twice)
std::string signature(const GpuSolver& s) {
  const Dims d = s.dims();
  // (the pass depth only matters to the schedules that fuse steps: a single-step schedule ignores it)
  const int depth = s.mode() == "single-step" ? 1 : s.options().temporal;
  return s.mode() + "/" + s.transport() + "/" + (s.overlapped() ? "ov" : "seq") + "/S" + std::to_string(depth) + "/" +
         std::to_string(d.px) + "x" + std::to_string(d.py) + "x" + std::to_string(d.pz) + "/cs" +
         std::to_string(s.sdma() ? s.copy_streams() : 0) + (s.overlapped() && s.options().shells_concurrent ? "/conc" : "");
}
}  // namespace

AutotuneResult autotune(const Problem& prob, const SolverOptions& base, int rank, int world, std::shared_ptr<Comm> comm,
                        const HostColl& hc, bool fake, bool with_push, int rounds, double tie) {
  struct Live {
    Candidate c;
    std::unique_ptr<GpuSolver> s;
    double best = 1e300;
    bool stable = true;
    bool timed = false;  // timed alone already (memory)
    bool ok = true;      // accepted (its solver may still have been freed: timed alone and clearly slower)
  };
  std::vector<Live> live;
  std::vector<std::string> sigs;
  std::vector<double> ref_log;
  AutotuneResult res;
  rounds = std::max(1, rounds);
  auto reject = [&](const Candidate& c, const std::string& why) {
    res.rejected.emplace_back(c.name, why);
    std::fprintf(stderr, "[wave3d rank %d] candidate %s rejected: %s\n", rank, c.name.c_str(), why.c_str());
  };
  for (const Candidate& c : autotune_candidates(world, with_push)) {
    SolverOptions o = base;
    o.decomp = c.decomp;
    o.temporal = c.temporal;
    o.overlap = c.overlap;
    o.push = c.transport == "push";
    o.sdma = c.transport == "sdma";
    if (c.sdma_streams > 0) o.sdma_streams = c.sdma_streams;
    o.shells_concurrent = o.shells_concurrent || c.shells_concurrent;
    std::unique_ptr<GpuSolver> cand;
    std::string err;
    try {
      cand = std::make_unique<GpuSolver>(prob, o, rank, world, comm);
    } catch (const std::exception& e) {
      err = e.what();
    }
    if (!hc.agree(static_cast<bool>(cand))) {  // a schedule some rank cannot build: skipped everywhere
      reject(c, err.empty() ? "another rank could not build it" : err);
      continue;
    }
    const std::string sig = signature(*cand);
    const auto dup = std::find(sigs.begin(), sigs.end(), sig);
    if (!hc.agree(dup == sigs.end())) {  // a clone of an earlier candidate (e.g. one rank: no exchange to overlap)
      res.rejected.emplace_back(c.name, "same schedule as an earlier candidate (" + sig + ")");
      continue;
    }
    // (collective when the candidate connects to peers: every rank built it; agreed on its own, so a rank whose IPC
    // mapping failed does not reach the next agreement while its peers sit in the first solve's collectives)
    bool connected = false;
    try {
      connect_transport(*cand, hc, fake);
      connected = true;
    } catch (const std::exception& e) {
      err = e.what();
    }
    if (!hc.agree(connected)) {
      reject(c, err.empty() ? "a peer could not connect" : err);
      continue;
    }
    // every schedule computes bit-identical fields: a candidate that fails (a transport wait timed out) or whose error
    // log differs from the first accepted one's (a transport that delivered wrong ghosts) is rejected on every rank
    bool same = false;
    try {
      RunResult r0 = cand->run();  // eager: RCCL peer connections
      r0 = cand->run();            // graph capture
      // (a fake rank's log holds its own partials only: they differ between decompositions, nothing to compare)
      same = r0.finite && (fake || ref_log.empty() || r0.max_err == ref_log);
      if (!same) err = "its error log differs from the reference schedule's";
      if (same && ref_log.empty()) ref_log = r0.max_err;
    } catch (const std::exception& e) {
      err = e.what();
    }
    if (!hc.agree(same)) {
      reject(c, err.empty() ? "failed on another rank" : err);
      continue;
    }
    sigs.push_back(sig);
    Live l{c, std::move(cand)};
    // keep it for the interleaved rounds if the next candidate still fits next to it; else time it alone now
    size_t free_b = 0, total_b = 0;
    W3D_HIP(hipMemGetInfo(&free_b, &total_b));
    const double need = 1.25 * static_cast<double>(l.s->device_bytes()) + 1.0e9;
    if (!hc.agree(static_cast<double>(free_b) > need)) {
      for (int k = 0; k < rounds; ++k) {
        hc.barrier();
        const RunResult rk = l.s->run();
        l.best = std::min(l.best, rk.solve_s);
        l.stable = l.stable && rk.finite && (fake || rk.max_err == ref_log);
      }
      l.timed = true;
      l.best = hc.max(l.best);
      if (!hc.agree(l.stable)) {
        reject(c, "a timed solve's error log differs");
        continue;
      }
      // alone-timed candidates clearly slower than another alone-timed one are freed (they cannot be chosen)
      for (Live& o2 : live)
        if (o2.timed && o2.s && o2.best > l.best * (1.0 + tie)) o2.s.reset();
      for (Live& o2 : live)
        if (o2.timed && o2.s && l.best > o2.best * (1.0 + tie)) l.s.reset();
    }
    live.push_back(std::move(l));
  }
  W3D_REQUIRE(!live.empty(), "autotune: no candidate schedule could be built");
  // interleaved rounds: drift of the node (clocks, other jobs) hits every candidate alike
  for (int k = 0; k < rounds; ++k)
    for (Live& l : live) {
      if (l.timed || !l.s) continue;
      hc.barrier();
      const RunResult rk = l.s->run();
      l.best = std::min(l.best, rk.solve_s);
      l.stable = l.stable && rk.finite && (fake || rk.max_err == ref_log);
    }
  res.rounds = rounds;
  double best = 1e300;
  for (Live& l : live) {
    if (!l.timed) {
      l.best = hc.max(l.best);
      if (!hc.agree(l.stable)) {
        reject(l.c, "a timed solve's error log differs");
        l.s.reset();
        l.ok = false;
        continue;
      }
    }
    res.times.emplace_back(l.c.name, l.best);
    best = std::min(best, l.best);
  }
  W3D_REQUIRE(best < 1e299, "autotune: every candidate was rejected");
  // the simplest (earliest) candidate within `tie` of the fastest: candidates this close are not told apart reliably
  for (Live& l : live)
    if (l.ok && l.s && l.best <= best * (1.0 + tie)) {
      res.solver = std::move(l.s);
      res.name = l.c.name;
      break;
    }
  return res;
}

}  // namespace wave3d
