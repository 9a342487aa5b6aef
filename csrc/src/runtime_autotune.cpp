// Multi-rank schedule autotune of the native runtime (bench.py's --autotune on every rank; Python Solver(autotune=True)).
// See wave3d/runtime.hpp.
//
// Why a runtime choice: the halo volume of S-deep passes against the per-step exchanges of single steps, overlap against
// whole passes, slabs against blocks and RCCL copy kernels against the copy engines trade xGMI bandwidth and latency
// against HBM traffic and compute units, and the balance depends on the node. So every
// candidate is timed on the real interconnect and all ranks adopt the one whose slowest rank was fastest.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "wave3d/runtime.hpp"

namespace wave3d {

std::vector<Candidate> autotune_candidates(int world, bool with_push, bool with_sdma) {
  std::vector<Candidate> v;
  auto add = [&](const char* name, const char* decomp, const char* transport, int temporal, bool overlap,
                 int streams = 0, bool conc = false, int reserve = 0) {
    v.push_back(Candidate{name, decomp, transport, temporal, overlap, streams, conc, reserve});
  };
  if (world <= 1) {  // one rank: only the pass depth matters
    add("slab-S5", "slab", "rccl", 5, true);
    add("slab-S4", "slab", "rccl", 4, true);
    add("slab-S3", "slab", "rccl", 3, true);
    add("slab-S2", "slab", "rccl", 2, true);
    add("slab-S1", "slab", "rccl", 1, true);
    return v;
  }
  // simplest first: sequential before overlapped, RCCL before the copy engines, deep passes before shallow ones.
  // The copy-engine and push candidates are opt-in across devices: neither has yet run between two GPUs (every
  // rehearsal shared one GPU); a fake rank (one process) always includes the copy engines.
  add("slab-S4-seq", "slab", "rccl", 4, false);
  add("slab-S5-seq", "slab", "rccl", 5, false);  // (pair-tiled 5-step passes: one exchange per 5 steps)
  add("slab-S4", "slab", "rccl", 4, true);
  add("slab-S5", "slab", "rccl", 5, true);
  // (overlapped RCCL with 16 CUs — two per XCD — kept free of the passes: RCCL's kernels start at once instead of after
  // the pass's last workgroups; the pass loses 1/16 of the CUs)
  add("slab-S4-rsv16", "slab", "rccl", 4, true, 0, false, 16);
  if (with_sdma) {
    add("slab-S4-sdma-seq", "slab", "sdma", 4, false);
    add("slab-S5-sdma-seq", "slab", "sdma", 5, false);
    add("slab-S4-sdma", "slab", "sdma", 4, true);
    add("slab-S5-sdma", "slab", "sdma", 5, true);  // (the 5-step pass beside the copy-engine transfer)
  }
  if (with_push) {
    add("slab-S4-push-seq", "slab", "push", 4, false);
    add("slab-S4-push", "slab", "push", 4, true);
  }
  add("slab-S3", "slab", "rccl", 3, true);
  add("slab-S2", "slab", "rccl", 2, true);
  add("slab-S1", "slab", "rccl", 1, true);
  if (world >= 4) {  // (2 ranks: "block" is the slab)
    add("block-S4-seq", "block", "rccl", 4, false);
    add("block-S5-seq", "block", "rccl", 5, false);  // (pair-tiled 5-step passes over the whole block)
    add("block-S4", "block", "rccl", 4, true);
    add("block-S5", "block", "rccl", 5, true);  // (pair-tiled shells and interior, cut on whole pairs)
    add("block-S4-conc", "block", "rccl", 4, true, 0, true);  // (shells beside the interior)
    add("block-S4-rsv16", "block", "rccl", 4, true, 0, false, 16);
    if (with_sdma) {
      add("block-S4-sdma-seq", "block", "sdma", 4, false);
      add("block-S5-sdma-seq", "block", "sdma", 5, false);
      add("block-S4-sdma", "block", "sdma", 4, true);         // (one copy stream)
      add("block-S5-sdma", "block", "sdma", 5, true);
      add("block-S4-sdma-x2", "block", "sdma", 4, true, 2);  // (two copy streams: two engines)
    }
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
         std::to_string(s.sdma() ? s.copy_streams() : 0) + (s.overlapped() && s.options().shells_concurrent ? "/conc" : "") +
         (s.options().reserve_cus > 0 ? "/rsv" + std::to_string(s.options().reserve_cus) : "");
}
}  // namespace

AutotuneResult autotune(const Problem& prob, const SolverOptions& base, int rank, int world, std::shared_ptr<Comm> comm,
                        const HostColl& hc, bool fake, const AutotuneOptions& ao) {
  struct Live {
    Candidate c;
    std::unique_ptr<GpuSolver> s;
    std::vector<double> per;  // per round: mean of `reps` back-to-back solves (max over ranks)
    double med = 1e300, best = 1e300;
    bool stable = true;
    bool timed = false;  // timed alone already (memory)
    bool ok = true;      // accepted (its solver may still have been freed: timed alone and clearly slower)
  };
  std::vector<Live> live;
  std::vector<std::string> sigs;
  std::vector<double> ref_max, ref_rms;
  unsigned long long ref_hash[2] = {0, 0};
  bool have_ref = false;
  AutotuneResult res;
  const int rounds = std::max(1, ao.rounds), reps = std::max(1, ao.reps);
  const double t_start = wall_s();
  // (every rank takes the same branch: the slowest rank's elapsed time decides)
  auto over_budget = [&] { return ao.budget_s > 0.0 && hc.max(wall_s() - t_start) > ao.budget_s; };
  auto reject = [&](const Candidate& c, const std::string& why) {
    res.rejected.emplace_back(c.name, why);
    std::fprintf(stderr, "[wave3d rank %d] candidate %s rejected: %s\n", rank, c.name.c_str(), why.c_str());
  };
  // the log and the field a solve left must be the reference schedule's: L∞ exactly (a max is order-free), the RMS to
  // 1e-12 (its Σe² is summed per rank, so the decomposition moves its last bits), and u^K, u^{K−1} bit for bit through
  // the decomposition-free field hash summed over the ranks (a wrong ghost far from the L∞ node shows there)
  auto global_hash = [&](const GpuSolver& s, int which) {
    const unsigned long long h = s.field_hash(which);
    unsigned long long sum = 0;
    for (const std::string& b : hc.allgather(std::string(reinterpret_cast<const char*>(&h), sizeof h))) {
      unsigned long long x = 0;
      std::memcpy(&x, b.data(), sizeof x);
      sum += x;
    }
    return sum;
  };
  auto same_log = [&](const RunResult& r) {
    if (!r.finite) return false;
    if (fake || !have_ref) return true;
    if (r.max_err != ref_max || r.rms_err.size() != ref_rms.size()) return false;
    for (size_t i = 0; i < ref_rms.size(); ++i)
      if (!(std::fabs(r.rms_err[i] - ref_rms[i]) <= 1e-12 * std::fabs(ref_rms[i]))) return false;
    return true;
  };
  // one timing round of a candidate: `reps` back-to-back solves between barriers, as the bench runs them
  auto time_round = [&](Live& l) {
    hc.barrier();
    const double t0 = wall_s();
    RunResult rk;
    for (int k = 0; k < reps; ++k) {
      rk = l.s->run();
      l.stable = l.stable && same_log(rk);
    }
    const double t = hc.max((wall_s() - t0) / reps);
    l.per.push_back(t);
    l.best = std::min(l.best, t);
  };
  auto median = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    const size_t n = v.size();
    return n == 0 ? 1e300 : n % 2 ? v[n / 2] : 0.5 * (v[n / 2 - 1] + v[n / 2]);
  };
  bool stopped = false;
  for (const Candidate& c : autotune_candidates(world, ao.with_push, ao.with_sdma || fake)) {
    if (!stopped && over_budget()) stopped = true;
    if (stopped) {
      reject(c, "autotune wall-time budget spent");
      continue;
    }
    SolverOptions o = base;
    o.decomp = c.decomp;
    o.temporal = c.temporal;
    o.overlap = c.overlap;
    o.push = c.transport == "push";
    o.sdma = c.transport == "sdma";
    if (c.sdma_streams > 0) o.sdma_streams = c.sdma_streams;
    o.shells_concurrent = o.shells_concurrent || c.shells_concurrent;
    if (c.reserve_cus > 0) o.reserve_cus = c.reserve_cus;
    // a short in-kernel flag bound while tuning: a candidate whose peer is lost costs seconds (k_flag_sync ends the
    // rest of the solve's waits after the first timeout); baked into the graphs, so the chosen solver keeps it
    if (ao.flag_timeout_s > 0.0 && (o.flag_timeout_s <= 0.0 || o.flag_timeout_s > ao.flag_timeout_s))
      o.flag_timeout_s = ao.flag_timeout_s;
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
    // every schedule computes bit-identical fields: a candidate that fails (a transport wait timed out) or whose log
    // or field differs from the first accepted one's (a transport that delivered wrong ghosts) is rejected everywhere
    bool same = false;
    RunResult r0;
    try {
      r0 = cand->run();  // eager: RCCL peer connections
      r0 = cand->run();  // graph capture
      same = same_log(r0);
      if (!same) err = "its error log differs from the reference schedule's";
    } catch (const std::exception& e) {
      err = e.what();
    }
    if (!hc.agree(same)) {
      reject(c, err.empty() ? "failed on another rank" : err);
      continue;
    }
    if (!fake) {  // (a fake rank's field is its own box with stale ghosts: nothing to compare)
      const unsigned long long h0 = global_hash(*cand, 0), h1 = global_hash(*cand, 1);
      if (!have_ref) {
        ref_max = r0.max_err;
        ref_rms = r0.rms_err;
        ref_hash[0] = h0;
        ref_hash[1] = h1;
        have_ref = true;
      } else if (h0 != ref_hash[0] || h1 != ref_hash[1]) {  // (the same on every rank: a global sum)
        reject(c, "its final fields differ from the reference schedule's (field hash)");
        continue;
      }
    }
    sigs.push_back(sig);
    Live l{c, std::move(cand)};
    // keep it for the interleaved rounds if the next candidate still fits next to it; else time it alone now
    size_t free_b = 0, total_b = 0;
    W3D_HIP(hipMemGetInfo(&free_b, &total_b));
    const double need = 1.25 * static_cast<double>(l.s->device_bytes()) + 1.0e9;
    if (!hc.agree(static_cast<double>(free_b) > need)) {
      for (int k = 0; k < rounds; ++k) time_round(l);
      l.timed = true;
      l.med = median(l.per);
      if (!hc.agree(l.stable)) {
        reject(c, "a timed solve's error log differs");
        continue;
      }
      // alone-timed candidates clearly slower than another alone-timed one are freed (they cannot be chosen)
      for (Live& o2 : live)
        if (o2.timed && o2.s && o2.med > l.med * (1.0 + ao.tie)) o2.s.reset();
      for (Live& o2 : live)
        if (o2.timed && o2.s && l.med > o2.med * (1.0 + ao.tie)) l.s.reset();
    }
    live.push_back(std::move(l));
  }
  W3D_REQUIRE(!live.empty(), "autotune: no candidate schedule could be built");
  // interleaved rounds: drift of the node (clocks, other jobs) hits every candidate alike; the budget may end them
  // early (every surviving candidate then has the same number of rounds, at least one)
  int done_rounds = 0;
  for (int k = 0; k < rounds; ++k) {
    if (k > 0 && over_budget()) break;
    for (Live& l : live)
      if (!l.timed && l.s) time_round(l);
    ++done_rounds;
  }
  res.rounds = done_rounds;
  res.reps = reps;
  double best = 1e300;
  for (Live& l : live) {
    if (!l.timed) {
      l.med = median(l.per);
      if (!hc.agree(l.stable)) {
        reject(l.c, "a timed solve's error log differs");
        l.s.reset();
        l.ok = false;
        continue;
      }
    }
    res.times.emplace_back(l.c.name, l.med);
    res.best_times.emplace_back(l.c.name, l.best);
    best = std::min(best, l.med);
  }
  W3D_REQUIRE(best < 1e299, "autotune: every candidate was rejected");
  // the simplest (earliest) candidate within `tie` of the fastest median: candidates this close are not told apart
  // reliably
  for (Live& l : live)
    if (l.ok && l.s && l.med <= best * (1.0 + ao.tie)) {
      res.solver = std::move(l.s);
      res.name = l.c.name;
      break;
    }
  res.wall_s = wall_s() - t_start;
  return res;
}

}  // namespace wave3d
