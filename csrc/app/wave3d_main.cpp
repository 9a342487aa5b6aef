// wave3d — standalone CLI, compatible with the reference's `mpigpu-1 N tau K 1` / `wave N tau K` invocations.
//
//   wave3d N tau K [L] [options]                 one GPU (or --cpu)
//   wave3d N tau K [L] --np P [options]          P ranks on P GPUs of this node (self-spawned, like `mpirun -np P`)
//   torchrun --no-python --nproc-per-node P bin/wave3d N tau K [L]   same, under an external launcher
//
// Reference CLI and output: report.pdf p.15 §4.2.4 (`mpirun -np 2 ./mpigpu-1 512 0.001 20 1`), p.15-16 §4.3 (per-step
// "Step %d, t = %f, Max Error = %e, L2 Error = %e" lines), p.16 §4.4 (timing breakdown); SURVEY.md §1.3-1.4, §5.5-5.6.
// Rank discovery: RANK/WORLD_SIZE/LOCAL_RANK (torchrun), OMPI_COMM_WORLD_*, PMI_RANK/PMI_SIZE, or the
// built-in --np self-spawn. The RCCL unique id travels through a rendezvous file (single node).
#include <fcntl.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cctype>
#include <chrono>
#include <cmath>
#include <cstring>
#include <ctime>
#include <fstream>
#include <iostream>
#include <memory>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "cli.hpp"
#include "wave3d/capture_guard.hpp"
#include "wave3d/cpu.hpp"
#include "wave3d/cpu_dist.hpp"
#include "wave3d/runtime.hpp"
#include "wave3d/solver.hpp"

using namespace wave3d;

using namespace wave3d::cli;

namespace {

// Ranks without a communicator (--no-rccl): the solve's error log over all ranks through the host collectives (L∞:
// max; RMS: from the per-rank Σe² shares)
void combine_logs(RunResult& r, const HostColl& hc) {
  std::string mine;
  for (size_t i = 0; i < r.steps.size(); ++i) {
    const double v[2] = {r.max_err[i], r.rms_err[i] * r.rms_err[i]};
    mine.append(reinterpret_cast<const char*>(v), sizeof v);
  }
  const std::vector<std::string> all = hc.allgather(mine);
  for (size_t i = 0; i < r.steps.size(); ++i) {
    double m = 0.0, q = 0.0;
    for (const std::string& b : all) {
      double v[2];
      std::memcpy(v, b.data() + i * sizeof v, sizeof v);
      m = v[0] > m || std::isnan(v[0]) ? v[0] : m;
      q += v[1];
    }
    r.max_err[i] = m;
    r.rms_err[i] = std::sqrt(q);
  }
}

// --serve (GPU): the rank's solver stays up and answers one command per stdin line (cli.hpp serve_loop) — the native
// rank process behind the Python Solver(runtime="process") (mpi_cuda_amd/parallel/native_proc.py): a torch process
// cannot capture the multi-rank schedules (HIP 7.0 runtime, see multistream_capture_safe), this process's ROCm 7.2
// runtime can. Every rank must receive the same command sequence (run and quit are collective).
//   run            one solve (barrier first): {"solve_s" (max over ranks), "local_s", "graph", "finite", "steps"}
//   hash W         field_hash of u^K (W = 0) / u^{K−1} (W = 1) over this rank's owned nodes
//   traffic        GpuSolver::traffic of the last solve's schedule
//   dump PREFIX    write u^K of this rank (wave3d-dump-v1)
//   quit           leave the loop (exit status 0)
int serve(const Args& a, GpuSolver& s, const HostColl& hc, bool file_coll, const std::string& sched) {
  const Dims d = s.dims();
  std::ostringstream g;
  g << "{\"ready\": true, \"backend\": \"hip\", \"rank\": " << s.rank() << ", \"world\": " << s.world()
    << ", \"dims\": [" << d.px << ", " << d.py << ", " << d.pz << "], \"schedule\": " << jstr(sched)
    << ", \"mode\": " << jstr(s.mode()) << ", \"transport\": " << jstr(s.transport()) << "}";
  return serve_loop(g.str(), [&](const std::string& cmd, std::istream& in) -> std::string {
    std::ostringstream o;
    if (cmd == "run") {
      if (hc.idle_barrier)
        hc.idle_barrier();
      else
        hc.barrier();
      RunResult r = s.run();
      const double t = hc.max(r.solve_s);
      if (file_coll) combine_logs(r, hc);
      o << "{\"solve_s\": " << jexact(t) << ", \"local_s\": " << jexact(r.solve_s) << ", \"graph\": "
        << (s.options().graph ? "true" : "false") << ", \"overlap\": " << (s.overlapped() ? "true" : "false")
        << ", \"finite\": " << (r.finite ? "true" : "false") << ", \"steps\": " << steps_exact(r.steps, r.max_err, r.rms_err)
        << "}";
    } else if (cmd == "hash") {
      int w = 0;
      in >> w;
      o << "{\"hash\": \"" << std::to_string(s.field_hash(w)) << "\"}";
    } else if (cmd == "traffic") {
      const GpuSolver::Traffic tr = s.traffic();
      o << "{\"field_bytes\": " << jexact(tr.field_bytes) << ", \"halo_bytes\": " << jexact(tr.halo_bytes) << "}";
    } else if (cmd == "dump") {
      std::string prefix;
      in >> prefix;
      write_dump(prefix, a.prob, s.layout(), s.download(0), s.rank(), s.world(), d);
      o << "{\"dump\": " << jstr(prefix) << "}";
    } else {
      o << "{\"error\": " << jstr("unknown command: " + cmd) << "}";
    }
    return o.str();
  });
}

int run_group(const Args& a, const SolverOptions& o, const hipDeviceProp_t& prop) {
  GpuGroup g(a.prob, o, a.group, a.group_transport);
  if (!a.resume.empty()) {
    std::vector<double> prev, cur;
    const int n0 = load_checkpoint(a.resume, a.prob, prev, cur);
    g.set_state(prev.data(), cur.data(), n0);
  }
  if (a.serve) {
    // --group P --serve: all P ranks in this process (the Python Solver(world=P, runtime="process") of ONE Python
    // process); run / hash (summed over the ranks) / traffic (summed) / dump (one file per rank) / quit
    const Dims d0 = g.rank(0).dims();
    std::ostringstream gr;
    gr << "{\"ready\": true, \"backend\": \"hip\", \"rank\": 0, \"world\": " << g.world() << ", \"dims\": [" << d0.px
       << ", " << d0.py << ", " << d0.pz << "], \"schedule\": " << jstr(g.rank(0).mode()) << ", \"mode\": "
       << jstr(g.rank(0).mode()) << ", \"transport\": " << jstr(g.transport()) << "}";
    return serve_loop(gr.str(), [&](const std::string& cmd, std::istream& in) -> std::string {
      std::ostringstream out;
      if (cmd == "run") {
        const RunResult r = g.run();
        out << "{\"solve_s\": " << jexact(r.solve_s) << ", \"local_s\": " << jexact(r.solve_s) << ", \"graph\": "
            << (g.graph_enabled() ? "true" : "false") << ", \"overlap\": false, \"finite\": "
            << (r.finite ? "true" : "false") << ", \"steps\": " << steps_exact(r.steps, r.max_err, r.rms_err) << "}";
      } else if (cmd == "hash") {
        int w = 0;
        in >> w;
        unsigned long long h = 0;
        for (int q = 0; q < g.world(); ++q) h += g.rank(q).field_hash(w);
        out << "{\"hash\": \"" << std::to_string(h) << "\"}";
      } else if (cmd == "traffic") {
        double fb = 0, hb = 0;
        for (int q = 0; q < g.world(); ++q) {
          const GpuSolver::Traffic t = g.rank(q).traffic();
          fb += t.field_bytes;
          hb += t.halo_bytes;
        }
        out << "{\"field_bytes\": " << jexact(fb) << ", \"halo_bytes\": " << jexact(hb) << "}";
      } else if (cmd == "dump") {
        std::string prefix;
        in >> prefix;
        for (int q = 0; q < g.world(); ++q)
          write_dump(prefix, a.prob, g.rank(q).layout(), g.rank(q).download(0), q, g.world(), d0);
        out << "{\"dump\": " << jstr(prefix) << "}";
      } else {
        out << "{\"error\": " << jstr("unknown command: " + cmd) << "}";
      }
      return out.str();
    });
  }
  RunResult r;
  double best = 1e30, sum = 0;
  for (int i = 0; i < a.warmup + a.repeat; ++i) {
    r = g.run();
    if (i >= a.warmup) {
      best = std::min(best, r.solve_s);
      sum += r.solve_s;
    }
  }
  const Dims d = g.rank(0).dims();
  if (!a.quiet) {
    std::printf("wave3d: N=%lld tau=%g K=%d L=%g group of %d ranks (%s) decomp=%dx%dx%d device=%s\n",
                static_cast<long long>(a.prob.N), a.prob.tau, a.prob.K, a.prob.L, a.group, a.group_transport.c_str(),
                d.px, d.py, d.pz, prop.gcnArchName);
    print_errors(r.steps, r.max_err, r.rms_err, a.prob.tau);
  }
  std::printf("Total time: %.6f s (group solve on one GPU; best of %d, mean %.6f s); schedule %s, graph %s\n", best,
              a.repeat, sum / a.repeat, g.rank(0).mode().c_str(), g.graph_enabled() ? "on" : "off");
  if (!a.dump.empty())
    for (int q = 0; q < g.world(); ++q)
      write_dump(a.dump, a.prob, g.rank(q).layout(), g.rank(q).download(0), q, g.world(), d);
  if (!a.checkpoint.empty())
    for (int q = 0; q < g.world(); ++q)
      write_checkpoint(a.checkpoint, a.prob, g.rank(q).layout(), g.rank(q).download(0), g.rank(q).download(1), q,
                       g.world(), d);
  if (!a.json.empty()) {
    std::vector<int> cc = g.comm_counts();
    std::ofstream j(a.json);
    j << "{\"backend\": \"hip\", \"group\": " << a.group << ", \"transport\": " << jstr(a.group_transport)
      << ", \"graph\": " << (g.graph_enabled() ? "true" : "false") << ", \"schedule\": " << jstr(g.rank(0).mode())
      << ", \"temporal\": " << g.rank(0).options().temporal << ", \"rccl_comms\": " << cc.size() << ", \"solve_s\": " << jnum(best) << ", \"steps\": [";
    for (size_t i = 0; i < r.steps.size(); ++i)
      j << (i ? ", " : "") << "[" << r.steps[i] << ", " << jnum(r.max_err[i]) << ", " << jnum(r.rms_err[i]) << "]";
    j << "]}\n";
  }
  return r.finite ? 0 : 3;
}

int run_gpu(const Args& a) {
  int rank = env_int(kRankEnv, 0), world = env_int(kSizeEnv, 1);
  const bool fake = a.fake_rank >= 0;
  if (fake) {
    rank = a.fake_rank;
    world = a.fake_world;
  }
  const double t_proc0 = wall_s();
  int ndev = 0;
  W3D_HIP(hipGetDeviceCount(&ndev));
  W3D_REQUIRE(ndev > 0, "no GPU visible (use --cpu for the CPU path)");
  const int local = env_int(kLocalEnv, rank);
  const int dev = local % ndev;
  W3D_HIP(hipSetDevice(dev));
  hipDeviceProp_t prop;
  W3D_HIP(hipGetDeviceProperties(&prop, dev));
  if (a.capture_selftest >= 0) {  // (tests: the stream-capture guard on this process's ROCm runtime)
    std::printf("capture selftest mode %d: %s\n", a.capture_selftest, capture::selftest(a.capture_selftest).c_str());
    return 0;
  }
  const SolverOptions base = options_from(a, fake);
  if (a.group > 0) return run_group(a, base, prop);

  std::shared_ptr<Comm> comm;
  const double t_comm0 = wall_s();
  if (fake && a.fake_traffic) {  // a one-rank communicator for the fake rank's self traffic (--fake-traffic)
    comm = std::make_shared<Comm>(0, 1, Comm::make_unique_id());
  } else if (world > 1 && !fake && !a.no_rccl) {
    W3D_REQUIRE(local < ndev || std::getenv("W3D_SHARE_GPUS"),
                "rank " + std::to_string(rank) + " has local rank " + std::to_string(local) + " but only " +
                    std::to_string(ndev) + " GPU(s) are visible (RCCL needs one GPU per rank)");
    const std::string id = exchange_unique_id(rank);
    comm = std::make_shared<Comm>(rank, world, id);
    if (rank == 0) std::remove(rdzv_path().c_str());
  }
  const double t_comm = wall_s() - t_comm0;
  const int rccl_nranks = comm ? comm->count() : 0;
  // fault injection: W3D_FAULT_RANK=r makes rank r fail right after the communicator is up; its peers
  // then fail in their next collective (GPU-wait timeout W3D_TIMEOUT_S) instead of hanging
  if (const char* fr = std::getenv("W3D_FAULT_RANK"); fr && std::atoi(fr) == rank && !std::getenv("W3D_FAULT_AT_SOLVE"))
    fail("injected fault");
  // host collectives: RCCL; files for ranks without a communicator (--no-rccl rehearsal, outside timed regions); none
  // for one rank or a fake rank
  const bool file_coll = !comm && world > 1 && !fake;
  const HostColl hc = comm && !fake ? HostColl::rccl(comm)
                      : file_coll       ? HostColl::files(rank, world)
                                        : HostColl::single(rank);
  W3D_REQUIRE(!a.no_rccl || world == 1 || fake || ((a.transport == "push" || a.transport == "sdma") && !a.autotune),
              "--no-rccl: ranks without a communicator can only run the push or sdma transport (no autotune)");
  std::unique_ptr<GpuSolver> s;
  std::string sched = a.decomp + "-S" + std::to_string(a.temporal) + (a.overlap ? "" : "-seq") +
                      (a.transport == "rccl" ? "" : "-" + a.transport);
  AutotuneResult tuned;
  if (a.autotune && (world > 1 || a.fake_rank < 0)) {
    AutotuneOptions ao;
    ao.with_push = a.transport == "push";
    const char* es = std::getenv("W3D_AUTOTUNE_SDMA");
    ao.with_sdma = a.autotune_sdma || a.transport == "sdma" || (es && *es == '1');
    ao.rounds = a.autotune_rounds;
    ao.reps = a.autotune_reps;
    ao.budget_s = a.autotune_budget;
    tuned = autotune(a.prob, base, rank, world, comm, hc, fake, ao);
    s = std::move(tuned.solver);
    sched = tuned.name;
  } else {
    s = std::make_unique<GpuSolver>(a.prob, base, rank, world, comm);
    connect_transport(*s, hc, fake);
  }

  if (!a.resume.empty()) {
    std::vector<double> prev, cur;
    const int n0 = load_checkpoint(a.resume, a.prob, prev, cur);
    s->set_state(prev.data(), cur.data(), n0);
  }
  if (a.serve) {
    const int rc = serve(a, *s, hc, file_coll, sched);
    if ((s->push() || s->sdma()) && !comm && !fake)
      std::remove((rdzv_path() + (s->push() ? ".push" : ".sdma") + std::to_string(rank)).c_str());
    hc.cleanup();
    return rc;
  }
  RunResult r;
  double best = 1e30, sum = 0, first = 0;
  // lost-peer injection: W3D_FAULT_RANK=r with W3D_FAULT_AT_SOLVE=i makes rank r vanish right after the barrier of
  // solve i, so its peers run into that solve alone (their transport waits must end it within one bound)
  const char* fas = std::getenv("W3D_FAULT_AT_SOLVE");
  const char* frk = std::getenv("W3D_FAULT_RANK");
  const int fault_at = fas && frk && std::atoi(frk) == rank ? std::atoi(fas) : -1;
  // --verify-repeat: this rank's local error log and field hash after every solve against the first solve's
  std::vector<double> ref_max, ref_rms;
  unsigned long long ref_hash = 0;
  int mismatches = 0;
  std::vector<double> times;  // this rank's solve times, warmup included (--json solve_times_s: tails, parity patterns)
  for (int i = 0; i < a.warmup + a.repeat; ++i) {
    hc.barrier();
    if (i == fault_at) fail("injected fault: rank " + std::to_string(rank) + " lost before solve " + std::to_string(i));
    r = s->run();
    times.push_back(r.solve_s);
    if (a.verify_repeat) {
      const unsigned long long h = s->field_hash(0);
      if (i == 0) {
        ref_max = r.max_err;
        ref_rms = r.rms_err;
        ref_hash = h;
      } else if (r.max_err != ref_max || r.rms_err != ref_rms || h != ref_hash) {
        if (mismatches++ < 5)
          std::fprintf(stderr, "wave3d: rank %d solve %d differs from solve 0 (field hash %016llx vs %016llx)\n", rank,
                       i, h, ref_hash);
      }
    }
    const double t = hc.max(r.solve_s);
    if (i == 0) first = t;
    if (i >= a.warmup) {
      best = std::min(best, t);
      sum += t;
    }
  }
  // --bench-steps K: the bench.py contract — K back-to-back solves bracketed by a device sync + barrier on both sides,
  // elapsed time max over ranks
  double bench_s = 0.0;
  if (a.bench_steps > 0) {
    W3D_HIP(hipDeviceSynchronize());
    hc.barrier();
    const double t0 = wall_s();
    const RunResult warm = r;
    // (W3D_BENCH_SYNC_EACH=1: one host round trip per solve, as before run_batch — A/B runs)
    std::vector<RunResult> rs;
    if (std::getenv("W3D_BENCH_SYNC_EACH"))
      for (int i = 0; i < a.bench_steps; ++i) rs.push_back(s->run());
    else
      rs = s->run_batch(a.bench_steps);
    W3D_HIP(hipDeviceSynchronize());
    hc.barrier();
    bench_s = hc.max(wall_s() - t0);
    // every timed solve's own log equals the warmup solve's (exact; a fake rank's ghosts are never filled: skipped)
    for (size_t i = 0; i < rs.size() && a.fake_rank < 0; ++i)
      if (rs[i].max_err != warm.max_err || rs[i].rms_err != warm.rms_err || !rs[i].finite)
        fail("bench: timed solve " + std::to_string(i) + " of rank " + std::to_string(rank) +
             " produced a different error log than the warmup solve");
    r = rs.back();
  }
  // per-phase breakdown of the schedule that was timed: one more solve with the same kernels, traced with events
  PhaseTimes ph;
  if (a.phases && !a.timers) {
    s->set_timers(true);  // same solver, same schedule and kernels, launched eagerly with events around each phase
    hc.barrier();
    ph = s->run().phases;
    s->set_timers(false);
    ph.init_ms = hc.max(ph.init_ms);
    ph.shell_ms = hc.max(ph.shell_ms);
    ph.interior_ms = hc.max(ph.interior_ms);
    ph.comm_ms = hc.max(ph.comm_ms);
    ph.check_ms = hc.max(ph.check_ms);
    ph.gather_ms = hc.max(ph.gather_ms);
  }
  if (file_coll) combine_logs(r, hc);
  if (a.verify_repeat) {
    const int bad = static_cast<int>(hc.max(static_cast<double>(mismatches)));
    if (rank == 0 || fake)
      std::printf("Repeat check: %d solves per rank, %s\n", a.warmup + a.repeat,
                  bad ? "SOME SOLVES DIFFER from the first" : "every solve bit-identical to the first on every rank");
    if (bad) return 4;
  }
  const double mean = sum / a.repeat;
  const double t_proc = wall_s() - t_proc0;
  const Dims d = s->dims();
  int hipv = 0;
  (void)hipRuntimeGetVersion(&hipv);
  if (rank == 0 || fake) {
    if (!a.quiet) {
      std::printf("wave3d: N=%lld tau=%g K=%d L=%g ranks=%d decomp=%dx%dx%d device=%s courant=%.3f\n",
                  static_cast<long long>(a.prob.N), a.prob.tau, a.prob.K, a.prob.L, world, d.px, d.py, d.pz,
                  prop.gcnArchName, a.prob.courant());
      print_errors(r.steps, r.max_err, r.rms_err, a.prob.tau);
    }
    const double gcell = a.prob.cell_updates() / best / 1e9;
    std::printf("Total time: %.6f s (solve region, max over %d rank%s; best of %d, mean %.6f s, first %.6f s)\n", best,
                world, world > 1 ? "s" : "", a.repeat, mean, first);
    std::printf(
        "Throughput: %.2f GCell/s; process wall-clock %.3f s (RCCL init %.3f s, %d ranks); schedule %s (%s), graph %s,"
        " overlap %s\n",
        gcell, t_proc, t_comm, rccl_nranks, s->mode().c_str(), sched.c_str(), s->options().graph ? "on" : "off",
        s->overlapped() ? "on" : "off");
    const GpuSolver::Traffic tr = s->traffic();
    std::printf("Traffic%s: %.3f GB of compulsory field reads + writes per solve = %.0f GB/s effective; halo %.2f MB"
                " sent per solve\n",
                world > 1 ? " (this rank)" : "", tr.field_bytes / 1e9, tr.field_bytes / best / 1e9, tr.halo_bytes / 1e6);
    if (a.bench_steps > 0)
      std::printf("Bench: %d solves in %.6f s (%.6f s per solve, max over ranks)\n", a.bench_steps, bench_s,
                  bench_s / a.bench_steps);
    const PhaseTimes& pp = a.timers ? r.phases : ph;
    if (a.timers || a.phases)
      std::printf(
          "Phases (%s, device ms, max over ranks): init %.3f | compute %.3f (shell %.3f) | exchange %.3f | check %.3f"
          " | error-log gather (all-gather + D2H) %.3f\n",
          a.timers ? "this run" : "traced solve of the timed schedule", pp.init_ms, pp.interior_ms + pp.shell_ms,
          pp.shell_ms, pp.comm_ms, pp.check_ms, pp.gather_ms);
    if (!a.json.empty()) {
      std::ofstream j(a.json);
      j << "{\"backend\": \"hip\", \"N\": " << a.prob.N << ", \"tau\": " << jnum(a.prob.tau) << ", \"K\": " << a.prob.K
        << ", \"L\": " << jnum(a.prob.L) << ", \"ranks\": " << world << ", \"dims\": [" << d.px << ", " << d.py
        << ", " << d.pz << "], \"solve_s\": " << jnum(best) << ", \"mean_s\": " << jnum(mean)
        << ", \"first_s\": " << jnum(first) << ", \"process_s\": " << jnum(t_proc) << ", \"rccl_init_s\": "
        << jnum(t_comm) << ", \"rccl_nranks\": " << rccl_nranks << ", \"rccl_version\": " << rccl_version()
        << ", \"hip_runtime\": " << hipv << ", \"gcell_per_s\": " << jnum(gcell)
        << ", \"field_bytes\": " << jnum(tr.field_bytes) << ", \"halo_bytes\": " << jnum(tr.halo_bytes)
        << ", \"effective_gbs\": " << jnum(tr.field_bytes / best / 1e9)
        << ", \"graph\": " << (s->options().graph ? "true" : "false") << ", \"overlap\": "
        << (s->overlapped() ? "true" : "false") << ", \"overlap_requested\": " << (s->options().overlap ? "true" : "false")
        << ", \"temporal\": " << s->options().temporal
        << ", \"schedule\": " << jstr(sched) << ", \"mode\": " << jstr(s->mode())
        << ", \"transport\": " << jstr(s->transport()) << ", \"device\": "
        << jstr(prop.gcnArchName) << ", \"bench_steps\": " << a.bench_steps << ", \"bench_s\": " << jnum(bench_s)
        << ", \"bench_pipelined\": " << (a.bench_steps > 0 && r.batched ? "true" : "false")
        << ", \"warmup\": " << a.warmup << ", \"finite\": " << (r.finite ? "true" : "false") << ", \"autotune_s\": {";
      for (size_t i = 0; i < tuned.times.size(); ++i)
        j << (i ? ", " : "") << jstr(tuned.times[i].first) << ": " << jnum(tuned.times[i].second);
      j << "}, \"autotune_best_s\": {";
      for (size_t i = 0; i < tuned.best_times.size(); ++i)
        j << (i ? ", " : "") << jstr(tuned.best_times[i].first) << ": " << jnum(tuned.best_times[i].second);
      j << "}, \"autotune_rounds\": " << tuned.rounds << ", \"autotune_reps\": " << tuned.reps
        << ", \"autotune_wall_s\": " << jnum(tuned.wall_s) << ", \"autotune_rejected\": {";
      for (size_t i = 0; i < tuned.rejected.size(); ++i)
        j << (i ? ", " : "") << jstr(tuned.rejected[i].first) << ": " << jstr(json_escape(tuned.rejected[i].second));
      j << "}";
      if (a.timers || a.phases)
        j << ", \"phases_ms\": {\"init\": " << jnum(pp.init_ms) << ", \"compute\": "
          << jnum(pp.interior_ms + pp.shell_ms) << ", \"shell\": " << jnum(pp.shell_ms) << ", \"exchange\": "
          << jnum(pp.comm_ms) << ", \"check\": " << jnum(pp.check_ms) << ", \"gather\": " << jnum(pp.gather_ms)
          << "}";
      j << ", \"solve_times_s\": [";
      for (size_t i = 0; i < times.size(); ++i) j << (i ? ", " : "") << jnum(times[i]);
      j << "], \"steps\": [";
      for (size_t i = 0; i < r.steps.size(); ++i)
        j << (i ? ", " : "") << "[" << r.steps[i] << ", " << jnum(r.max_err[i]) << ", " << jnum(r.rms_err[i]) << "]";
      j << "]}\n";
    }
  }
  if (!a.trace.empty()) {  // per-unit device times of the last run, one JSON object per line
    const std::string path = world > 1 ? a.trace + ".rank" + std::to_string(rank) : a.trace;
    std::ofstream t(path);
    t.precision(6);
    for (const UnitTrace& u : r.trace)
      t << "{\"rank\": " << rank << ", \"unit\": " << u.unit << ", \"n\": " << u.n << ", \"steps\": " << u.steps
        << ", \"schedule\": \"" << s->mode() << "\", \"shell_ms\": " << u.shell_ms << ", \"comm_ms\": " << u.comm_ms
        << ", \"compute_ms\": " << u.compute_ms << ", \"check_ms\": " << u.check_ms << "}\n";
  }
  if (!a.dump.empty()) write_dump(a.dump, a.prob, s->layout(), s->download(0), rank, world, d);
  if (!a.checkpoint.empty())
    write_checkpoint(a.checkpoint, a.prob, s->layout(), s->download(0), s->download(1), rank, world, d);
  if ((s->push() || s->sdma()) && !comm && !fake)
    std::remove((rdzv_path() + (s->push() ? ".push" : ".sdma") + std::to_string(rank)).c_str());
  hc.cleanup();
  return r.finite ? 0 : 3;
}

}  // namespace

int main(int argc, char** argv) {
  try {
    Args a = parse(argc, argv);
    a.prob.validate();
    if (!a.prob.cfl_ok()) {
      std::fprintf(stderr,
                   "wave3d: CFL violated: courant = tau*sqrt(3)/h = %.4f > 1 (tau_max = %.3e for N=%lld, L=%g); the "
                   "leapfrog scheme is unstable.%s\n",
                   a.prob.courant(), a.prob.tau_max(), static_cast<long long>(a.prob.N), a.prob.L,
                   a.force ? " Continuing (--force)." : " Use a smaller tau, or --force.");
      if (!a.force) return 2;
    }
    // multi-process CPU path: the shared segment is mapped before the fork so every rank inherits it (--np), or, for
    // ranks started by an external launcher, a named segment keyed by the job
    std::unique_ptr<ShmGroup> group;
    int cpu_rank = 0;
    if (a.cpu && a.np > 1 && !std::getenv("W3D_SPAWNED"))
      group = std::make_unique<ShmGroup>(a.prob, parse_dims(a.decomp, a.np, a.prob.N), a.np);
    if (a.np > 1 && !std::getenv("W3D_SPAWNED")) {
      const int rc = spawn_ranks(a.np);  // (fork before anything touches the GPU)
      if (rc >= 0) return rc;  // parent
    }
    if (group) cpu_rank = env_int(kRankEnv, 0);
    const int lworld = env_int(kSizeEnv, 1);
    if (a.cpu && !group && a.np <= 1 && lworld > 1 && a.fake_rank < 0) {
      cpu_rank = env_int(kRankEnv, 0);
      group = std::make_unique<ShmGroup>(a.prob, parse_dims(a.decomp, lworld, a.prob.N), lworld, job_segment_name(),
                                         cpu_rank);
    }
    const int rc = a.cpu ? (group ? run_cpu_rank(a, *group, cpu_rank) : run_cpu(a)) : run_gpu(a);
    if (rc == 3) std::fprintf(stderr, "wave3d: solution blew up (non-finite error)\n");
    return rc;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
}
