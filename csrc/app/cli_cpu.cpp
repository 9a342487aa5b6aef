// wave3d CLI: the CPU programs — the reference's sequential / OpenMP (`wave`, `wave3dOMP`) and MPI / MPI+OpenMP
// (`onlyMPI`, `mpiomp`) executables (readme.md:33-48, report.pdf p.20-26). See cli.hpp.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>

#include "cli.hpp"
#include "wave3d/cpu.hpp"
#include "wave3d/runtime.hpp"

namespace wave3d::cli {

int run_cpu(const Args& a) {
  CpuSolver s(a.prob, a.check_every, a.threads);
  if (!a.resume.empty()) {
    std::vector<double> prev, cur;
    const int n0 = load_checkpoint(a.resume, a.prob, prev, cur);
    s.set_state(prev.data(), cur.data(), n0);
  }
  if (a.serve) {  // (the rank-process protocol on the CPU solver: run / dump / quit — cli.hpp serve_loop)
    const std::string greeting = "{\"ready\": true, \"backend\": \"cpu\", \"rank\": 0, \"world\": 1, \"dims\": [1, 1, 1], "
                                 "\"schedule\": \"cpu-openmp\", \"mode\": \"cpu\", \"transport\": \"none\"}";
    return serve_loop(greeting, [&](const std::string& cmd, std::istream& in) -> std::string {
      if (cmd == "run") {
        const CpuResult r = s.run();
        return "{\"solve_s\": " + jexact(r.solve_s) + ", \"local_s\": " + jexact(r.solve_s) +
               ", \"graph\": false, \"overlap\": false, \"finite\": " + (r.finite ? "true" : "false") +
               ", \"steps\": " + steps_exact(r.steps, r.max_err, r.rms_err) + "}";
      }
      if (cmd == "dump") {
        std::string prefix;
        in >> prefix;
        write_dump(prefix, a.prob, s.layout(), s.field(0), 0, 1, Dims{1, 1, 1});
        return "{\"dump\": " + jstr(prefix) + "}";
      }
      return "{\"error\": " + jstr("unknown command: " + cmd) + "}";
    });
  }
  CpuResult r, rb;  // rb: the best solve (its phases are printed)
  double best = 1e30, sum = 0;
  for (int i = 0; i < a.warmup + a.repeat; ++i) {
    r = s.run();
    if (i >= a.warmup) {
      if (r.solve_s < best) rb = r;
      best = std::min(best, r.solve_s);
      sum += r.solve_s;
    }
  }
  double bench_s = 0.0;
  if (a.bench_steps > 0) {
    const double t0 = wall_s();
    for (int i = 0; i < a.bench_steps; ++i) r = s.run();
    bench_s = wall_s() - t0;
  }
  if (!a.quiet) print_errors(r.steps, r.max_err, r.rms_err, a.prob.tau);
  const double gcell = a.prob.cell_updates() / best / 1e9;
  std::printf("Total time: %.6f s (init %.6f s, compute %.6f s), threads %d, %.3f GCell/s\n", best, rb.init_s,
              rb.compute_s, cpu_max_threads(), gcell);
  // the reference's CPU phase columns (report.pdf p.16): one process has no halo (Dirichlet zeros are structural)
  std::printf("Phases (s): init %.6f | compute %.6f | boundary %.6f | exchange %.6f\n", rb.init_s, rb.compute_s,
              rb.boundary_s, rb.exchange_s);
  if (!a.json.empty()) {
    std::ofstream j(a.json);
    j << "{\"backend\": \"cpu\", \"N\": " << a.prob.N << ", \"tau\": " << jnum(a.prob.tau) << ", \"K\": "
      << a.prob.K << ", \"L\": " << jnum(a.prob.L) << ", \"ranks\": 1, \"dims\": [1, 1, 1], \"threads\": "
      << cpu_max_threads() << ", \"solve_s\": " << jnum(best) << ", \"mean_s\": " << jnum(sum / a.repeat)
      << ", \"gcell_per_s\": " << jnum(gcell) << ", \"schedule\": \"cpu-openmp\", \"bench_steps\": " << a.bench_steps
      << ", \"bench_s\": " << jnum(bench_s) << ", \"finite\": " << (r.finite ? "true" : "false")
      << ", \"phases_s\": {\"init\": " << jnum(rb.init_s) << ", \"compute\": " << jnum(rb.compute_s)
      << ", \"boundary\": " << jnum(rb.boundary_s) << ", \"exchange\": " << jnum(rb.exchange_s) << "}"
      << ", \"phases_slowest_rank_s\": {\"init\": " << jnum(rb.init_s) << ", \"compute\": " << jnum(rb.compute_s)
      << ", \"boundary\": " << jnum(rb.boundary_s) << ", \"exchange\": " << jnum(rb.exchange_s) << "}"
      << ", \"steps\": " << steps_json(r.steps, r.max_err, r.rms_err) << "}\n";
  }
  if (!a.dump.empty()) write_dump(a.dump, a.prob, s.layout(), s.field(0), 0, 1, Dims{1, 1, 1});
  if (!a.checkpoint.empty())
    write_checkpoint(a.checkpoint, a.prob, s.layout(), s.field(0), s.field(1), 0, 1, Dims{1, 1, 1});
  return r.finite ? 0 : 3;
}

// One rank of the multi-process CPU path (--cpu --np P): the reference's MPI / MPI+OpenMP programs.
int run_cpu_rank(const Args& a, ShmGroup& g, int rank) {
  W3D_REQUIRE(a.resume.empty(), "--resume runs on one CPU process (--cpu) or on the GPU path, not the CPU ranks");
  try {
    CpuRankSolver s(a.prob, g, rank, a.check_every, a.threads);
    // fault injection: W3D_FAULT_RANK=r makes rank r fail before its first exchange
    if (const char* fr = std::getenv("W3D_FAULT_RANK"); fr && std::atoi(fr) == rank) fail("injected fault");
    CpuResult r, rb;  // rb: the best solve (its phases, each the max over ranks, are printed)
    double best = 1e30, sum = 0;
    for (int i = 0; i < a.warmup + a.repeat; ++i) {
      r = s.run();
      if (i >= a.warmup) {
        if (r.solve_s < best) rb = r;
        best = std::min(best, r.solve_s);
        sum += r.solve_s;
      }
    }
    const double exch = rb.exchange_s;
    double bench_s = 0.0;  // the end barrier waits for the slowest rank: rank 0's interval is the max over ranks
    if (a.bench_steps > 0) {
      g.barrier();
      const double t0 = wall_s();
      for (int i = 0; i < a.bench_steps; ++i) r = s.run();
      g.barrier();
      bench_s = wall_s() - t0;
    }
    const Dims d = g.dims();
    if (rank == 0) {
      if (!a.quiet) print_errors(r.steps, r.max_err, r.rms_err, a.prob.tau);
      const double gcell = a.prob.cell_updates() / best / 1e9;
      std::printf("Total time: %.6f s (max over %d ranks, decomp %dx%dx%d; exchange %.6f s), threads %d per rank, "
                  "%.3f GCell/s\n", best, g.world(), d.px, d.py, d.pz, exch, cpu_max_threads(), gcell);
      std::printf("Phases (s, max over ranks): init %.6f | compute %.6f | boundary %.6f | exchange %.6f\n", rb.init_s,
                  rb.compute_s, rb.boundary_s, rb.exchange_s);
      std::printf("Phases (s, slowest rank): init %.6f | compute %.6f | boundary %.6f | exchange %.6f\n",
                  rb.slow_phases[0], rb.slow_phases[1], rb.slow_phases[2], rb.slow_phases[3]);
      if (!a.json.empty()) {
        std::ofstream j(a.json);
        j << "{\"backend\": \"cpu\", \"ranks\": " << g.world() << ", \"dims\": [" << d.px << ", " << d.py << ", "
          << d.pz << "], \"N\": " << a.prob.N << ", \"tau\": " << a.prob.tau << ", \"K\": " << a.prob.K
          << ", \"L\": " << a.prob.L << ", \"threads\": " << cpu_max_threads() << ", \"solve_s\": " << best
          << ", \"mean_s\": " << sum / a.repeat << ", \"exchange_s\": " << exch << ", \"gcell_per_s\": " << gcell
          << ", \"final_max_err\": " << (r.max_err.empty() ? 0.0 : r.max_err.back())
          << ", \"final_rms_err\": " << (r.rms_err.empty() ? 0.0 : r.rms_err.back())
          << ", \"schedule\": \"cpu-openmp-ranks\", \"bench_steps\": " << a.bench_steps << ", \"bench_s\": "
          << jnum(bench_s) << ", \"finite\": " << (r.finite ? "true" : "false")
          << ", \"phases_s\": {\"init\": " << jnum(rb.init_s) << ", \"compute\": " << jnum(rb.compute_s)
          << ", \"boundary\": " << jnum(rb.boundary_s) << ", \"exchange\": " << jnum(rb.exchange_s) << "}"
          << ", \"phases_slowest_rank_s\": {\"init\": " << jnum(rb.slow_phases[0]) << ", \"compute\": "
          << jnum(rb.slow_phases[1]) << ", \"boundary\": " << jnum(rb.slow_phases[2]) << ", \"exchange\": "
          << jnum(rb.slow_phases[3]) << "}"
          << ", \"steps\": " << steps_json(r.steps, r.max_err, r.rms_err) << "}\n";
      }
    }
    if (!a.dump.empty()) write_dump(a.dump, a.prob, s.layout(), s.field(0), rank, g.world(), d);
    if (!a.checkpoint.empty())
      write_checkpoint(a.checkpoint, a.prob, s.layout(), s.field(0), s.field(1), rank, g.world(), d);
    return r.finite ? 0 : 3;
  } catch (...) {
    g.abort();  // the other ranks leave their barriers with an error instead of waiting for the timeout
    throw;
  }
}

// Solver options from the command line (one candidate of the multi-rank schedule autotune overrides a few of them).
}  // namespace wave3d::cli
