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

#include "wave3d/cpu.hpp"
#include "wave3d/cpu_dist.hpp"
#include "wave3d/runtime.hpp"
#include "wave3d/solver.hpp"

using namespace wave3d;

namespace {

struct Args {
  Problem prob;
  bool have_L = false;
  std::string decomp = "slab";
  int check_every = 2;
  bool cpu = false;
  int threads = 0;
  bool overlap = true;
  bool graph = true;
  bool timers = false;
  bool debug_sync = false;
  bool poison = false;
  int temporal = 4;
  bool tb = true;
  int tb_threads = 0;
  int tb_init_threads = 0;
  bool init2 = true;
  int fake_rank = -1, fake_world = 0;
  int group = 0;                       // --group P: all P ranks in this process on one GPU
  int bench_steps = 0;                 // --bench-steps K: timed block of K solves (bench.py contract)
  bool autotune = false;               // --autotune: time the multi-rank schedule candidates, keep the fastest
  int autotune_rounds = 5;             // --autotune-rounds R: interleaved timing rounds
  bool phases = false;                 // --phases: per-phase breakdown from a traced solve of the timed schedule
  std::string group_transport = "rccl-self";
  std::string transport = "rccl";      // --transport rccl | push (slab LDS passes: halos pushed by the passes)
  bool push_cp_wait = false;           // --push-cp-wait: push waits by the command processor (eager launches)
  bool no_rccl = false;                // --no-rccl: ranks without a communicator (push rehearsal on one shared GPU)
  int t2_rows = 0, t2_target = -1, deep_min = -1, t2_occ = -1, tb_min = -1;
  bool force = false;
  int repeat = 1;
  int warmup = 0;
  int np = 0;
  int tile_rows = -1;
  int variant = -1;
  int target_blocks = 0;
  int nt_store = -1;
  std::string json, dump, trace, checkpoint, resume;
  bool quiet = false;
  std::string program = "wave3d";  // reference program personality (argv[0])
};

// The reference's five programs (readme.md:33-62, report.pdf p.11-15, p.20-26) by executable name, so
// symlinks to this binary accept their command lines unchanged:
//   wave N tau K                 sequential          openmpwave / wave3dOMP N tau K T   OpenMP, T threads
//   [mpirun -np P] onlyMPI|mpi N tau K              MPI: one CPU process per rank
//   [mpirun -np P] mpiomp N tau K T                 MPI+OpenMP: P processes × T threads
//   [mpirun -np P] mpigpu-1 N tau K L               MPI+CUDA → one MI355X per rank (the 4th argument is L)
// (ranks under an external launcher come from its environment; `--np P` spawns them here instead)
struct Personality {
  const char* name;
  bool cpu;
  bool pos4_threads;  // 4th positional = OpenMP threads (else L)
  int threads;        // default threads (0: OpenMP default)
};
constexpr Personality kPersonalities[] = {
    {"wave", true, false, 1},      {"openmpwave", true, true, 0}, {"wave3dOMP", true, true, 0},
    {"onlyMPI", true, false, 1},   {"mpi", true, false, 1},       {"mpiomp", true, true, 0},
    {"mpigpu-1", false, false, 0},
};

[[noreturn]] void usage(const char* msg = nullptr) {
  if (msg) std::fprintf(stderr, "wave3d: %s\n\n", msg);
  std::fprintf(stderr,
               "usage: wave3d N tau K [L] [options]\n"
               "  N        intervals per axis ((N+1)^3 nodes)      tau   time step\n"
               "  K        number of steps                          L     cube edge (default 1)\n"
               "options:\n"
               "  --np P             spawn P ranks on this node (one GPU each; with --cpu: P CPU processes, the\n"
               "                     reference's MPI / MPI+OpenMP programs, halos through shared memory)\n"
               "  --decomp D         slab | block | PxQxR (default slab)\n"
               "  --check-every C    error check cadence (default 2, as the reference)\n"
               "  --cpu [--threads T] sequential/OpenMP CPU path\n"
               "  --no-overlap       halo exchange on the compute stream (A/B switch)\n"
               "  --no-graph         eager launches instead of one captured hipGraph\n"
               "  --timers           per-phase GPU timers (init / compute / exchange / check)\n"
               "  --no-temporal      one leapfrog step per HBM pass (disable temporal blocking)\n"
               "  --temporal S       at most S (2..4) leapfrog steps per HBM pass (default 4)\n"
               "  --no-tb            two-step register-queue passes instead of the LDS S-step kernel\n"
               "  --tb-min-planes M  slab ranks: LDS S-step passes with S-deep halos from M owned planes (default 16)\n"
               "  --deep-min-planes M  slab ranks without the LDS kernel: two-step passes from M planes (default 96)\n"
               "  --tb-threads T     LDS S-step kernel workgroup size (768 or 1024; default 1024)\n"
               "  --tb-init-threads T  ... of the analytic-start pass (768 or 1024; default 768)\n"
               "  --no-init2         start from u0,u1 + a first step instead of analytic u1,u2\n"
               "  --debug-sync       synchronize after every step (race triage)\n"
               "  --poison-ghosts    NaN-fill ghost layers before every exchange (missed-halo detector)\n"
               "  --fake-rank R/P    perf study: time rank R of a P-rank decomposition alone on one GPU, no transport\n"
               "  --group P          all P ranks of the decomposition in this process on one GPU (rehearsal of the\n"
               "                     multi-rank path; --group-transport rccl-self (default: RCCL send/recv, each rank\n"
               "                     over a one-rank communicator), loopback (device copies) or push)\n"
               "  --transport T      rccl (default) | push: slab LDS passes store their face planes straight into the\n"
               "                     neighbours' fine-grained staging over xGMI and signal them with flags (no exchange)\n"
               "  --push-cp-wait     push: wait for the neighbours with hipStreamWaitValue32 (eager) instead of in-kernel\n"
               "  --no-rccl          ranks without an RCCL communicator (push only; IPC handles through files; error\n"
               "                     logs per rank): the multi-process push rehearsal on one shared GPU\n"
               "  --t2-rows R / --t2-target W   fused two-step kernel: rows per wave, x-chunking target (waves)\n"
               "  --repeat R / --warmup W   timed / untimed solves (report min and mean)\n"
               "  --bench-steps K    then K back-to-back solves between two sync+barriers (max over ranks)\n"
               "  --autotune         time the multi-rank schedule candidates (slab S4/S4-seq/S4-push/S3/S2/S1, block S4/S4-seq/S3/S1)\n"
               "                     and\n"
               "                     keep the fastest (slowest rank decides)\n"
               "  --phases           per-phase device times (init/compute/exchange/check) of the timed schedule\n"
               "  --variant V        leapfrog kernel: 1 = register-queue waves (default), 0 = LDS-staged tile\n"
               "  --tile-rows T      rows per wave (v1: 1,2,4,8) or per workgroup (v0: 4,8,16)\n"
               "  --target-blocks B  x-chunking target (waves for v1, workgroups for v0)\n"
               "  --nt-store 0/1     non-temporal stores of u^{n+1} (default 1)\n"
               "  --json PATH        machine-readable summary (rank 0)\n"
               "  --trace PATH       per-unit device times as JSON lines (PATH[.rankR] per rank; implies --timers)\n"
               "  --dump PREFIX      write u^K: PREFIX[.rankR].bin (fp64, C order, owned nodes) + .json\n"
               "  --checkpoint P     write u^{K-1}, u^K as P.prev / P.cur dumps (resumable)\n"
               "  --resume P         start from the P.prev / P.cur checkpoint (step n0) and continue to K\n"
               "  --force            run even if the CFL condition is violated\n"
               "  --quiet            only the summary\n");
  std::exit(2);
}

Args parse(int argc, char** argv) {
  Args a;
  const Personality* pers = nullptr;
  {
    std::string prog = argv[0];
    const size_t sl = prog.find_last_of('/');
    if (sl != std::string::npos) prog = prog.substr(sl + 1);
    for (const Personality& q : kPersonalities)
      if (prog == q.name) pers = &q;
    if (pers) {
      a.program = pers->name;
      a.cpu = pers->cpu;
      a.threads = pers->threads;
    }
  }
  std::vector<std::string> pos;
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) usage(("missing value for " + s).c_str());
      return argv[++i];
    };
    if (s == "--np") a.np = std::stoi(next());
    else if (s == "--decomp") a.decomp = next();
    else if (s == "--check-every") a.check_every = std::stoi(next());
    else if (s == "--cpu") a.cpu = true;
    else if (s == "--threads") a.threads = std::stoi(next());
    else if (s == "--no-overlap") a.overlap = false;
    else if (s == "--no-graph") a.graph = false;
    else if (s == "--timers") a.timers = true;
    else if (s == "--debug-sync") a.debug_sync = true;
    else if (s == "--poison-ghosts") a.poison = true;
    else if (s == "--no-temporal") a.temporal = 1;
    else if (s == "--temporal") a.temporal = std::stoi(next());
    else if (s == "--no-tb") a.tb = false;
    else if (s == "--tb-threads") a.tb_threads = std::stoi(next());
    else if (s == "--tb-init-threads") a.tb_init_threads = std::stoi(next());
    else if (s == "--no-init2") a.init2 = false;
    else if (s == "--t2-rows") a.t2_rows = std::stoi(next());
    else if (s == "--deep-min-planes") a.deep_min = std::stoi(next());
    else if (s == "--tb-min-planes") a.tb_min = std::stoi(next());
    else if (s == "--t2-target") a.t2_target = std::stoi(next());
    else if (s == "--t2-occ") a.t2_occ = std::stoi(next());
    else if (s == "--fake-rank") {
      const std::string v = next();  // R/P: time rank R of a P-rank decomposition alone, no transport
      a.fake_rank = std::stoi(v.substr(0, v.find('/')));
      a.fake_world = std::stoi(v.substr(v.find('/') + 1));
    }
    else if (s == "--group") a.group = std::stoi(next());
    else if (s == "--bench-steps") a.bench_steps = std::stoi(next());
    else if (s == "--autotune") a.autotune = true;
    else if (s == "--autotune-rounds") a.autotune_rounds = std::stoi(next());
    else if (s == "--phases") a.phases = true;
    else if (s == "--group-transport") a.group_transport = next();
    else if (s == "--transport") a.transport = next();
    else if (s == "--push-cp-wait") a.push_cp_wait = true;
    else if (s == "--no-rccl") a.no_rccl = true;
    else if (s == "--repeat") a.repeat = std::stoi(next());
    else if (s == "--warmup") a.warmup = std::stoi(next());
    else if (s == "--tile-rows") a.tile_rows = std::stoi(next());
    else if (s == "--variant") a.variant = std::stoi(next());
    else if (s == "--target-blocks") a.target_blocks = std::stoi(next());
    else if (s == "--nt-store") a.nt_store = std::stoi(next());
    else if (s == "--json") a.json = next();
    else if (s == "--trace") {
      a.trace = next();
      a.timers = true;
    }
    else if (s == "--dump") a.dump = next();
    else if (s == "--checkpoint") a.checkpoint = next();
    else if (s == "--resume") a.resume = next();
    else if (s == "--force") a.force = true;
    else if (s == "--quiet") a.quiet = true;
    else if (s == "-h" || s == "--help") usage();
    else if (!s.empty() && s[0] == '-' && s.size() > 1 && !std::isdigit(static_cast<unsigned char>(s[1])) && s[1] != '.')
      usage(("unknown option " + s).c_str());
    else pos.push_back(s);
  }
  if (pos.size() < 3 || pos.size() > 4) usage("expected positional N tau K [L]");
  a.prob.N = std::stoll(pos[0]);
  a.prob.tau = std::stod(pos[1]);
  a.prob.K = std::stoi(pos[2]);
  if (pos.size() == 4) {
    if (pers && pers->pos4_threads) {
      a.threads = std::stoi(pos[3]);
    } else {
      a.prob.L = std::stod(pos[3]);
      a.have_L = true;
    }
  }
  if (a.repeat < 1) a.repeat = 1;
  return a;
}

void print_errors(const std::vector<int>& steps, const std::vector<double>& mx, const std::vector<double>& rms,
                  double tau) {
  for (size_t i = 0; i < steps.size(); ++i)
    std::printf("Step %d, t = %f, Max Error = %e, L2 Error = %e\n", steps[i], steps[i] * tau, mx[i], rms[i]);
}

// json helpers for the summary line
std::string jstr(const std::string& v) { return "\"" + v + "\""; }
std::string json_escape(const std::string& v) {
  std::string o;
  for (char c : v) {
    if (c == '"' || c == '\\') o += '\\';
    if (static_cast<unsigned char>(c) >= 0x20) o += c;
  }
  return o;
}
std::string jnum(double v) {
  char b[64];
  std::snprintf(b, sizeof b, "%.10g", v);
  return b;
}
std::string steps_json(const std::vector<int>& st, const std::vector<double>& mx, const std::vector<double>& rms) {
  std::string o = "[";
  for (size_t i = 0; i < st.size(); ++i)
    o += (i ? ", [" : "[") + std::to_string(st[i]) + ", " + jnum(mx[i]) + ", " + jnum(rms[i]) + "]";
  return o + "]";
}

int run_cpu(const Args& a) {
  CpuSolver s(a.prob, a.check_every, a.threads);
  if (!a.resume.empty()) {
    std::vector<double> prev, cur;
    const int n0 = load_checkpoint(a.resume, a.prob, prev, cur);
    s.set_state(prev.data(), cur.data(), n0);
  }
  CpuResult r;
  double best = 1e30, sum = 0;
  for (int i = 0; i < a.warmup + a.repeat; ++i) {
    r = s.run();
    if (i >= a.warmup) {
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
  std::printf("Total time: %.6f s (init %.6f s, compute %.6f s), threads %d, %.3f GCell/s\n", best, r.init_s,
              r.compute_s, cpu_max_threads(), gcell);
  if (!a.json.empty()) {
    std::ofstream j(a.json);
    j << "{\"backend\": \"cpu\", \"N\": " << a.prob.N << ", \"tau\": " << jnum(a.prob.tau) << ", \"K\": "
      << a.prob.K << ", \"L\": " << jnum(a.prob.L) << ", \"ranks\": 1, \"dims\": [1, 1, 1], \"threads\": "
      << cpu_max_threads() << ", \"solve_s\": " << jnum(best) << ", \"mean_s\": " << jnum(sum / a.repeat)
      << ", \"gcell_per_s\": " << jnum(gcell) << ", \"schedule\": \"cpu-openmp\", \"bench_steps\": " << a.bench_steps
      << ", \"bench_s\": " << jnum(bench_s) << ", \"finite\": " << (r.finite ? "true" : "false") << ", \"steps\": "
      << steps_json(r.steps, r.max_err, r.rms_err) << "}\n";
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
    CpuResult r;
    double best = 1e30, sum = 0, exch = 0;
    for (int i = 0; i < a.warmup + a.repeat; ++i) {
      r = s.run();
      if (i >= a.warmup) {
        if (r.solve_s < best) exch = s.exchange_s();
        best = std::min(best, r.solve_s);
        sum += r.solve_s;
      }
    }
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
      if (!a.json.empty()) {
        std::ofstream j(a.json);
        j << "{\"backend\": \"cpu\", \"ranks\": " << g.world() << ", \"dims\": [" << d.px << ", " << d.py << ", "
          << d.pz << "], \"N\": " << a.prob.N << ", \"tau\": " << a.prob.tau << ", \"K\": " << a.prob.K
          << ", \"L\": " << a.prob.L << ", \"threads\": " << cpu_max_threads() << ", \"solve_s\": " << best
          << ", \"mean_s\": " << sum / a.repeat << ", \"exchange_s\": " << exch << ", \"gcell_per_s\": " << gcell
          << ", \"final_max_err\": " << (r.max_err.empty() ? 0.0 : r.max_err.back())
          << ", \"final_rms_err\": " << (r.rms_err.empty() ? 0.0 : r.rms_err.back())
          << ", \"schedule\": \"cpu-openmp-ranks\", \"bench_steps\": " << a.bench_steps << ", \"bench_s\": "
          << jnum(bench_s) << ", \"finite\": " << (r.finite ? "true" : "false") << ", \"steps\": "
          << steps_json(r.steps, r.max_err, r.rms_err) << "}\n";
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
SolverOptions options_from(const Args& a, bool fake) {
  SolverOptions o;
  o.decomp = a.decomp;
  o.check_every = a.check_every;
  o.overlap = a.overlap;
  o.graph = a.graph;
  o.timers = a.timers;
  o.debug_sync = a.debug_sync;
  o.poison_ghosts = a.poison;
  o.temporal = a.temporal;
  o.tb = a.tb;
  if (a.tb_threads > 0) o.tiling_tb.threads = a.tb_threads;
  if (a.tb_init_threads > 0) o.tiling_tb.init_threads = a.tb_init_threads;
  o.init2 = a.init2;
  o.fake_comm = fake;
  W3D_REQUIRE(a.transport == "rccl" || a.transport == "push" || a.transport == "sdma",
              "--transport must be rccl, push or sdma, not " + a.transport);
  o.push = a.transport == "push";
  o.sdma = a.transport == "sdma";
  o.push_cp_wait = a.push_cp_wait;
  o.push_no_collective = a.no_rccl;  // (no end-of-solve collective: the flag epochs run on, eager launches)
  if (a.t2_rows > 0) o.tiling2.rows = a.t2_rows;
  if (a.deep_min >= 0) o.deep_min_planes = a.deep_min;
  if (a.tb_min >= 0) o.tb_min_planes = a.tb_min;
  if (a.t2_occ >= 0) o.tiling2.occupancy = a.t2_occ;
  if (a.t2_target >= 0) o.tiling2.target_waves = a.t2_target;
  if (a.variant >= 0) o.tiling.variant = a.variant;
  if (a.tile_rows > 0) (o.tiling.variant == 1 ? o.tiling.rows : o.tiling.ty) = a.tile_rows;
  o.tiling.target_blocks = a.target_blocks;
  if (a.nt_store >= 0) o.tiling.nt_store = a.nt_store != 0;
  return o;
}

int run_group(const Args& a, const SolverOptions& o, const hipDeviceProp_t& prop) {
  GpuGroup g(a.prob, o, a.group, a.group_transport);
  if (!a.resume.empty()) {
    std::vector<double> prev, cur;
    const int n0 = load_checkpoint(a.resume, a.prob, prev, cur);
    g.set_state(prev.data(), cur.data(), n0);
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
      << ", \"rccl_comms\": " << cc.size() << ", \"solve_s\": " << jnum(best) << ", \"steps\": [";
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
  const SolverOptions base = options_from(a, fake);
  if (a.group > 0) return run_group(a, base, prop);

  std::shared_ptr<Comm> comm;
  const double t_comm0 = wall_s();
  if (world > 1 && !fake && !a.no_rccl) {
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
  if (const char* fr = std::getenv("W3D_FAULT_RANK"); fr && std::atoi(fr) == rank) fail("injected fault");
  // host collectives: RCCL; files for ranks without a communicator (--no-rccl rehearsal, outside timed regions); none
  // for one rank or a fake rank
  const bool file_coll = !comm && world > 1 && !fake;
  const HostColl hc = comm ? HostColl::rccl(comm) : file_coll ? HostColl::files(rank, world) : HostColl::single(rank);
  W3D_REQUIRE(!a.no_rccl || world == 1 || fake || ((a.transport == "push" || a.transport == "sdma") && !a.autotune),
              "--no-rccl: ranks without a communicator can only run the push or sdma transport (no autotune)");
  std::unique_ptr<GpuSolver> s;
  std::string sched = a.decomp + "-S" + std::to_string(a.temporal) + (a.overlap ? "" : "-seq") +
                      (a.transport == "rccl" ? "" : "-" + a.transport);
  AutotuneResult tuned;
  if (a.autotune && (world > 1 || a.fake_rank < 0)) {
    tuned = autotune(a.prob, base, rank, world, comm, hc, fake, a.transport == "push", a.autotune_rounds);
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
  RunResult r;
  double best = 1e30, sum = 0, first = 0;
  for (int i = 0; i < a.warmup + a.repeat; ++i) {
    hc.barrier();
    r = s->run();
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
    for (int i = 0; i < a.bench_steps; ++i) r = s->run();
    W3D_HIP(hipDeviceSynchronize());
    hc.barrier();
    bench_s = hc.max(wall_s() - t0);
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
  if (file_coll) {  // the last solve's error log over all ranks (L∞: max; RMS: from the per-rank Σe² shares)
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
        << ", \"graph\": " << (s->options().graph ? "true" : "false") << ", \"overlap\": "
        << (s->overlapped() ? "true" : "false") << ", \"overlap_requested\": " << (s->options().overlap ? "true" : "false")
        << ", \"temporal\": " << s->options().temporal
        << ", \"schedule\": " << jstr(sched) << ", \"mode\": " << jstr(s->mode())
        << ", \"transport\": " << jstr(s->transport()) << ", \"device\": "
        << jstr(prop.gcnArchName) << ", \"bench_steps\": " << a.bench_steps << ", \"bench_s\": " << jnum(bench_s)
        << ", \"warmup\": " << a.warmup << ", \"finite\": " << (r.finite ? "true" : "false") << ", \"autotune_s\": {";
      for (size_t i = 0; i < tuned.times.size(); ++i)
        j << (i ? ", " : "") << jstr(tuned.times[i].first) << ": " << jnum(tuned.times[i].second);
      j << "}, \"autotune_rounds\": " << tuned.rounds << ", \"autotune_rejected\": {";
      for (size_t i = 0; i < tuned.rejected.size(); ++i)
        j << (i ? ", " : "") << jstr(tuned.rejected[i].first) << ": " << jstr(json_escape(tuned.rejected[i].second));
      j << "}";
      if (a.timers || a.phases)
        j << ", \"phases_ms\": {\"init\": " << jnum(pp.init_ms) << ", \"compute\": "
          << jnum(pp.interior_ms + pp.shell_ms) << ", \"shell\": " << jnum(pp.shell_ms) << ", \"exchange\": "
          << jnum(pp.comm_ms) << ", \"check\": " << jnum(pp.check_ms) << ", \"gather\": " << jnum(pp.gather_ms)
          << "}";
      j << ", \"steps\": [";
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
