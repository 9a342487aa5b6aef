// wave3d CLI: command line, reference program personalities, output helpers. See cli.hpp; reference CLI: report.pdf
// p.12-15 §4.2, p.20-26 §5.
#include <fcntl.h>
#include <unistd.h>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "cli.hpp"

namespace wave3d::cli {


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

[[noreturn]] void usage(const char* msg) {
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
               "  --no-fused-pack    3-D block passes: pack the z faces with the pack kernel too (A/B switch)\n"
               "  --no-ghost-store   slab passes: exchange S-1 planes of u^{n+S-1}, not S-2 plus a stored ghost (A/B)\n"
               "  --no-graph         eager launches instead of one captured hipGraph\n"
               "  --timers           per-phase GPU timers (init / compute / exchange / check)\n"
               "  --no-temporal      one leapfrog step per HBM pass (disable temporal blocking)\n"
               "  --temporal S       at most S (2..5) leapfrog steps per HBM pass (default 5; the push transport: at most 4)\n"
               "  --no-tb            two-step register-queue passes instead of the LDS S-step kernel\n"
               "  --tb-min-planes M  slab ranks: LDS S-step passes with S-deep halos from M owned planes (default 16)\n"
               "  --deep-min-planes M  slab ranks without the LDS kernel: two-step passes from M planes (default 96)\n"
               "  --tb-threads T     LDS S-step kernel workgroup size (768 or 1024; default 1024)\n"
               "  --tb-init-threads T  ... of the analytic-start pass (768 or 1024; default 768)\n"
               "  --no-init2         start from u0,u1 + a first step instead of analytic u1,u2\n"
               "  --debug-sync       synchronize after every step (race triage)\n"
               "  --poison-ghosts    NaN-fill ghost layers before every exchange (missed-halo detector)\n"
               "  --fake-rank R/P    perf study: time rank R of a P-rank decomposition alone on one GPU, no transport\n"
               "  --fake-traffic     with --fake-rank: every exchange sends and receives the rank's exact messages to\n"
               "                     itself over a one-rank RCCL communicator (real RCCL kernels and bytes; values wrong)\n"
               "  --reserve-cus N    keep N CUs (a multiple of 8: N/8 per XCD) off the passes for RCCL's copy kernels\n"
               "  --capture-selftest M  run the stream-capture guard on probe topology M (0 production, 2 the\n"
               "                     round-4 split it refuses) on this runtime, print the result, exit\n"
               "  --group P          all P ranks of the decomposition in this process on one GPU (rehearsal of the\n"
               "                     multi-rank path; --group-transport rccl-self (default: RCCL send/recv, each rank\n"
               "                     over a one-rank communicator), loopback (device copies) or push)\n"
               "  --transport T      rccl (default) | sdma: the copy engines move the halos into the neighbours' memory\n"
               "                     (IPC-mapped, no compute unit used), ordered by flag words | push: slab LDS passes\n"
               "                     store their face planes straight into the neighbours' staging (no exchange phase)\n"
               "  --push-cp-wait     push: wait for the neighbours with hipStreamWaitValue32 (eager) instead of in-kernel\n"
               "  --no-rccl          ranks without an RCCL communicator (push / sdma; IPC handles through files; error\n"
               "                     logs per rank): the multi-process push rehearsal on one shared GPU\n"
               "  --t2-rows R / --t2-target W   fused two-step kernel: rows per wave, x-chunking target (waves)\n"
               "  --repeat R / --warmup W   timed / untimed solves (report min and mean)\n"
               "  --bench-steps K    then K back-to-back solves between two sync+barriers (max over ranks)\n"
               "  --autotune         time the multi-rank schedule candidates (slab / block x pass depth x overlap x RCCL /\n"
               "                     copy engines; push with --transport push) in interleaved rounds, keep the fastest\n"
               "                     (slowest rank decides; the simplest within 2%%)\n"
               "  --autotune-rounds R  interleaved timing rounds of the autotune (default 5); the median decides\n"
               "  --autotune-reps B  back-to-back solves per candidate and round (default 5, as the bench runs them)\n"
               "  --autotune-budget S  wall-time budget of the autotune in seconds (default 120; 0: none)\n"
               "  --autotune-sdma    include the copy-engine candidates across GPUs (also W3D_AUTOTUNE_SDMA=1)\n"
               "  --phases           per-phase device times (init/compute/exchange/check) of the timed schedule\n"
               "  --serve            keep the solver up: run / hash W / traffic / dump P / quit, one per stdin line,\n"
               "                     one JSON reply line each (the Python Solver(runtime=\"process\") rank process)\n"
               "  --verify-repeat    every solve (warmup included) must reproduce the first one's error log and u^K\n"
               "                     field hash on this rank bit for bit (exit 4 otherwise): halo-visibility stress\n"
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
    else if (s == "--no-fused-pack") a.fused_pack = false;
    else if (s == "--no-ghost-store") a.ghost_store = false;
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
    else if (s == "--fake-traffic") a.fake_traffic = true;
    else if (s == "--reserve-cus") a.reserve_cus = std::stoi(next());
    else if (s == "--capture-selftest") a.capture_selftest = std::stoi(next());
    else if (s == "--group") a.group = std::stoi(next());
    else if (s == "--bench-steps") a.bench_steps = std::stoi(next());
    else if (s == "--autotune") a.autotune = true;
    else if (s == "--autotune-rounds") a.autotune_rounds = std::stoi(next());
    else if (s == "--autotune-reps") a.autotune_reps = std::stoi(next());
    else if (s == "--autotune-budget") a.autotune_budget = std::stod(next());
    else if (s == "--autotune-sdma") a.autotune_sdma = true;
    else if (s == "--phases") a.phases = true;
    else if (s == "--verify-repeat") a.verify_repeat = true;
    else if (s == "--serve") a.serve = true;
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

std::string jexact(double v) {
  char b[40];
  std::snprintf(b, sizeof b, "%.17g", v);
  return b;
}
std::string steps_exact(const std::vector<int>& st, const std::vector<double>& mx, const std::vector<double>& rms) {
  std::string o = "[";
  for (size_t i = 0; i < st.size(); ++i)
    o += (i ? ", [" : "[") + std::to_string(st[i]) + ", " + jexact(mx[i]) + ", " + jexact(rms[i]) + "]";
  return o + "]";
}

int serve_loop(const std::string& greeting,
               const std::function<std::string(const std::string&, std::istream&)>& handle) {
  // Private descriptors for the protocol: the commands keep arriving on what was fd 0 and the replies leave on what
  // was fd 1, while fd 0 becomes /dev/null and fd 1 the stderr stream. Measured: a process with RCCL communicators lost
  // the commands queued in its stdin during a graph capture (rccl-self group), and RCCL prints its banner to stdout.
  std::fflush(stdout);
  const int in_fd = dup(0), out_fd = dup(1);
  W3D_REQUIRE(in_fd >= 0 && out_fd >= 0, "serve: cannot duplicate stdin / stdout");
  const int nul = open("/dev/null", O_RDONLY);
  if (nul >= 0) {
    dup2(nul, 0);
    close(nul);
  }
  dup2(2, 1);
  FILE* cmd_in = fdopen(in_fd, "r");
  FILE* rep_out = fdopen(out_fd, "w");
  W3D_REQUIRE(cmd_in && rep_out, "serve: cannot open the protocol streams");
  auto reply = [&](const std::string& line) {
    std::fputs(line.c_str(), rep_out);
    std::fputc('\n', rep_out);
    std::fflush(rep_out);
  };
  reply(greeting);
  char* buf = nullptr;
  size_t cap = 0;
  int rc = 0;
  for (;;) {
    const ssize_t n = getline(&buf, &cap, cmd_in);
    if (n < 0) break;  // (stdin closed: the parent is gone)
    std::istringstream in(std::string(buf, static_cast<size_t>(n)));
    std::string cmd;
    in >> cmd;
    if (cmd.empty()) continue;
    if (cmd == "quit") {
      reply("{\"bye\": true}");
      break;
    }
    try {
      reply(handle(cmd, in));
    } catch (const std::exception& e) {
      reply("{\"error\": " + jstr(json_escape(e.what())) + "}");
      rc = 1;  // (a failed collective leaves the peers to their own timeouts: this rank is gone)
      break;
    }
  }
  std::free(buf);
  std::fclose(cmd_in);
  std::fclose(rep_out);
  return rc;
}

SolverOptions options_from(const Args& a, bool fake) {
  SolverOptions o;
  o.decomp = a.decomp;
  o.check_every = a.check_every;
  o.overlap = a.overlap;
  o.fused_pack = a.fused_pack;
  o.ghost_store = a.ghost_store;
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
  o.fake_traffic = fake && a.fake_traffic;
  o.reserve_cus = a.reserve_cus;
  W3D_REQUIRE(a.transport == "rccl" || a.transport == "push" || a.transport == "sdma",
              "--transport must be rccl, push or sdma, not " + a.transport);
  o.push = a.transport == "push";
  o.sdma = a.transport == "sdma";
  if (const char* sh = std::getenv("W3D_SHELLS")) o.shells_concurrent = std::string(sh) == "concurrent";
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

}  // namespace wave3d::cli
