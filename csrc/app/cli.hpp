// wave3d CLI internals shared by its translation units (csrc/app/): the parsed command line, its parser, the
// reference's output lines, the JSON helpers of the summary, and the CPU programs' runners.
#pragma once

#include <functional>
#include <istream>
#include <string>
#include <vector>

#include "wave3d/cpu_dist.hpp"
#include "wave3d/problem.hpp"
#include "wave3d/solver.hpp"

namespace wave3d::cli {

struct Args {
  Problem prob;
  bool have_L = false;
  std::string decomp = "slab";
  int check_every = 2;
  bool cpu = false;
  int threads = 0;
  bool overlap = true;
  bool fused_pack = true;
  bool ghost_store = true;  // --no-ghost-store: slab passes do not store the u^{n+S-1} ghost plane (A/B)
  bool graph = true;
  bool timers = false;
  bool debug_sync = false;
  bool poison = false;
  int temporal = 5;
  bool tb = true;
  int tb_threads = 0;
  int tb_init_threads = 0;
  bool init2 = true;
  int fake_rank = -1, fake_world = 0;
  bool fake_traffic = false;  // --fake-traffic: the fake rank sends / receives its real messages to itself over RCCL
  int reserve_cus = 0;        // --reserve-cus N: CUs kept off the passes for RCCL's kernels
  int capture_selftest = -1;  // --capture-selftest M: the capture guard's probe topology M, then exit (tests)
  int group = 0;                       // --group P: all P ranks in this process on one GPU
  int bench_steps = 0;                 // --bench-steps K: timed block of K solves (bench.py contract)
  bool autotune = false;               // --autotune: time the multi-rank schedule candidates, keep the fastest
  int autotune_rounds = 5;             // --autotune-rounds R: interleaved timing rounds
  int autotune_reps = 5;               // --autotune-reps B: back-to-back solves per candidate and round
  double autotune_budget = 120.0;      // --autotune-budget S: wall-time budget of the autotune (s)
  bool autotune_sdma = false;          // --autotune-sdma (or W3D_AUTOTUNE_SDMA=1): copy-engine candidates too
  bool phases = false;                 // --phases: per-phase breakdown from a traced solve of the timed schedule
  bool serve = false;                  // --serve: keep the solver up, one command per stdin line (Python runtime="process")
  bool verify_repeat = false;          // --verify-repeat: every solve's error log and field hash equal the first's
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

// argv → Args (positional N tau K [L], long options; argv[0] picks the reference program's personality)
Args parse(int argc, char** argv);

// --serve: print `greeting` (one JSON line), then answer one command per stdin line with one JSON line on stdout —
// handle(cmd, rest of the line) returns the reply; "quit" ends the loop (exit 0), an unknown command or a thrown error
// is reported as {"error": ...} (a thrown error also ends the loop, exit 1: the rank's state may be inconsistent).
// The Python side is mpi_cuda_amd/parallel/native_proc.py.
int serve_loop(const std::string& greeting, const std::function<std::string(const std::string&, std::istream&)>& handle);
std::string jexact(double v);  // every digit (%.17g): logs and byte counts compared exactly on the Python side
std::string steps_exact(const std::vector<int>& st, const std::vector<double>& mx, const std::vector<double>& rms);
[[noreturn]] void usage(const char* msg = nullptr);
// the reference's per-step line (report.pdf p.15-16 §4.3): "Step %d, t = %f, Max Error = %e, L2 Error = %e"
void print_errors(const std::vector<int>& steps, const std::vector<double>& mx, const std::vector<double>& rms,
                  double tau);
std::string jstr(const std::string& v);
std::string json_escape(const std::string& v);
std::string jnum(double v);
std::string steps_json(const std::vector<int>& st, const std::vector<double>& mx, const std::vector<double>& rms);
// solver options from the command line
SolverOptions options_from(const Args& a, bool fake);
// the reference's sequential / OpenMP programs (one process) and MPI / MPI+OpenMP programs (one CPU rank)
int run_cpu(const Args& a);
int run_cpu_rank(const Args& a, ShmGroup& g, int rank);

}  // namespace wave3d::cli
