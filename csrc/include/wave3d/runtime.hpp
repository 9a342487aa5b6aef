// Native job runtime around the solvers (everything the reference's `mpirun -np P ./mpigpu-1 N tau K 1` gets from MPI
// and its shell scripts, report.pdf p.15 §4.2.4): rank discovery and the --np self-spawn, the RCCL
// unique-id rendezvous, host collectives (RCCL, files, or none), field dumps / checkpoints (wave3d-dump-v1, SURVEY.md
// §5.9) and the multi-rank schedule autotune. Shared by the CLI (csrc/app/wave3d_main.cpp) and the Python bindings, so
// both entry points run the same autotune.
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "wave3d/solver.hpp"

namespace wave3d {

// ---- launch (runtime_launch.cpp) ------------------------------------------------------------------------------
// Rank / world / local-rank environment of the launchers we accept: torchrun, Open MPI, MPICH hydra (PMI), Slurm.
extern const char* const kRankEnv[];
extern const char* const kSizeEnv[];
extern const char* const kLocalEnv[];
int env_int(const char* const* names, int dflt);
double wall_s();  // steady clock, seconds
// Name of the shared segment of the CPU ranks of one launcher job (W3D_JOB_ID, the launcher's job id, MASTER_PORT, or
// the parent pid).
std::string job_segment_name();
// Rendezvous file of the RCCL unique id (W3D_RDZV_FILE, else one derived from the launcher) and the exchange itself:
// rank 0 publishes a fresh id atomically, the others wait for a file written after they started.
std::string rdzv_path();
std::string exchange_unique_id(int rank);
// Every rank's bytes (equal sizes) through files next to the rendezvous file, in rank order.
// timeout_s: 0 = W3D_FILE_TIMEOUT_S (default 120 s), < 0 = as long as the parent process lives
std::vector<std::string> file_allgather(int rank, int world, const std::string& mine, const std::string& tag,
                                        double timeout_s = 0.0);
double proc_timeout_s();
// Fork P ranks before anything touches the GPU (RANK / LOCAL_RANK / WORLD_SIZE / W3D_RDZV_FILE in their env). Returns
// -1 in a child (continue as that rank), the first non-zero exit status of the children in the parent.
int spawn_ranks(int np);

// ---- host collectives -------------------------------------------------------------------------------------------
// What the runtime modules need from the job: agreement on a flag (every rank must take the same branch), max over
// ranks, barrier, and an all-gather of equal-size byte strings. Blocking, outside timed regions.
struct HostColl {
  int rank = 0, world = 1;
  std::function<bool(bool)> agree;
  std::function<double(double)> max;
  std::function<void()> barrier;
  std::function<void()> idle_barrier;  // (optional) a barrier between requests of the serve loop: no fixed bound
  std::function<std::vector<std::string>(const std::string&)> allgather;
  std::function<void()> cleanup;  // files of a file-based collective (the last one stays: a peer may still read it)
  static HostColl single(int rank = 0);                         // one rank (or a fake rank): identity collectives
  static HostColl rccl(std::shared_ptr<Comm> c);                // over the RCCL communicator
  static HostColl files(int rank, int world);                   // through files next to the rendezvous file
};

// ---- field dumps / checkpoints (runtime_io.cpp) -------------------------------------------------------------------
// PREFIX[.rankR].bin (raw little-endian fp64, C order [x][y][z], owned nodes) + .json sidecar (wave3d-dump-v1).
void write_dump(const std::string& prefix, const Problem& p, const Layout& l, const std::vector<double>& u, int rank,
                int world, const Dims& d, int step = -1);
// u^K → PREFIX.cur, u^{K−1} → PREFIX.prev
void write_checkpoint(const std::string& prefix, const Problem& p, const Layout& l, const std::vector<double>& cur,
                      const std::vector<double>& prev, int rank, int world, const Dims& d);
// numbers after "key": in a one-line JSON object (the sidecars above)
std::vector<double> json_numbers(const std::string& text, const std::string& key);
// the GLOBAL (N+1)³ field of a dump of any decomposition; checks N, tau and L against `p`; returns its step
int load_dump_global(const std::string& prefix, const Problem& p, std::vector<double>& g);
// PREFIX.prev / PREFIX.cur → u^{n0−1}, u^{n0}; returns n0
int load_checkpoint(const std::string& prefix, const Problem& p, std::vector<double>& prev, std::vector<double>& cur);

// ---- multi-rank schedule autotune (runtime_autotune.cpp) ----------------------------------------------------------
// One candidate: decomposition × pass depth × overlap × halo transport. The list is in order of
// simplicity; a later candidate must beat every earlier one by more than the tie margin to be chosen.
struct Candidate {
  std::string name, decomp, transport;  // transport: rccl | sdma | push
  int temporal = 5;
  bool overlap = true;
  int sdma_streams = 0;            // copy streams (0: the solver's default)
  bool shells_concurrent = false;  // overlap: shells beside the interior instead of before it
  int reserve_cus = 0;             // CUs kept off the passes for RCCL's kernels (SolverOptions::reserve_cus)
};
// the candidates for `world` ranks (fake: one rank of a `world`-rank job alone); push and copy-engine candidates only on
// request (neither has run between two GPUs yet)
std::vector<Candidate> autotune_candidates(int world, bool with_push, bool with_sdma = false);
// connect a solver's transport to its peers (IPC handles through hc.allgather; a fake rank connects to itself)
void connect_transport(GpuSolver& s, const HostColl& hc, bool fake);
struct AutotuneResult {
  std::unique_ptr<GpuSolver> solver;
  std::string name;
  std::vector<std::pair<std::string, double>> times;       // per timed candidate: median per-solve time (max over ranks)
  std::vector<std::pair<std::string, double>> best_times;  // ... and its best round
  std::vector<std::pair<std::string, std::string>> rejected;  // candidate, reason
  int rounds = 0, reps = 0;
  double wall_s = 0.0;  // the autotune's own wall time
};
struct AutotuneOptions {
  bool with_push = false;   // the push transport's candidates (opt-in)
  bool with_sdma = false;   // the copy-engine candidates (opt-in across devices; a fake rank always has them)
  int rounds = 5;           // interleaved timing rounds
  int reps = 5;             // back-to-back solves per candidate and round (the bench's pattern)
  double tie = 0.02;        // a later candidate must beat the simplest by more than this (relative) to be chosen
  double budget_s = 120.0;  // wall-time budget: no new candidate, and no new round, once spent (<= 0: none)
  double flag_timeout_s = 10.0;  // in-kernel flag-wait bound of the candidates (copy engines; <= 0: the default)
};
// Build every candidate on every rank (a candidate one rank cannot build is skipped everywhere), drop clones (same
// mode, transport, overlap, depth and decomposition as an earlier one), run each twice (eager + capture), reject any
// whose log or fields differ from the first accepted candidate's (L∞ exact, RMS to 1e-12, u^K and u^{K−1} through the
// decomposition-free field hash — every schedule computes bit-identical fields), then time the survivors in `rounds`
// interleaved rounds of `reps` back-to-back solves each (barrier before each round) and keep the fastest MEDIAN — or
// the simplest within `tie` of it. The slowest rank decides every time. Candidates that do not fit in device memory
// next to the others are timed alone right away. The wall-time budget stops the candidate list and the rounds early.
AutotuneResult autotune(const Problem& prob, const SolverOptions& base, int rank, int world, std::shared_ptr<Comm> comm,
                        const HostColl& hc, bool fake, const AutotuneOptions& opt);

}  // namespace wave3d
