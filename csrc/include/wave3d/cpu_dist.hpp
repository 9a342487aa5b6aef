// Native multi-process CPU solver: the reference's MPI (`mpi`/`onlyMPI`) and MPI+OpenMP (`mpiomp`) programs
// (readme.md:38-48, report.pdf p.12-14 §4.2.2-4.2.3, p.21-26 §5.3-5.4).
//
// One process per rank, each updating its block of the decomposition with the OpenMP kernels of the sequential path,
// ghost layers exchanged every step. There is no MPI on this platform, so the ranks of one node talk through a
// shared-memory segment mapped before the ranks are forked (ShmGroup): per-rank outboxes for the faces, a
// sense-reversing barrier with a timeout (a dead rank turns into an error, not a hang), and per-rank slots for the
// error partials and phase timers, combined in rank order so the printed log does not depend on scheduling.
// `wave3d N tau K [L] --cpu --np P [--threads T] [--decomp D]` ≈ `mpirun -np P ./mpiomp N tau K T`.
#pragma once

#include <atomic>
#include <cstddef>
#include <string>
#include <vector>

#include "wave3d/cpu.hpp"
#include "wave3d/decomp.hpp"

namespace wave3d {

class ShmGroup {
 public:
  // Map the segment (anonymous, MAP_SHARED) in the parent BEFORE forking the ranks; every child inherits it.
  ShmGroup(const Problem& p, const Dims& d, int world);
  // Ranks started by an external launcher (`mpirun -np P ./onlyMPI …`, `torchrun --no-python …`, srun): a named POSIX
  // segment (shm_open), created and initialised by rank 0 and attached by the others once it is marked ready; rank 0
  // unlinks the name when it is done. Fails after `timeout_s` if rank 0 never shows up.
  ShmGroup(const Problem& p, const Dims& d, int world, const std::string& name, int rank, double timeout_s = 120.0);
  ~ShmGroup();
  ShmGroup(const ShmGroup&) = delete;
  ShmGroup& operator=(const ShmGroup&) = delete;

  int world() const { return world_; }
  const Dims& dims() const { return dims_; }
  // All ranks wait here; fails after `timeout_s` (a rank died or hangs) or once any rank has called abort().
  void barrier(double timeout_s = 300.0);
  void abort();  // mark the group failed: every barrier then throws
  // Outbox of `rank`'s face number f of make_halo_plan(layout of rank) (count doubles, written by rank, read by peer).
  double* outbox(int rank, int f) const;
  // Per-rank double slots (error log and timers): slot(rank)[0 .. slot_doubles).
  double* slot(int rank) const;
  size_t slot_doubles() const { return slot_doubles_; }

 private:
  struct Header {
    std::atomic<int> count;
    std::atomic<int> sense;
    std::atomic<int> failed;
    std::atomic<int> ready;  // named segments: set by rank 0 after initialisation
  };
  void layout(const Problem& p);  // face and slot offsets, bytes_
  int world_;
  Dims dims_;
  size_t bytes_ = 0, slot_doubles_ = 0;
  void* base_ = nullptr;
  Header* hdr_ = nullptr;
  std::vector<std::vector<size_t>> face_off_;  // [rank][face] offset in doubles from data()
  size_t slot_off_ = 0;
  double* data() const;
  int local_sense_ = 0;  // per process (each rank is its own process)
  std::string name_;     // named segment (empty: anonymous)
  bool owner_ = false;   // this process unlinks the name
};

// One rank's block, OpenMP inside the rank. run(): init (analytic, ghosts included) → K−1 steps of {exchange the
// current field's faces, leapfrog on the compute box} with error partials on check steps → rank-ordered combine.
class CpuRankSolver {
 public:
  CpuRankSolver(const Problem& p, ShmGroup& g, int rank, int check_every = 2, int threads = 0);
  CpuResult run();  // global errors on every rank; solve/exchange times are the max over ranks
  const Layout& layout() const { return lay_; }
  const std::vector<double>& field(int which) const { return which == 0 ? u_[final_] : u_[1 - final_]; }
  std::vector<int> check_steps() const;
  double exchange_s() const { return exchange_s_; }

 private:
  void exchange(double* u);
  Problem prob_;
  ShmGroup& g_;
  int rank_, check_every_;
  Layout lay_;
  HaloPlan plan_;
  std::vector<int> peer_face_;  // per face: index of the matching face in the peer's halo plan (its outbox)
  std::vector<double> u_[2];
  std::vector<double> s_;
  int final_ = 1;
  double exchange_s_ = 0.0, boundary_s_ = 0.0;
};

}  // namespace wave3d
