// GPU solver runtime: one process (rank) per MI355X, RCCL point-to-point halo exchange over xGMI.
//
// Reference call stack being replaced (report.pdf p.15-16 §4.2.4-4.4): MPI_Init → cudaSetDevice →
// host init + H2D → per step {D2H faces → MPI_Sendrecv → H2D; step kernel; BC kernel; error kernel + MPI_Reduce}.
// Here:
//   * fields are initialised on the device (no H2D), both in-place leapfrog levels live in HBM;
//   * per step the boundary SHELL of the local box is updated first, then its faces go to the neighbours with
//     ncclSend/ncclRecv on a side stream while the INTERIOR update runs on the compute stream;
//   * error partials stay on the device; the whole error log crosses to the host once, with one all-gather;
//   * the full K-step solve can be captured into one hipGraph and replayed.
#pragma once

#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstdio>
#include <memory>
#include <string>
#include <vector>

#include "wave3d/decomp.hpp"
#include "wave3d/kernels.hpp"
#include "wave3d/problem.hpp"

namespace wave3d {

#define W3D_HIP(expr)                                                                                \
  do {                                                                                               \
    hipError_t _e = (expr);                                                                          \
    if (_e != hipSuccess) ::wave3d::fail(std::string(#expr) + ": " + hipGetErrorString(_e));          \
  } while (0)

struct SolverOptions {
  std::string decomp = "slab";  // slab | block | PxQxR
  int check_every = 2;          // error check cadence (reference prints every 2nd step); 0 = only the last step
  bool overlap = true;          // shell/interior split with the halo exchange on a side stream
  bool graph = true;            // capture the whole solve into a hipGraph, replay it on every run()
  bool timers = false;          // per-phase hipEvent timers (adds events to the stream; disables the graph)
  bool debug_sync = false;      // hipDeviceSynchronize after every step (race triage; disables the graph)
  bool poison_ghosts = false;   // NaN-fill ghost layers before each exchange (a missed halo poisons the errors)
  bool fake_comm = false;       // perf study only: run rank `rank` of `world` alone, exchanges replaced by no-ops
  bool fake_traffic = false;    // ... unless set: the exact message set goes to itself over a one-rank communicator
                                // (RCCL copy kernels and bytes next to the passes; the received values are its own)
  LeapfrogTiling tiling;
  // Temporal blocking: up to `temporal` (2..5) steps per HBM pass wherever no halo exchange intervenes. One rank:
  // k_leapfrog_p2 passes (pair-tiled, S ≤ 5; all levels in LDS, error checks at any level), the steps split into
  // passes by measured per-step cost; slab and 3-D block ranks: the same passes with `temporal`-deep ghosts, one
  // exchange per pass (the push transport: k_leapfrog_tb, S ≤ 4; tb = false: two-step k_leapfrog2 passes with 2-deep
  // halos). 1 = one step per pass everywhere.
  int temporal = 5;
  bool tb = true;  // one rank: LDS kernel (false: k_leapfrog2 pairs, only where the intermediate step has no check)
  Leapfrog2Tiling tiling2;
  LeapfrogTbTiling tiling_tb;
  // Start from u¹, u² computed analytically in one write-only pass (k_init_two) instead of u⁰, u¹ + a first step.
  bool init2 = true;
  // Slab ranks use the deep-halo fused schedule only from this many owned x-planes up (below, single steps are faster).
  int deep_min_planes = 96;
  // Slab ranks use the LDS multi-step passes (deep-tb) when every rank owns at least this many x-planes (and at least
  // 2·temporal: each pass first computes the `steps` planes next to each neighbour, the shells that are sent).
  int tb_min_planes = 16;
  // Slab LDS passes (deep-tb) only: the "push" halo transport. Each pass stores the face planes its neighbours read as
  // ghosts a second time, straight into their fine-grained staging over xGMI (TbPush, kernels.hpp): no exchange phase,
  // no RCCL kernels competing for CUs, no shell launches; with `overlap` the pass produces both face regions first so
  // the remote stores drain while it marches on. Cross-rank order: flags in uncached memory, raised at the end of a
  // pass and waited for at the start of the next one (in the kernel; push_cp_wait: by the command processor with
  // hipStreamWaitValue32 — eager launches only, for ranks that share one GPU). Peers are connected with
  // connect_push() (multi-process: IPC handles) or by a GpuGroup.
  bool push = false;
  // Copy-engine ("sdma") transport (deep-tb slab and block ranks): the halo regions are copied into the neighbours'
  // memory (IPC-mapped: their field buffers' ghost planes for slabs, their staging buffers for blocks) by
  // hipMemcpyAsync(..., hipMemcpyDeviceToDeviceNoCU) on copy streams — the SDMA engines move them, no compute unit is
  // taken from the LDS passes — and cross-rank order is kept by flag words in uncached device memory (waits: one-
  // workgroup kernels; "arrived": a 4-byte copy-engine write behind the data). See transport_sdma.cpp for the protocol.
  bool sdma = false;
  // 3-D block LDS passes: the pass stores the z-face message parts of the next exchange straight into the send staging
  // (TbPack, kernels.hpp); the pack kernel then copies only the x / y faces, edges and corners (A/B: --no-fused-pack)
  bool fused_pack = true;
  // slab LDS passes (deep-tb, pair-tiled kernel; RCCL / loopback / copy-engine transports): each pass also stores the
  // u^{n+S−1} plane next to each neighbour face (it computes it anyway), so the exchange sends S planes of u^{n+S} and
  // S − 2 (not S − 1) of u^{n+S−1} per face — 8 instead of 9 planes for a 5-step pass (A/B: --no-ghost-store)
  bool ghost_store = true;
  // deep-tb with overlap: the shell boxes run on the side stream concurrently with the interior (true), or on s0 before
  // it (false: they get the whole GPU and finish first, so the exchange starts earlier — measured faster with the copy
  // engines at 512³ and 2048³; concurrent helps the small block shells when no transfer follows; env W3D_SHELLS)
  bool shells_concurrent = false;
  // CUs kept free of the passes for RCCL's copy kernels (0: none). The compute stream gets a CU mask without the top
  // `reserve_cus` CUs (KFD deals mask bits to the XCDs round-robin, so a multiple of 8 frees the same number of CUs in
  // every XCD); a pass occupies a whole CU (LDS, VGPRs), so without a reserve RCCL's kernels of an overlapped exchange
  // wait for the pass's last workgroups. The passes' x chunking then targets the remaining CUs. Env W3D_RESERVE_CUS.
  int reserve_cus = 0;
  // copy-engine transport: copy streams (each gets its own SDMA engine; 0 = auto: one per slab face, one for a block
  // rank's messages — in a replayed graph a second copy stream made the 2048³ 2x2x2 rank slower, 48.8 vs 43.6 ms)
  int sdma_streams = 0;
  // copy-engine transport: bound of one in-kernel flag wait in seconds (0 = min(W3D_TIMEOUT_S / 2, 60)); the autotune
  // sets a short one so a candidate whose peer is lost costs seconds, not minutes. It is baked into the captured
  // graphs. Half the host's own wait bound by default, so the device reports the lost peer before the host gives up.
  double flag_timeout_s = 0.0;
  bool push_cp_wait = false;
  // push ranks without an end-of-solve collective (no RCCL communicator): the flag epochs run on over the solves
  // instead of being reset (eager launches: every launch carries its own epochs)
  bool push_no_collective = false;
};

// Summed device time per phase of the last run() (SolverOptions::timers). compute = interior / whole-box / fused
// passes; comm overlaps compute when the exchange runs on the side stream; gather is host wall time.
struct PhaseTimes {
  double init_ms = 0, shell_ms = 0, interior_ms = 0, comm_ms = 0, check_ms = 0, gather_ms = 0;
};

// Device time of one schedule unit (SolverOptions::timers; --trace): shell = the boundary part computed first,
// comm = its exchange (side stream, overlapping compute), compute = the rest, check = error reductions.
struct UnitTrace {
  int unit = 0, n = 0, steps = 0;
  double shell_ms = 0, comm_ms = 0, compute_ms = 0, check_ms = 0;
};

struct RunResult {
  std::vector<int> steps;         // checked steps
  std::vector<double> max_err;    // L∞ (global)
  std::vector<double> rms_err;    // sqrt(Σe² / (N−1)³) (global)
  double solve_s = 0.0;           // host wall time of run(): field init → last error gathered
  PhaseTimes phases;              // only with SolverOptions::timers
  std::vector<UnitTrace> trace;   // per unit, only with SolverOptions::timers
  bool finite = true;
  bool batched = false;           // run_batch's pipelined path: solve_s is the batch's wall time / n
};

// Thin owner of an RCCL communicator.
class Comm {
 public:
  // 128-byte ncclUniqueId as raw bytes (call on rank 0, ship to the others).
  static std::string make_unique_id();
  Comm(int rank, int world, const std::string& unique_id);
  // every visible device's rank of one communicator, created in this process (ncclCommInitAll over devices
  // 0..world−1): the single-process multi-GPU mode
  static std::vector<std::shared_ptr<Comm>> init_all(int world);
  ~Comm();
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;
  int rank() const { return rank_; }
  int world() const { return world_; }
  // ranks of the communicator as RCCL itself reports them (ncclCommCount): proof of what RCCL saw
  int count() const;
  // device the communicator is bound to (ncclCommCuDevice)
  int device() const;
  void* raw() const { return comm_; }  // ncclComm_t
  // Raise if RCCL reported an asynchronous error.
  void check_async() const;

 private:
  Comm() = default;
  int rank_ = 0, world_ = 1;
  void* comm_ = nullptr;
};

class GpuSolver {
 public:
  // loopback = true: this rank is driven by a GpuGroup (in-process ranks, device-copy halos; tests)
  GpuSolver(const Problem& prob, const SolverOptions& opt, int rank, int world, std::shared_ptr<Comm> comm,
            bool loopback = false);
  ~GpuSolver();
  GpuSolver(const GpuSolver&) = delete;
  GpuSolver& operator=(const GpuSolver&) = delete;

  // One full solve: u⁰, u¹ → K−1 leapfrog steps with error checks → global error log on the host.
  RunResult run();
  // n solves back to back (bench.py's timed block): a one-rank solver with a captured graph enqueues all n replays,
  // each followed by the copy of its own error log into its slot of a pinned host buffer, and synchronises once at
  // the end; the CLI then checks every timed solve's log against the warmup solve's. Every solve runs in full. (The
  // host round trip it removes between solves measured within noise of 0 at 512³: profiles/r4/vmcnt/README.md.)
  // Other solvers (several ranks, copy engines, push, timers, resume, no graph) call run() n times. solve_s: on the
  // pipelined path the batch's wall time / n (RunResult::batched = true), otherwise each run()'s own time.
  std::vector<RunResult> run_batch(int n);
  // Per-phase event timers for the following run() calls (those launch eagerly; the captured graph is kept for when
  // the timers are switched off again): a phase breakdown of exactly the schedule the graph replays.
  void set_timers(bool on) { opt_.timers = on; }
  // Loaded-field start (resume): every following run() starts at step n0 from u^{n0−1} = prev and
  // u^{n0} = cur (GLOBAL (N+1)³ C-order fields; each rank takes its box and all its ghost layers from them, so the
  // first pass needs no exchange) and continues the same schedule kinds to K, checking the steps after n0. The
  // state is uploaded at the start of each run (eager launches, no graph).
  void set_state(const double* prev_global, const double* cur_global, int n0);

  // Host copy of the local array holding u^K (which = 0) or u^{K−1} (which = 1), full padded layout.
  std::vector<double> download(int which) const;
  // Order-independent 64-bit hash of the OWNED nodes of u^K (which = 0) or u^{K−1} (which = 1) after the last run():
  // Σ mix(bits(u) ^ mix(global node index)) mod 2⁶⁴. Summed over the ranks (mod 2⁶⁴) it is the same for every
  // decomposition and schedule that computes bit-identical fields — the autotune's field check (one read pass).
  unsigned long long field_hash(int which) const;
  int device() const { return dev_; }  // the HIP device this rank's buffers and streams live on

  const Layout& layout() const { return lay_; }
  const Dims& dims() const { return dims_; }
  const HaloPlan& halo() const { return plan_; }
  const Problem& problem() const { return prob_; }
  const SolverOptions& options() const { return opt_; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  std::vector<LBox> shell_boxes() const { return shell_; }
  LBox interior_box() const { return interior_; }
  std::vector<int> check_steps() const;
  size_t device_bytes() const;
  // "single-step" | "fused-single" (temporal blocking, one rank) | "deep-tb" (LDS multi-step passes, slab ranks)
  // | "deep-halo" (two-step passes, slab ranks)
  std::string mode() const;
  // push transport: this rank's staging + flag IPC handles (opaque bytes), and connecting to the neighbours from
  // every rank's handles (index = rank); GpuGroup ranks are connected in-process instead
  bool push() const { return push_; }
  std::string push_handles() const;
  void connect_push(const std::vector<std::string>& all);
  void connect_push_self();  // perf study (fake rank): forward into the own staging, wait for the own signals
  // copy-engine transport: this rank's IPC handles (field buffers, staging, flags) + layout facts, and connecting to
  // every neighbour from all ranks' handles (index = rank); a fake rank connects to itself
  bool sdma() const { return sdma_; }
  int copy_streams() const { return static_cast<int>(xcs_.size()); }
  std::string sdma_handles() const;
  void connect_sdma(const std::vector<std::string>& all);
  void connect_sdma_self();
  // the halo overlap that actually runs: the exchange is issued on the side stream while the pass's interior runs
  // (push: the passes produce their face planes first); false for schedules that exchange after the whole pass,
  // whatever options().overlap says
  bool overlapped() const {
    if (!plan_.any() || world_ == 1) return false;
    return push_ ? opt_.overlap : xstream() != s0_;
  }
  // halo transport actually in use: "none" (one rank), "rccl", "push", "sdma", "fake" (perf study, no transport)
  std::string transport() const;
  // Bytes one solve moves, from the unit schedule (SURVEY.md §5.5 effective GB/s). field_bytes: the compulsory
  // device-memory traffic over the nodes this rank updates — a fused pass reads u^n, u^{n−1} and writes two levels,
  // an analytic-start pass only writes its two, a single step reads two and writes one, the init kernel writes two;
  // tile-halo re-reads that miss L2 are not in it (rocprof FETCH_SIZE counts those). halo_bytes: what this rank sends
  // its neighbours per solve (RCCL / copy-engine messages, or the push transport's forwarded face planes).
  struct Traffic {
    double field_bytes = 0.0, halo_bytes = 0.0;
  };
  Traffic traffic();

 private:
  friend class GpuGroup;
  void enqueue_solve();  // all device work of one solve on s0/s1 (graph-capturable)
  // One halo exchange on stream st: pack → ncclGroup{ncclSend/ncclRecv per message} → unpack. `pull` != null: this
  // rank belongs to an in-process group driven over a one-rank communicator (GpuGroup "rccl-self"); every message is
  // then moved by a self send/recv pair on THIS rank's communicator, sending the peer's matching face (already packed
  // by the peer) into this rank's receive region — the same RCCL calls, stream and events as the multi-process path.
  void exchange(hipStream_t st, const std::vector<GpuSolver*>* pull = nullptr);
  bool packs() const;               // this schedule's messages go through the staging buffers
  void pack_halo(hipStream_t st);   // faces (single steps) / S-deep regions (block passes) → send_buf_
  void unpack_halo(hipStream_t st); // recv_buf_ → ghost layers
  void gather_errors(RunResult& r);
  void decode_log(const Partial* host, int nsrc, RunResult& r) const;  // per-rank partials → r's log (rank order)
  // Schedule: a solve is phase_init() followed by units; a unit advances one step (in place over u^{n−1}) or 2..4
  // (a fused pass into the two free buffers). Multi-rank units run shell -> exchange -> interior.
  enum class Mode { kSingleStep, kFusedSingle, kDeep, kDeepTb };
  struct Unit {
    int n;      // current level u^n before the unit
    int steps;  // 1: in-place single step; >= 2: one fused pass writing u^{n+steps−1}, u^{n+steps}
    bool analytic = false;  // LDS pass from n = 1 computing u⁰, u¹ in the kernel (no init kernel, no reads)
    bool fused() const { return steps >= 2; }
  };
  // one point-to-point message of an exchange: `tag` pairs it with the peer's matching message
  struct Msg {
    int peer, tag;
    const double* send;
    double* recv;
    i64 count;
  };
  const Msg& peer_msg(const Msg& m, const std::vector<GpuSolver*>& ranks) const;
  bool split() const;
  bool post_exchange() const;  // the unit's NEW field is exchanged after its shell (else: current field, before)
  // deep-tb without overlap: no shell launches; each pass runs whole and its faces are exchanged after it (on s0)
  bool late_exchange() const;
  bool needs_exchange(int i) const;
  int ghost_bits(int i) const;  // x sides whose u^{n+S−1} ghost plane unit i's passes store (SolverOptions::ghost_store)
  hipStream_t xstream() const;
  bool pairable() const;
  bool analytic_ok() const;  // the first unit can be an analytic-start LDS pass
  void build_units();
  void build_msgs(int i);
  void phase_init();
  void unit_shell(int i);
  void unit_exchange_rccl(int i);
  void unit_interior(int i);
  void tb_pass(const Unit& u, const LBox& box, int phase, hipStream_t st = nullptr);  // one k_leapfrog_tb launch
  // the unit's shell boxes in ONE pair-tiled launch when that applies (returns false: launch them one by one)
  bool tb_pass_boxes(const Unit& u, const std::vector<LBox>& boxes, int phase, hipStream_t st);
  // deep-tb with overlap: unit i's shell boxes (what the neighbours receive, computed first) and the interior box
  void tb_split(int i, std::vector<LBox>& shells, LBox& interior) const;
  std::vector<LBox> tb_shells(int i) const;
  LBox tb_interior(int i) const;
  // in-process group steps (GpuGroup): pack own faces → (group barrier) → pull peers' faces → (group barrier)
  void lb_pack(int i);
  void lb_pull(int i, const std::vector<GpuSolver*>& ranks, hipEvent_t all_packed);
  void lb_fence(int i, hipEvent_t all_pulled);

  Problem prob_;
  SolverOptions opt_;
  Coeffs coef_;
  int dev_ = 0;
  int rank_, world_;
  std::shared_ptr<Comm> comm_;
  bool loopback_ = false;
  Dims dims_;
  Layout lay_;
  HaloPlan plan_;
  std::vector<LBox> shell_;
  LBox interior_;
  LBox full_;

  double* u_[4] = {nullptr, nullptr, nullptr, nullptr};  // [2], [3] only with temporal blocking
  int nbuf_ = 2;
  Mode mode_ = Mode::kSingleStep;
  std::vector<Unit> units_;
  std::vector<Msg> msgs_;
  int uf_[2] = {2, 3};            // output buffers of the current fused unit
  std::vector<LBox> dshell_;      // deep mode: output x-slabs next to neighbours (shell) ...
  LBox dint_;                     // ... and the rest (interior)
  i64 sx0_ = 0, sx1_ = 0;         // deep mode: stage-1 x range (one ghost plane beyond each neighbour face)
  LBox sreal_;                    // deep-tb: stage-real ranges per axis (temporal − 1 nodes into each neighbour's ghosts)
  bool block_tb_ = false;         // deep-tb on a 3-D block decomposition (S-deep ghosts on every split axis)
  DeepPlan deep_[6];              // block_tb_: exchange plan before a pass of s steps (index s = 2..temporal)
  BoxCopyTable pack_tab_[6], unpack_tab_[6];  // ... and its device job tables (send / receive regions)
  TbPack pk_host_[6];                          // fused z-face pack per exchange depth (fused_pack; w = 0: none)
  TbPack* pk_dev_ = nullptr;                   // ... the same five entries in device memory
  i64 deep_max_ = 0;              // largest staging buffer of those plans (doubles): the receive staging
  i64 sbase_[6] = {};             // send staging: the region of depth s starts at sbase_[s] (one region per depth)
  i64 send_total_ = 0;            // ... and its size (doubles)
  int deep_s_ = 2;                // depth of the exchange being issued
  std::vector<int> n_dshell_;     // partials per deep shell launch
  int n_dint_ = 0;
  int prev_buf_ = 1;             // buffer index holding u^{K−1} after a solve
  double* d_s_ = nullptr;        // extended sin table (+1 applied when passed to kernels)
  double* send_buf_ = nullptr;   // packed y/z faces
  double* recv_buf_ = nullptr;
  Partial* partials_ = nullptr;
  int n_partials_ = 0;
  Partial* errlog_ = nullptr;    // [K+1]
  Partial* errall_ = nullptr;    // [world][K+1]
  Partial* hbatch_ = nullptr;    // pinned [batch][K+1] (run_batch)
  int hbatch_n_ = 0;
  std::vector<double> ct_;       // cos(a_t n τ)
  hipStream_t s0_ = nullptr, s1_ = nullptr;
  bool own_s0_ = true;  // false: a GpuGroup "push" rank on the group's shared compute stream
  hipEvent_t ev_shell_ = nullptr, ev_halo_ = nullptr, ev_packed_ = nullptr;
  int n_full_ = 0, n_shell_ = 0, n_int_ = 0, n_fused_ = 0;  // error partials of each launch kind
  int n_tb_ = 0;                                            // ... per level of a k_leapfrog_tb pass
  // deep-tb: per level, the partials of this unit's launches (shell lo, shell hi, interior) follow each other
  int tb_slots_ = 0;                                        // launches of the current unit with partials so far
  // LDS passes: each unit's partials go to region tb_region_ of kTbRegions; their reductions are queued and issued as
  // one batched launch when the regions wrap and at the end of the solve (one launch instead of one per checked step)
  static constexpr int kTbRegions = 8;
  static constexpr int kTbSlots = 8;  // launches with partials per level and unit (shell boxes + interior)
  static constexpr int kTbLevels = 5; // levels per pass (5-step passes: k_leapfrog_p2)
  Partial* tb_partials_ = nullptr;
  int tb_region_ = 0;
  std::vector<ReduceJob> pending_;
  void flush_reduces();
  bool nb_lo_ = false, nb_hi_ = false;                      // x neighbours (slab ranks)
  int cur_ = 1, old_ = 0;                     // buffer roles during enqueue
  int start_n_ = 1;                           // first leapfrog step after the init kernel
  bool analytic_ = false;                     // the first unit computes u⁰, u¹ itself (no init kernel)
  std::vector<char> is_check_;
  int resume_n_ = 0;                  // > 0: runs start at this step from resume_[0..1]
  std::vector<double> resume_[2];     // local (padded) u^{n0−1}, u^{n0}
  hipGraphExec_t graph_exec_ = nullptr;
  int runs_ = 0;  // completed run() calls (RCCL ranks capture the graph only after one eager solve)
  int final_buf_ = 0;            // buffer index holding u^K after a solve
  // per-phase timers
  enum { kPhaseInit = 0, kPhaseShell, kPhaseCompute, kPhaseComm, kPhaseCheck, kPhaseGather, kNumPhases };
  struct Mark {
    int phase, unit;  // unit −1: init
    hipEvent_t b, e;
  };
  int cur_unit_ = -1;
  std::vector<hipEvent_t> ev_pool_;
  size_t ev_next_ = 0;
  std::vector<Mark> marks_;
  template <class F>
  void timed(int phase, hipStream_t st, F&& f);
  void collect_phases(RunResult& r);
  void poison(hipStream_t st);
  // push transport (slab deep-tb)
  bool push_ = false;
  double* stg_ = nullptr;       // [parity][field (0: u^{n+S−1}, 1: u^{n+S})][side (0: lo ghosts, 1: hi)][T planes]
  unsigned* flags_ = nullptr;   // uncached: [0] raised by the lower neighbour, [1] by the upper, [4] timeout, [8] done
  double* peer_stg_[2] = {nullptr, nullptr};   // neighbours' staging (lo, hi)
  unsigned* peer_flags_[2] = {nullptr, nullptr};
  bool peer_ipc_[2] = {false, false};          // opened with hipIpcOpenMemHandle (closed in the destructor)
  int push_epoch_ = 0;                         // passes of the earlier solves (push_cp_wait: epochs run on)
  TbPush* push_host_ = nullptr;                // per pass of a solve (pinned; [0, K) captured, [K, 2K) eager), ...
  TbPush* push_tab_ = nullptr;                 // ... the half the solve being enqueued uses, uploaded at its start ...
  TbPush* push_dev_ = nullptr;                 // ... to this device table the passes read
  TbPush make_push(int j, int npass) const;    // pass j (1-based) of npass
  mutable unsigned push_uid_ = 0;              // solver instance number (table tags)
  i64 stg_off(int par, int field, int side) const { return ((par * 2 + field) * 2 + side) * lay_.xg * lay_.plane; }
  void connect_push_peer(int side, double* stg, unsigned* flags, bool ipc);
  void push_finish(hipStream_t st);  // end of a solve: zero this rank's flags (after its last wait)
  void push_check();                 // after a solve: fail if a wait timed out
  // copy-engine transport (transport_sdma.cpp). Link k = one neighbour: slab ranks [lo, hi] (faces that exist),
  // block ranks the peers of deep_[] in direction order. This rank's flag words: [2k] "arrived" (link k's copies into
  // this rank are complete), [2k + 1] "done" (link k has consumed this rank's previous message and finished the pass
  // that read the regions the next message overwrites).
  struct XLink {
    int peer = -1;
    int side = 0;                  // slab: 0 = lower neighbour, 1 = upper
    int slot = 0;                  // this rank's link index in the PEER's flags
    unsigned* flags = nullptr;     // the peer's flag words (IPC-mapped, or this rank's own for a fake rank)
    double* u[4] = {nullptr, nullptr, nullptr, nullptr};  // slab: the peer's field buffers
    double* recv = nullptr;        // block: the peer's receive staging
    i64 peer_nx = 0;               // slab: the peer's owned planes
    i64 recv_off[6] = {0, 0, 0, 0, 0, 0};  // block: offset of this rank's message in the peer's staging, per depth
                                           // s = 2..5 (indexed by s, like deep_[] and sbase_[])
    bool ipc = false;              // mapped with hipIpcOpenMemHandle (closed in the destructor)
  };
  bool sdma_ = false;
  std::vector<XLink> xlinks_;
  unsigned* xflags_ = nullptr;     // uncached: 2 words per link
  int xpar_ = 0;                   // parity of the solve being enqueued (flag values alternate between two sets)
  unsigned long long xsolves_ = 0; // solves enqueued so far (every rank runs the same number)
  hipGraphExec_t xgraph_[2] = {nullptr, nullptr};  // captured solves of either parity
  // copy streams: link k's wait / copies / signal go to xcs_[k % size] (each stream gets its own SDMA engine, measured:
  // 2 streams move 118 GB/s on one GPU where one moves 60), forked from the exchange stream and joined back
  std::vector<hipStream_t> xcs_;
  std::vector<hipEvent_t> xcev_;
  hipEvent_t xfork_ = nullptr;
  // flag values as device words ([parity][i] = xval(i)): the "arrived" signal is a 4-byte copy-engine write queued
  // after the data copies on the same stream, so no compute queue waits for the copies (a signal kernel would, and a
  // hardware queue shared with s0 would hold the interior pass behind it: measured, profiles/r3)
  unsigned* xvals_ = nullptr;
  unsigned xval(int i) const { return (xpar_ ? 0x10000u : 0u) + static_cast<unsigned>(i + 1); }
  unsigned xend(int par) const { return (par ? 0x10000u : 0u) + 0xFFFFu; }
  void sdma_alloc();
  std::vector<XLink> sdma_links() const;  // link geometry (peer, side, slot) without pointers
  unsigned* xsig(const XLink& l, int word) const { return l.flags + 2 * l.slot + word; }
  void unit_exchange_sdma(int i);  // side stream after unit i's shells (or s0 after the pass): copies + "arrived"
  void sdma_receive(int i);        // s0 before unit i ≥ 1: wait "arrived" (i − 1), unpack, signal "done" (i − 1)
  void sdma_finish();              // s0 after the last unit: "done" for the next solve's first exchange
  void sdma_poison(int i, const int uf[2]);  // --poison-ghosts: NaN into the regions exchange i fills
  unsigned long long flag_ticks() const;     // bound of one in-kernel flag wait (wall-clock ticks)
  // every link has the peer pointers its copies and signals use (connect_sdma / connect_sdma_self / a group): a
  // solver used unconnected would make the copy engines and k_flag_sync write through null + offset (a GPU fault)
  void sdma_check_connected() const;
};

// Per-phase device timers (SolverOptions::timers, eager launches only): every timed launch group is bracketed by two
// events on its stream; after the solve the intervals are summed per phase (and per unit for --trace). Each group is
// also a roctx range ("w3d:<phase>:u<unit>"), so rocprofv3 --marker-trace timelines show the schedule.
template <class F>
void GpuSolver::timed(int phase, hipStream_t st, F&& f) {
  if (!opt_.timers) {
    f();
    return;
  }
  static const char* const kNames[kNumPhases] = {"init", "shell", "compute", "exchange", "check", "gather"};
  char label[48];
  std::snprintf(label, sizeof label, "w3d:%s:u%d", kNames[phase], cur_unit_);
  roctxRangePushA(label);
  auto take = [&]() {
    if (ev_next_ == ev_pool_.size()) {
      hipEvent_t e;
      W3D_HIP(hipEventCreate(&e));
      ev_pool_.push_back(e);
    }
    return ev_pool_[ev_next_++];
  };
  hipEvent_t a = take(), b = take();
  W3D_HIP(hipEventRecord(a, st));
  f();
  W3D_HIP(hipEventRecord(b, st));
  roctxRangePop();
  marks_.push_back({phase, cur_unit_, a, b});
}

}  // namespace wave3d

namespace wave3d {

// P ranks of one decomposition inside ONE process on the current device, halos moved by device-to-device copies.
// Same GpuSolver code as production except the transport; used to validate the multi-rank path on one GPU.
// Transports:
//   "loopback"  : halos by hipMemcpyAsync between the ranks' buffers (no RCCL);
//   "multi-device": rank r on device r (world ≤ visible GPUs), one RCCL communicator over all of them from
//                 ncclCommInitAll, each rank's production solve driven by its own host thread (RCCL needs the ranks'
//                 calls concurrently): real cross-device RCCL / copy-engine traffic without a launcher;
//   "rccl-self" : every rank owns a ONE-rank RCCL communicator (RCCL refuses two ranks of one communicator on one
//                 device, but a one-rank communicator may send to itself) and moves each of its messages with
//                 ncclGroupStart; ncclSend(peer's face, 0); ncclRecv(own ghosts, 0); ncclGroupEnd on its side stream,
//                 the error logs go through ncclAllGather on the same communicators. This executes the production
//                 RCCL calls, their stream placement and event joins on a one-GPU box.
// With options.graph the whole group solve (every rank's streams forked from one group stream) is captured into one
// hipGraph after the first (eager) run and replayed, RCCL kernels included.
class GpuGroup {
 public:
  GpuGroup(const Problem& prob, const SolverOptions& opt, int world, const std::string& transport = "loopback");
  ~GpuGroup();
  GpuGroup(const GpuGroup&) = delete;
  GpuGroup& operator=(const GpuGroup&) = delete;
  RunResult run();  // global error log (rank-ordered combine), solve_s = wall time of the group solve
  GpuSolver& rank(int r) { return *ranks_[static_cast<size_t>(r)]; }
  int world() const { return static_cast<int>(ranks_.size()); }
  const std::string& transport() const { return transport_; }
  bool graph_enabled() const { return multi_ ? ranks_[0]->options().graph : graph_; }
  // RCCL communicators in use and the rank count each reports (rccl-self: world one-rank communicators)
  std::vector<int> comm_counts() const;
  void set_state(const double* prev_global, const double* cur_global, int n0);  // every rank (GpuSolver::set_state)

 private:
  void enqueue();
  void join();
  std::vector<std::unique_ptr<GpuSolver>> ranks_;
  std::string transport_;
  bool graph_ = false;
  int runs_ = 0;
  hipStream_t gs_ = nullptr;
  hipEvent_t fork_ = nullptr;
  hipEvent_t all_packed_ = nullptr, all_pulled_ = nullptr;  // group barriers on gs_ (see enqueue)
  std::vector<hipEvent_t> join_;
  hipGraphExec_t exec_ = nullptr;
  bool multi_ = false;  // "multi-device": every rank on its own GPU, solved by its own thread
};

// Host-scalar collectives over the RCCL communicator (timer max-reduction, barriers). Blocking.
double comm_allreduce(const Comm& c, double v, bool max_op);
// Every rank's bytes (equal sizes), in rank order, through ncclAllGather. Blocking.
std::vector<std::string> comm_allgather_bytes(const Comm& c, const std::string& mine);
int rccl_version();  // ncclGetVersion of the RCCL resolved at run time
// Whether this process's HIP runtime captures the multi-rank (multi-stream) schedules correctly (HIP >= 7.2).
bool multistream_capture_safe();
void comm_barrier(const Comm& c);
}  // namespace wave3d
