// Job launch pieces of the native runtime: launcher environments, the --np self-spawn, the RCCL unique-id rendezvous
// and host collectives. See wave3d/runtime.hpp. (The reference launches with `mpirun -np P` under LSF, report.pdf
// p.12-15; here torchrun / mpiexec / srun environments or the built-in spawn)
#include <signal.h>
#include <sys/prctl.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <sstream>
#include <thread>

#include "wave3d/runtime.hpp"

namespace wave3d {

const char* const kRankEnv[] = {"RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "SLURM_PROCID", nullptr};
const char* const kSizeEnv[] = {"WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "SLURM_NTASKS", nullptr};
const char* const kLocalEnv[] = {"LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", "SLURM_LOCALID",
                                 nullptr};

int env_int(const char* const* names, int dflt) {
  for (const char* const* n = names; *n; ++n) {
    const char* v = std::getenv(*n);
    if (v && *v) return std::atoi(v);
  }
  return dflt;
}

double wall_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// W3D_JOB_ID, else the launcher's job id (torchrun TORCHELASTIC_RUN_ID, SLURM_JOB_ID, PMIx namespace), else
// MASTER_PORT, else the parent pid (the ranks of one node are children of the same launcher process).
std::string job_segment_name() {
  static const char* const kJob[] = {"W3D_JOB_ID", "TORCHELASTIC_RUN_ID", "SLURM_JOB_ID", "PMIX_NAMESPACE",
                                     "OMPI_MCA_orte_ess_jobid", "MASTER_PORT", nullptr};
  std::string id;
  for (const char* const* n = kJob; *n && id.empty(); ++n)
    if (const char* v = std::getenv(*n); v && *v) id = v;
  if (id.empty()) id = std::to_string(static_cast<long long>(getppid()));
  std::string name = "/wave3d-cpu-";
  for (char c : id) name += std::isalnum(static_cast<unsigned char>(c)) ? c : '_';
  return name;
}

// The name is per launch: W3D_RDZV_FILE (the --np self-spawn and bench.py pass a fresh nonce), else MASTER_PORT +
// TORCHELASTIC_RUN_ID + the launcher's pid (the ranks of one torchrun/mpiexec job share their parent). Rank 0 removes a
// stale file of that name before publishing, and the other ranks only accept a file written after they started (minus
// a grace period for a fast rank 0), so a file left by a crashed earlier job is never consumed.
std::string rdzv_path() {
  if (const char* p = std::getenv("W3D_RDZV_FILE")) return p;
  const char* port = std::getenv("MASTER_PORT");
  const char* run = std::getenv("TORCHELASTIC_RUN_ID");
  std::ostringstream os;
  os << "/tmp/wave3d-rdzv-" << (port ? port : "0") << "-" << (run ? run : "x") << "-" << getppid() << ".uid";
  return os.str();
}

namespace {
const double kProcessStart = static_cast<double>(std::time(nullptr));  // (static init: before main)

bool fresh_file(const std::string& path) {
  struct stat st {};
  return stat(path.c_str(), &st) == 0 && static_cast<double>(st.st_mtime) >= kProcessStart - 60.0;
}

std::string slurp(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  return std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

void publish(const std::string& path, const std::string& bytes) {
  const std::string tmp = path + ".tmp";
  {
    std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
    f.write(bytes.data(), static_cast<std::streamsize>(bytes.size()));
    if (!f) fail("cannot write " + tmp);
  }
  if (std::rename(tmp.c_str(), path.c_str()) != 0) fail("cannot publish " + path);
}
}  // namespace

std::string exchange_unique_id(int rank) {
  const std::string path = rdzv_path();
  if (rank == 0) {
    std::remove(path.c_str());
    const std::string id = Comm::make_unique_id();
    publish(path, id);
    return id;
  }
  const double t0 = wall_s();
  for (;;) {
    if (fresh_file(path)) {
      const std::string id = slurp(path);
      if (id.size() == 128) return id;
    }
    if (wall_s() - t0 > 120.0) fail("timed out waiting for rendezvous file " + path);
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

double proc_timeout_s() {
  const char* v = std::getenv("W3D_FILE_TIMEOUT_S");
  const double t = v ? std::atof(v) : 0.0;
  return t > 0.0 ? t : 120.0;
}

std::vector<std::string> file_allgather(int rank, int world, const std::string& mine, const std::string& tag,
                                        double timeout_s) {
  auto path = [&](int r) { return rdzv_path() + "." + tag + std::to_string(r); };
  publish(path(rank), mine);
  std::vector<std::string> all(static_cast<size_t>(world));
  const double t0 = wall_s();
  const double bound = timeout_s == 0.0 ? proc_timeout_s() : timeout_s;  // (< 0: while the parent lives)
  const pid_t parent = getppid();
  for (int r = 0; r < world; ++r) {
    for (;;) {
      if (fresh_file(path(r))) {
        std::string b = slurp(path(r));
        if (b.size() == mine.size()) {
          all[static_cast<size_t>(r)] = std::move(b);
          break;
        }
      }
      const double waited = wall_s() - t0;
      if (bound > 0.0 && waited > bound) fail("timed out waiting for " + path(r));  // (a peer that died)
      if (bound < 0.0 && getppid() != parent) fail("the parent process exited while waiting for " + path(r));
      // poll fast first: this is also the per-solve barrier of ranks without a communicator, and a rank leaving it
      // 20 ms after its peer made the peer's solve wait that long for its flags (solve-time mean 3x the best, measured
      // on 2 processes sharing one GPU: profiles/r4/proc_parity.md); back off once a peer is clearly slow
      std::this_thread::sleep_for(waited < 0.25 ? std::chrono::microseconds(50) : std::chrono::microseconds(20000));
    }
  }
  return all;
}

// The ranks live and die with the spawner: each child asks the kernel for SIGKILL when its parent
// exits (PR_SET_PDEATHSIG, before it touches the GPU), so a spawner killed by a timeout takes its ranks along instead
// of leaving them spinning on the GPU; and once one rank has failed, the spawner gives the others W3D_SPAWN_GRACE_S
// (default 20 s) to report their own error (a peer's lost-neighbour timeout) and then kills the rest.
int spawn_ranks(int np) {
  std::ostringstream rf;
  rf << "/tmp/wave3d-rdzv-spawn-" << getpid() << "-" << static_cast<long long>(wall_s() * 1e6) << ".uid";
  const std::string rdzv = rf.str();
  const pid_t parent = getpid();
  std::vector<pid_t> kids;
  for (int r = 0; r < np; ++r) {
    const pid_t pid = fork();
    if (pid < 0) {
      for (pid_t k : kids) kill(k, SIGKILL);
      fail("fork failed");
    }
    if (pid == 0) {
      if (prctl(PR_SET_PDEATHSIG, SIGKILL) != 0 || getppid() != parent) _exit(125);  // (parent already gone)
      setenv("RANK", std::to_string(r).c_str(), 1);
      setenv("LOCAL_RANK", std::to_string(r).c_str(), 1);
      setenv("WORLD_SIZE", std::to_string(np).c_str(), 1);
      setenv("W3D_RDZV_FILE", rdzv.c_str(), 1);
      setenv("W3D_SPAWNED", "1", 1);
      return -1;  // child: continue
    }
    kids.push_back(pid);
  }
  double grace = 20.0;
  if (const char* g = std::getenv("W3D_SPAWN_GRACE_S"); g && std::atof(g) >= 0.0) grace = std::atof(g);
  int rc = 0, left = np;
  double t_fail = -1.0;
  std::vector<char> alive(static_cast<size_t>(np), 1);
  while (left > 0) {
    int st = 0;
    const pid_t k = waitpid(-1, &st, WNOHANG);
    if (k < 0) break;  // (no children left)
    if (k == 0) {
      if (t_fail >= 0.0 && wall_s() - t_fail > grace) {
        for (int r = 0; r < np; ++r)
          if (alive[static_cast<size_t>(r)]) kill(kids[static_cast<size_t>(r)], SIGKILL);
        t_fail = 1e300;  // (killed once; keep reaping)
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
      continue;
    }
    for (int r = 0; r < np; ++r)
      if (kids[static_cast<size_t>(r)] == k) alive[static_cast<size_t>(r)] = 0;
    --left;
    const int c = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
    if (c != 0 && rc == 0) {
      rc = c;
      if (t_fail < 0.0) t_fail = wall_s();
    }
  }
  std::remove(rdzv.c_str());
  return rc;
}

// ---------------------------------------------------------------------------------------------------------------
HostColl HostColl::single(int rank) {
  HostColl h;
  h.rank = rank;
  h.world = 1;
  h.agree = [](bool ok) { return ok; };
  h.max = [](double v) { return v; };
  h.barrier = [] {};
  h.allgather = [](const std::string& b) { return std::vector<std::string>{b}; };
  h.cleanup = [] {};
  return h;
}

HostColl HostColl::rccl(std::shared_ptr<Comm> c) {
  HostColl h;
  h.rank = c->rank();
  h.world = c->world();
  const double w = static_cast<double>(c->world());
  h.agree = [c, w](bool ok) { return comm_allreduce(*c, ok ? 1.0 : 0.0, false) == w; };
  h.max = [c](double v) { return comm_allreduce(*c, v, true); };
  h.barrier = [c] { comm_barrier(*c); };
  h.allgather = [c](const std::string& b) { return comm_allgather_bytes(*c, b); };
  h.cleanup = [] {};
  return h;
}

HostColl HostColl::files(int rank, int world) {
  // every collective is a file all-gather with its own tag; each rank keeps the list of its files to remove them at the
  // end — all but the last one, which a peer may still be reading (every earlier one has been read by everyone, since
  // every peer has entered a later collective; removing a file a peer still needs would hang that peer)
  struct State {
    int n = 0;
    std::vector<std::string> mine;
  };
  auto st = std::make_shared<State>();
  auto gather_t = [st, rank, world](const std::string& b, double timeout_s) {
    const std::string tag = "c" + std::to_string(st->n++) + "r";
    st->mine.push_back(rdzv_path() + "." + tag + std::to_string(rank));
    return file_allgather(rank, world, b, tag, timeout_s);
  };
  auto gather = [gather_t](const std::string& b) { return gather_t(b, 0.0); };
  HostColl h;
  h.rank = rank;
  h.world = world;
  h.allgather = gather;
  h.agree = [gather](bool ok) {
    bool all = true;
    for (const std::string& b : gather(std::string(1, ok ? '1' : '0'))) all = all && b == "1";
    return all;
  };
  h.max = [gather](double v) {
    double m = v;
    for (const std::string& b : gather(std::string(reinterpret_cast<const char*>(&v), sizeof v))) {
      double x = 0.0;
      std::memcpy(&x, b.data(), sizeof x);
      m = std::max(m, x);
    }
    return m;
  };
  h.barrier = [gather] { (void)gather("b"); };
  // the serve loop's barrier before a solve: the peer ranks' Python callers may spend any time between run()
  // calls, so it waits as long as this rank's parent lives — or W3D_PROC_TIMEOUT_S if set, the bound the
  // Python side (NativeRankProcess) puts on every reply (the other file collectives: W3D_FILE_TIMEOUT_S, 120 s). A
  // rank whose peer died does not poll forever: its own caller's reply wait (300 s by default) kills it
  // (native_proc.py _read), and PDEATHSIG ends it with its parent
  h.idle_barrier = [gather_t] {
    const char* v = std::getenv("W3D_PROC_TIMEOUT_S");
    (void)gather_t("b", v && std::atof(v) > 0.0 ? std::atof(v) : -1.0);
  };
  h.cleanup = [st] {
    for (size_t i = 0; i + 1 < st->mine.size(); ++i) std::remove(st->mine[i].c_str());
  };
  return h;
}

}  // namespace wave3d
