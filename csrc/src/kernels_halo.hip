// Halo pack / unpack kernels: the strided (y and z) faces of the single-step 3-D block decomposition (k_pack) and the
// S-deep face/edge/corner regions of the multi-step block passes (k_box_copy) (reference kernel K6,
// SURVEY.md §2.5; the reference staged faces through the host, report.pdf p.16 §4.4 H2D/D2H column).
// x faces are whole contiguous planes and go to RCCL straight from the field: no kernel at all.
//
// One launch covers every strided face of a rank (blockIdx.y = face): a y face is nx rows of nz contiguous nodes
// (coalesced), a z face is nx·ny single nodes one pitch apart (gather, small).
#include <hip/hip_runtime.h>

#include "wave3d/kernels.hpp"

namespace wave3d {

namespace {

constexpr int kMaxPacked = 4;

struct PackFace {
  i64 count;     // nodes in the face
  i64 inner;     // length of the fast index (nz for y faces, ny for z faces)
  i64 buf_off;   // offset in the staging buffer
  i64 layer;     // layer index along the face axis (send layer for pack, ghost layer for unpack)
  int axis;
};

struct PackParams {
  double* field;
  double* buf;
  i64 plane, pitch, zs;
  int nface;
  PackFace f[kMaxPacked];
};

template <bool PACK>
__global__ __launch_bounds__(256) void k_pack(const PackParams p) {
  const int fi = blockIdx.y;
  PackFace f = p.f[0];
#pragma unroll
  for (int k = 1; k < kMaxPacked; ++k)
    if (k == fi) f = p.f[k];
  const i64 stride = static_cast<i64>(gridDim.x) * blockDim.x;
  for (i64 q = static_cast<i64>(blockIdx.x) * blockDim.x + threadIdx.x; q < f.count; q += stride) {
    const i64 ix = q / f.inner, r = q - ix * f.inner;
    i64 o;
    if (f.axis == 1)
      o = (ix + 1) * p.plane + (f.layer + 1) * p.pitch + (r + 1 + p.zs);
    else
      o = (ix + 1) * p.plane + (r + 1) * p.pitch + (f.layer + 1 + p.zs);
    if (PACK)
      p.buf[f.buf_off + q] = p.field[o];
    else
      p.field[o] = p.buf[f.buf_off + q];
  }
}

template <bool PACK>
void launch(const Layout& l, const HaloPlan& plan, double* field, double* buf, hipStream_t st) {
  PackParams p{};
  p.field = field + l.kbase();
  p.buf = buf;
  p.plane = l.plane;
  p.pitch = l.pitch;
  p.zs = l.zs;
  i64 maxc = 0;
  for (const Face& f : plan.faces) {
    if (f.contiguous) continue;
    W3D_REQUIRE(p.nface < kMaxPacked, "too many strided faces");
    PackFace& d = p.f[p.nface++];
    d.count = f.count;
    d.axis = f.axis;
    d.inner = f.axis == 1 ? l.nz : l.ny;
    d.buf_off = f.pack_off;
    d.layer = PACK ? f.send_layer : f.recv_layer;
    maxc = imax(maxc, f.count);
  }
  if (p.nface == 0) return;
  const unsigned gx = static_cast<unsigned>(imin(ceil_div(maxc, 256), 1024));
  hipLaunchKernelGGL(k_pack<PACK>, dim3(gx, p.nface), dim3(256), 0, st, p);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) fail(std::string("pack/unpack launch: ") + hipGetErrorString(e));
}

// ---------------------------------------------------------------------------------------------------------------
// k_box_copy: general box <-> staging-buffer copies of the S-deep exchanges (deep_plan.hpp). One launch moves every
// region of every peer message (both fields); the job table lives in device memory (built once per plan, so a
// captured graph holds only the pointers). Element e of a box runs in C order (x, y, z): consecutive lanes read
// consecutive z nodes of a row — whole 128-B lines for x and y faces, the w ≤ 4 contiguous nodes of each row for z
// faces (what the layout offers) — and the staging side is written fully contiguous.
// ---------------------------------------------------------------------------------------------------------------
constexpr int kBoxThreads = 256, kBoxPer = 4;  // elements per thread

struct BoxCopyParams {
  double* f[2];
  double* buf;
  const BoxJob* jobs;
  int njobs;
  i64 plane, pitch, zs;
};

template <int MODE>  // 0 pack, 1 unpack, 2 poison (NaN into the receive regions)
__global__ __launch_bounds__(kBoxThreads) void k_box_copy(const BoxCopyParams p) {
  const int b = static_cast<int>(blockIdx.x);
  int j = 0;
  while (j + 1 < p.njobs && p.jobs[j + 1].blk0 <= b) ++j;  // (≤ 52 jobs, wave-uniform scalar loads)
  const BoxJob jb = p.jobs[j];
  double* f = p.f[jb.field];
  const int base = (b - jb.blk0) * (kBoxThreads * kBoxPer) + static_cast<int>(threadIdx.x);
#pragma unroll
  for (int k = 0; k < kBoxPer; ++k) {
    const int e = base + k * kBoxThreads;
    if (e >= jb.count) break;
    const int t = e / jb.nz;
    const int z = jb.z0 + (e - t * jb.nz);
    const int yy = t / jb.ny;
    const int y = jb.y0 + (t - yy * jb.ny);
    const int x = jb.x0 + yy;
    const i64 o = static_cast<i64>(x + 1) * p.plane + static_cast<i64>(y + 1) * p.pitch + (z + 1 + p.zs);
    if constexpr (MODE == 0)
      p.buf[jb.buf + e] = f[o];
    else if constexpr (MODE == 1)
      f[o] = p.buf[jb.buf + e];
    else
      f[o] = __builtin_nan("");
  }
}

}  // namespace

BoxCopyTable make_box_copy_table(const DeepPlan& plan, bool recv_side, bool skip_zfaces) {
  std::vector<BoxJob> jobs;
  int blk = 0;
  for (const DeepPeer& q : plan.peers)
    for (const DeepPart& part : q.parts) {
      if (skip_zfaces && q.dir[0] == 0 && q.dir[1] == 0) continue;
      const LBox& b = recv_side ? part.recv : part.send;
      const i64 cnt = b.count();
      if (cnt == 0) continue;
      W3D_REQUIRE(cnt < (1ll << 31) - kBoxThreads * kBoxPer, "box copy: region too large for 32-bit indexing");
      BoxJob jb;
      jb.buf = q.buf_off + part.off;
      jb.count = static_cast<int>(cnt);
      jb.field = part.field;
      jb.x0 = static_cast<int>(b.x0);
      jb.y0 = static_cast<int>(b.y0);
      jb.z0 = static_cast<int>(b.z0);
      jb.ny = static_cast<int>(b.y1 - b.y0);
      jb.nz = static_cast<int>(b.z1 - b.z0);
      jb.blk0 = blk;
      blk += static_cast<int>(ceil_div(cnt, kBoxThreads * kBoxPer));
      jobs.push_back(jb);
    }
  BoxCopyTable t;
  t.njobs = static_cast<int>(jobs.size());
  t.nblocks = blk;
  if (!jobs.empty()) {
    hipError_t e = hipMalloc(&t.jobs, jobs.size() * sizeof(BoxJob));
    if (e == hipSuccess) e = hipMemcpy(t.jobs, jobs.data(), jobs.size() * sizeof(BoxJob), hipMemcpyHostToDevice);
    if (e != hipSuccess) fail(std::string("box copy table: ") + hipGetErrorString(e));
  }
  return t;
}

void free_box_copy_table(BoxCopyTable& t) {
  if (t.jobs) (void)hipFree(t.jobs);
  t.jobs = nullptr;
  t.njobs = t.nblocks = 0;
}

void launch_box_copy(const Layout& l, const BoxCopyTable& t, int mode, double* u_s, double* u_s1, double* buf,
                     hipStream_t st) {
  if (t.njobs == 0) return;
  BoxCopyParams p{};
  p.f[0] = u_s + l.kbase();
  p.f[1] = u_s1 + l.kbase();
  p.buf = buf;
  p.jobs = t.jobs;
  p.njobs = t.njobs;
  p.plane = l.plane;
  p.pitch = l.pitch;
  p.zs = l.zs;
  const dim3 grid(static_cast<unsigned>(t.nblocks));
  if (mode == 0)
    hipLaunchKernelGGL(k_box_copy<0>, grid, dim3(kBoxThreads), 0, st, p);
  else if (mode == 1)
    hipLaunchKernelGGL(k_box_copy<1>, grid, dim3(kBoxThreads), 0, st, p);
  else
    hipLaunchKernelGGL(k_box_copy<2>, grid, dim3(kBoxThreads), 0, st, p);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) fail(std::string("box copy launch: ") + hipGetErrorString(e));
}

void launch_pack(const Layout& l, const HaloPlan& plan, const double* u, double* buf, hipStream_t stream) {
  launch<true>(l, plan, const_cast<double*>(u), buf, stream);
}

void launch_unpack(const Layout& l, const HaloPlan& plan, const double* buf, double* u, hipStream_t stream) {
  launch<false>(l, plan, u, const_cast<double*>(buf), stream);
}

// ------------------------------------------------------------------------------------------------------------------
// Flag words of the copy-engine transport (transport_sdma.cpp): one-workgroup kernels, because a stream wait on a memory
// value (hipStreamWaitValue32) is not recorded into a hipGraph by this HIP runtime (it runs once, at capture time:
// tools/probes/memop_capture_probe.hip) while kernel nodes replay. Flag words live in uncached device memory (local or a
// peer's, IPC-mapped); every access is a system-scope vector atomic.
// ------------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_flag_sync(const FlagOp w, const FlagOp s) {
  const int t = static_cast<int>(threadIdx.x);
  // wait until every watched word equals the value (bounded: after `ticks` of the 100 MHz wall clock the status word
  // records a timeout and the kernel ends, so a lost peer turns into a host-side error instead of a hung queue).
  // Once any wait of this solve has timed out (status set, by this kernel or an earlier one on any stream of the rank)
  // the solve is lost: later waits return at once, so the rest of the solve drains in microseconds and a lost peer
  // costs one bound per solve, not one per wait. The status word is re-read inside
  // the spin too, so the lanes of one kernel (and concurrent kernels on the copy streams) give up together.
  if (t < w.n) {
    auto lost = [&] { return __hip_atomic_load(w.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u; };
    const unsigned long long t0 = wall_clock64();
    unsigned* a = w.addr[t];
    while (!lost() && __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != w.value) {
      if (wall_clock64() - t0 > w.ticks) {
        __hip_atomic_store(w.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
  }
  __syncthreads();
  if (t < s.n) __hip_atomic_store(s.addr[t], s.value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_flag_sync(const FlagOp& wait, const FlagOp& signal, hipStream_t stream) {
  W3D_REQUIRE(wait.n <= FlagOp::kMax && signal.n <= FlagOp::kMax && wait.n >= 0 && signal.n >= 0, "flag op: too many");
  if (wait.n == 0 && signal.n == 0) return;
  hipLaunchKernelGGL(k_flag_sync, dim3(1), dim3(64), 0, stream, wait, signal);
}

// ------------------------------------------------------------------------------------------------------------------
// Field hash (autotune field check): one workgroup per group of owned rows, a 64-bit sum that does not depend on the
// order in which nodes are visited, so it is the same for any decomposition of the same global field.
// ------------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {  // (splitmix64 finaliser)
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void k_field_hash(const double* f, const Layout l, unsigned long long* out) {
  unsigned long long acc = 0;
  const i64 rows = l.nx * l.ny, n1 = l.N + 1;
  for (i64 r = blockIdx.x; r < rows; r += gridDim.x) {
    const i64 x = r / l.ny, y = r - x * l.ny;
    const double* row = f + l.off(x, y, 0);
    const i64 g = ((l.gx0 + x) * n1 + (l.gy0 + y)) * n1 + l.gz0;
    for (i64 z = threadIdx.x; z < l.nz; z += blockDim.x)
      acc += mix64(static_cast<unsigned long long>(__double_as_longlong(row[z])) ^ mix64(static_cast<unsigned long long>(g + z)));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);
}

void launch_field_hash(const Layout& l, const double* f, unsigned long long* out, hipStream_t stream) {
  const i64 rows = l.nx * l.ny;
  if (rows <= 0 || l.nz <= 0) return;
  const unsigned blocks = static_cast<unsigned>(imin(rows, static_cast<i64>(4096)));
  hipLaunchKernelGGL(k_field_hash, dim3(blocks), dim3(256), 0, stream, f, l, out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) fail(std::string("field hash launch: ") + hipGetErrorString(e));
}

}  // namespace wave3d
