// Halo pack / unpack kernels for the strided (y and z) faces of the 3-D block decomposition (reference kernel K6,
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

}  // namespace

void launch_pack(const Layout& l, const HaloPlan& plan, const double* u, double* buf, hipStream_t stream) {
  launch<true>(l, plan, const_cast<double*>(u), buf, stream);
}

void launch_unpack(const Layout& l, const HaloPlan& plan, const double* buf, double* u, hipStream_t stream) {
  launch<false>(l, plan, u, const_cast<double*>(buf), stream);
}

}  // namespace wave3d
