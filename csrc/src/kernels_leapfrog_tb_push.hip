// Push-transport instantiations of the LDS S-step kernel (k_leapfrog_tb<…, PUSH = true>): the slab pass that also
// forwards its face planes into the neighbours' staging, reads its ghosts from its own staging and waits / signals
// with flags (TbPush, kernels.hpp). A separate translation unit so the PUSH = false kernels of one-rank and RCCL runs
// keep their own register allocation and the two halves compile in parallel.
#include "wave3d/leapfrog_tb_kernel.hpp"

namespace wave3d {
namespace tbk {

// the analytic-start pass with the tiling's init_threads (768: no spills, as on one rank), the others with 1024
void launch_push(const TbParams& p, int nblocks, int stages, bool init, int init_threads, hipStream_t st) {
  const bool i768 = init && init_threads == 768;
  switch (stages) {
    case 2:
      if (i768) launch_nt<2, 768, true, true>(p, nblocks, st);
      else init ? launch_nt<2, 1024, true, true>(p, nblocks, st) : launch_nt<2, 1024, false, true>(p, nblocks, st);
      break;
    case 3:
      if (i768) launch_nt<3, 768, true, true>(p, nblocks, st);
      else init ? launch_nt<3, 1024, true, true>(p, nblocks, st) : launch_nt<3, 1024, false, true>(p, nblocks, st);
      break;
    default:
      if (i768) launch_nt<4, 768, true, true>(p, nblocks, st);
      else init ? launch_nt<4, 1024, true, true>(p, nblocks, st) : launch_nt<4, 1024, false, true>(p, nblocks, st);
      break;
  }
}

void prepare_push() {
  prepare_nt<2, 1024, false, true>();
  prepare_nt<3, 1024, false, true>();
  prepare_nt<4, 1024, false, true>();
  prepare_nt<2, 1024, true, true>();
  prepare_nt<3, 1024, true, true>();
  prepare_nt<4, 1024, true, true>();
  prepare_nt<2, 768, true, true>();
  prepare_nt<3, 768, true, true>();
  prepare_nt<4, 768, true, true>();
}

}  // namespace tbk
}  // namespace wave3d
