// k_leapfrog_p2 instantiations for S = 4 (normal and analytic-start passes), one or two pairs per thread (1024- or
// 512-thread workgroups; LeapfrogTbTiling::p2_pairs). Design: kernels_leapfrog_p2.hip.
#include "wave3d/leapfrog_p2_launch.hpp"

namespace wave3d {
namespace p2k {

void launch_p2_s4(const P2Params& p, int nblocks, bool init, int pairs, hipStream_t st) {
  if (pairs == 2)
    init ? launch_cm<4, true, 2>(p, nblocks, st) : launch_cm<4, false, 2>(p, nblocks, st);
  else
    init ? launch_cm<4, true, 1>(p, nblocks, st) : launch_cm<4, false, 1>(p, nblocks, st);
}
void prepare_p2_s4() {
  prepare_all<4, false, 1>();
  prepare_all<4, true, 1>();
  prepare_all<4, false, 2>();
  prepare_all<4, true, 2>();
}

}  // namespace p2k
}  // namespace wave3d
