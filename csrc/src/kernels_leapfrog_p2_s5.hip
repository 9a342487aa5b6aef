// k_leapfrog_p2 instantiations for S = 5 (normal passes: the schedule's analytic start takes 4 steps). One or two
// pairs per thread (1024- or 512-thread workgroups; LeapfrogTbTiling::p2_pairs). Design: kernels_leapfrog_p2.hip.
#include "wave3d/leapfrog_p2_launch.hpp"

namespace wave3d {
namespace p2k {

void launch_p2_s5(const P2Params& p, int nblocks, int pairs, hipStream_t st) {
  pairs == 2 ? launch_cm<5, false, 2>(p, nblocks, st) : launch_cm<5, false, 1>(p, nblocks, st);
}
void prepare_p2_s5() {
  prepare_all<5, false, 1>();
  prepare_all<5, false, 2>();
}

}  // namespace p2k
}  // namespace wave3d
