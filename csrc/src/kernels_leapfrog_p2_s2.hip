// k_leapfrog_p2 instantiations for S = 2 (normal and analytic-start passes). Design: kernels_leapfrog_p2.hip.
#include "wave3d/leapfrog_p2_launch.hpp"

namespace wave3d {
namespace p2k {

void launch_p2_s2(const P2Params& p, int nblocks, bool init, hipStream_t st) {
  init ? launch_cm<2, true>(p, nblocks, st) : launch_cm<2, false>(p, nblocks, st);
}
void prepare_p2_s2() {
  prepare_all<2, false>();
  prepare_all<2, true>();
}

}  // namespace p2k
}  // namespace wave3d
