// k_leapfrog_p2 instantiations for S = 4 (normal and analytic-start passes). Design: kernels_leapfrog_p2.hip.
#include "wave3d/leapfrog_p2_launch.hpp"

namespace wave3d {
namespace p2k {

void launch_p2_s4(const P2Params& p, int nblocks, bool init, hipStream_t st) {
  init ? launch_cm<4, true>(p, nblocks, st) : launch_cm<4, false>(p, nblocks, st);
}
void prepare_p2_s4() {
  prepare_all<4, false>();
  prepare_all<4, true>();
}

}  // namespace p2k
}  // namespace wave3d
