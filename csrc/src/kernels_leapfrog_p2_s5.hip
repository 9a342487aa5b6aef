// k_leapfrog_p2 instantiations for S = 5 (normal passes only: an analytic-start pass of 5 stages needs one more level
// of register queues than 128 VGPRs hold). Design: kernels_leapfrog_p2.hip.
#include "wave3d/leapfrog_p2_launch.hpp"

namespace wave3d {
namespace p2k {

void launch_p2_s5(const P2Params& p, int nblocks, bool init, hipStream_t st) {
  W3D_REQUIRE(!init, "leapfrog_p2: the analytic-start pass takes at most 4 steps");
  launch_cm<5, false>(p, nblocks, st);
}
void prepare_p2_s5() { prepare_all<5, false>(); }

}  // namespace p2k
}  // namespace wave3d
