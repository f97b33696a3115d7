// Stride-2 tiles of the halo conv (fsmi_conv3d_halo_x3_ex, stride 2): the hourglass's
// BasicConv3d(k=3, s=2, p=1) (core/foundation_stereo.py:50-58) with KS = KD = 3, and -- as volumes of
// depth 1 -- the context net's 3x3 s2 p1 convs and 1x1 s2 projections (core/extractor.py:20-80).
// Register-weight tiles, no K groups.  The staged window of a TR x 32 output tile is
// (2 TR + KS - 2) x (63 + KS - 1) input pixels: for KS = 3, 52 KB of LDS at TR = 2 (three blocks
// per CU), 94 KB at TR = 4 (one).
#include "conv_halo.h"

namespace fsmi {
namespace halo {

template <int KS>
int launch_s2_ks(int cfg, const HaloArgs& a, hipStream_t s) {
  switch (cfg) {
    case 4: launch_tile<KS, 128, 2, 2, true, true, 1, 2>(a, s); break;
    case 5: launch_tile<KS, 64, 4, 1, true, true, 1, 2>(a, s); break;
    case 7: launch_tile<KS, 32, 4, 1, true, true, 1, 2>(a, s); break;
    case 10: launch_tile<KS, 64, 2, 2, true, true, 1, 2>(a, s); break;
    default:
      set_error("fsmi_conv3d_halo_x3: stride-2 tile %d (4, 5, 7, 10)", cfg);
      return FSMI_ERR_ARG;
  }
  return finish_launch("fsmi_conv3d_halo_x3 (stride 2)");
}

int launch_s2(int ks, int cfg, const HaloArgs& a, hipStream_t s) {
  return ks == 1 ? launch_s2_ks<1>(cfg, a, s) : launch_s2_ks<3>(cfg, a, s);
}

}  // namespace halo
}  // namespace fsmi
