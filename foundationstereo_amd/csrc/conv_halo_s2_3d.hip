// Stride-2 3x3x3 volume tiles of the halo conv: the hourglass's BasicConv3d(k=3, s=2, p=1)
// (core/foundation_stereo.py:50-58; fsmi_conv3d_s2_halo_x3).  Register-weight tiles, no K groups.
// The staged window of a TR x 32 output tile is (2 TR + 1) x 65 input pixels: 52 KB of LDS for
// TR = 2 (three blocks per CU), 94 KB for TR = 4 (one).
#include "conv_halo.h"

namespace fsmi {
namespace halo {

int launch_s2(int cfg, const HaloArgs& a, hipStream_t s) {
  switch (cfg) {
    case 4: launch_tile<3, 128, 2, 2, true, true, 1, 2>(a, s); break;
    case 5: launch_tile<3, 64, 4, 1, true, true, 1, 2>(a, s); break;
    case 7: launch_tile<3, 32, 4, 1, true, true, 1, 2>(a, s); break;
    case 10: launch_tile<3, 64, 2, 2, true, true, 1, 2>(a, s); break;
    default:
      set_error("fsmi_conv3d_s2_halo_x3: tile %d (4, 5, 7, 10)", cfg);
      return FSMI_ERR_ARG;
  }
  return finish_launch("fsmi_conv3d_s2_halo_x3");
}

}  // namespace halo
}  // namespace fsmi
