// 2x2 tiles of the halo conv on 2D maps: the four output phases of a ConvTranspose2d(k=4, s=2, p=1)
// (fsmi_conv2d_up2_halo_x3; spx_2_gru.conv1 and spx_gru, core/foundation_stereo.py:183-191).
// Register-weight tiles only (no K groups).
#include "conv_halo.h"

namespace fsmi {
namespace halo {

template <>
int launch_cfg<2, false>(int cfg, int kg, const HaloArgs& a, hipStream_t s) {
  if (kg != 1) {
    set_error("fsmi_conv_halo: 2x2 tiles have no K-group variant");
    return FSMI_ERR_ARG;
  }
  switch (cfg) {
    case 2: launch_tile<2, 64, 8, 1, true, false>(a, s); break;
    case 3: launch_tile<2, 128, 4, 2, true, false>(a, s); break;
    case 5: launch_tile<2, 64, 4, 1, true, false>(a, s); break;
    case 6: launch_tile<2, 32, 8, 1, true, false>(a, s); break;
    case 7: launch_tile<2, 32, 4, 1, true, false>(a, s); break;
    default:
      set_error("fsmi_conv_halo: 2x2 tile %d (2, 3, 5, 6, 7)", cfg);
      return FSMI_ERR_ARG;
  }
  return finish_launch("fsmi_conv_halo");
}

}  // namespace halo
}  // namespace fsmi
