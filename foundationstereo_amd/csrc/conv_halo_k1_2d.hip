// Halo conv tiles for 1x1 kernels on 2D maps (device code: conv_halo.h).
#include "conv_halo.h"

FSMI_HALO_LAUNCH_CFG(1, false)
