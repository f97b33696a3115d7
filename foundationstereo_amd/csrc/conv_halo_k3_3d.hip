// Halo conv tiles for 3x3 kernels on NCDHW volumes (KD x 3 x 3 taps) (device code: conv_halo.h).
#include "conv_halo.h"

FSMI_HALO_LAUNCH_CFG(3, true)
