// Halo conv tiles for 1x1 kernels on NCDHW volumes (KD x 1 x 1 taps) (device code: conv_halo.h).
#include "conv_halo.h"

FSMI_HALO_LAUNCH_CFG(1, true)
