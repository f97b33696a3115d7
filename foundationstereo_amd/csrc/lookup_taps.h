// Lookup tap math of geo_lookup_kernel (geometry.hip): the coordinate round trip of the CPU
// grid_sampler, per (pixel, level), shared by every channel of the level.
#pragma once
#include "fsmi_common.h"

namespace fsmi {
namespace {

// FP contraction is OFF for the coordinate math: fusing `ix - floor(ix)` into
// fma(h, x'+1, -floor) computes the fraction from the UNROUNDED ix and moves
// samples near integer positions by up to an ulp of ix (seen as 1e-5 errors
// at x ~ 80 on gfx950 before this pragma).
__device__ __forceinline__ float unnorm(float x, int n) {
#pragma clang fp contract(off)
  const float xn = (2.f * x) / static_cast<float>(n - 1) - 1.f;
  return (xn + 1.f) * (static_cast<float>(n - 1) / 2.f);
}

// The 2r+1 taps of one (pixel, level): window base, per-tap fraction and which
// window pair each tap reads.  Channel-independent, so computed once and
// reused for every channel of the level (the division lives here).
template <int R>
struct Taps {
  static constexpr int K = 2 * R + 1, NW = 2 * R + 4;
  int xb;            // window covers [xb, xb + NW)
  float f[K];        // fraction of tap k
  int sel[K];        // tap k interpolates elements xb+k+sel, xb+k+sel+1, sel in {0,1,2}

  __device__ __forceinline__ void init(float xc, int n) {
#pragma clang fp contract(off)
    // xc = centre coordinate (tap k sits at xc + (k - R)); clamp keeps int math defined
    const float xcl = fminf(fmaxf(xc, -1.0e6f), 1.0e6f);
    xb = static_cast<int>(floorf(xcl)) - R - 1;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float ix = unnorm(static_cast<float>(k - R) + xcl, n);
      const float fl = floorf(ix);
      f[k] = ix - fl;
      sel[k] = static_cast<int>(fl) - xb - k;
    }
  }
};

}  // namespace
}  // namespace fsmi
