// Lookup tap math shared by geo_lookup_kernel (geometry.hip) and the lookup-fused 1x1 conv
// (conv_pw.hip): identical code, hence identical fp32 values, on both paths.
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
  int sel[K];        // tap k interpolates win[k+sel], win[k+sel+1], sel in {0,1,2}
  bool lo, hi;       // window ends needed (only when a tap's round trip crossed an integer)

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
    lo = sel[0] == 0;       // only tap 0 can reach win[0]
    hi = sel[K - 1] == 2;   // only tap 2r can reach win[2r+3]
  }

  __device__ __forceinline__ void sample(const float* __restrict__ src, size_t stride, int n,
                                         float* __restrict__ dst, size_t dstride) const {
#pragma clang fp contract(off)
    // the 2r+2 window elements every tap set touches, plus the two ends only for lanes whose
    // taps need them: HBM sees the algorithmic 2r+2 loads per channel
    float win[NW];
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      const int x = xb + j;
      const bool need = (j == 0) ? lo : ((j == NW - 1) ? hi : true);
      win[j] = (need && x >= 0 && x < n) ? src[static_cast<size_t>(x) * stride] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float v0 = sel[k] == 0 ? win[k] : (sel[k] == 1 ? win[k + 1] : win[k + 2]);
      const float v1 = sel[k] == 0 ? win[k + 1] : (sel[k] == 1 ? win[k + 2] : win[k + 3]);
      dst[static_cast<size_t>(k) * dstride] = v0 * (1.f - f[k]) + v1 * f[k];
    }
  }
};

// The same samples as Taps, for callers that prefetch them across other work: each tap's two
// neighbours loaded directly (2 loads per tap instead of the shared 2r+4 window, so no window array
// is selected from -- a window held across a loop body was folded into one dynamically indexed
// scratch array).  Identical values: x0 = floor(ix) is the element Taps reads as win[k + sel[k]].
template <int R>
struct TapPairs {
  static constexpr int K = 2 * R + 1;
  float fr[K], v0[K], v1[K];

  __device__ __forceinline__ void load(const float* __restrict__ src, size_t stride, int n, float xc) {
#pragma clang fp contract(off)
    const float xcl = fminf(fmaxf(xc, -1.0e6f), 1.0e6f);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float ix = unnorm(static_cast<float>(k - R) + xcl, n);
      const float fl = floorf(ix);
      fr[k] = ix - fl;
      const int x0 = static_cast<int>(fl);
      v0[k] = (x0 >= 0 && x0 < n) ? src[static_cast<size_t>(x0) * stride] : 0.f;
      v1[k] = (x0 + 1 >= 0 && x0 + 1 < n) ? src[static_cast<size_t>(x0 + 1) * stride] : 0.f;
    }
  }
  __device__ __forceinline__ float value(int k) const {
#pragma clang fp contract(off)
    return v0[k] * (1.f - fr[k]) + v1[k] * fr[k];
  }
};

}  // namespace
}  // namespace fsmi
