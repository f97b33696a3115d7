// Small fused heads on the refinement path:
// soft-argmin over disparity, convex x4 upsampling, and the selective ConvGRU
// gate/blend elementwise work.  All HBM-bound: one thread per output pixel
// (channel loops inside), lanes over w so every access is coalesced.
#include "fsmi_common.h"

namespace fsmi {
namespace {

constexpr int kT = 256;

// core/submodule.py:431-435: sum_d d * p_d
__global__ __launch_bounds__(kT) void regression_kernel(const float* __restrict__ prob, float* __restrict__ out,
                                                        int D, int HW, long long P) {
  const long long p = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x;
  if (p >= P) return;
  const long long b = p / HW;
  const int hw = static_cast<int>(p - b * HW);
  const float* src = prob + b * D * HW + hw;
  float acc = 0.f;
  for (int d = 0; d < D; ++d) acc += src[static_cast<size_t>(d) * HW] * static_cast<float>(d);
  out[p] = acc;
}

// core/foundation_stereo.py:218-220: softmax over D, then sum_d d * p_d.
// Same op order as the reference: p_d = exp(x_d - max) / sum, then sum d*p_d.
__global__ __launch_bounds__(kT) void softmax_regression_kernel(const float* __restrict__ logit,
                                                                float* __restrict__ out, int D, int HW, long long P) {
  const long long p = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x;
  if (p >= P) return;
  const long long b = p / HW;
  const int hw = static_cast<int>(p - b * HW);
  const float* src = logit + b * D * HW + hw;
  // pass 1 from HBM with 8 loads in flight per lane; passes 2-3 re-read the column from L1/L2
  constexpr int U = 8;
  float m = -INFINITY;
  int d = 0;
  for (; d + U <= D; d += U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[static_cast<size_t>(d + u) * HW];
#pragma unroll
    for (int u = 0; u < U; ++u) m = fmaxf(m, v[u]);
  }
  for (; d < D; ++d) m = fmaxf(m, src[static_cast<size_t>(d) * HW]);
  float s = 0.f;
  for (d = 0; d + U <= D; d += U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[static_cast<size_t>(d + u) * HW];
#pragma unroll
    for (int u = 0; u < U; ++u) s += expf(v[u] - m);
  }
  for (; d < D; ++d) s += expf(src[static_cast<size_t>(d) * HW] - m);
  float acc = 0.f;
  for (d = 0; d + U <= D; d += U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[static_cast<size_t>(d + u) * HW];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += (expf(v[u] - m) / s) * static_cast<float>(d + u);
  }
  for (; d < D; ++d) acc += (expf(src[static_cast<size_t>(d) * HW] - m) / s) * static_cast<float>(d);
  out[p] = acc;
}

// core/submodule.py:456-468 (+ core/foundation_stereo.py:187-189 when SOFTMAX):
// out[b,y,x] = sum_k w_k(y,x) * scale*disp[b, y/4 + dy_k, x/4 + dx_k] (zero padded)
template <bool SOFTMAX>
__global__ __launch_bounds__(kT) void upsample_kernel(const float* __restrict__ disp, const float* __restrict__ wts,
                                                      float* __restrict__ out, float scale, int h, int w,
                                                      long long P) {
  const long long p = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x;
  if (p >= P) return;
  const int W4 = 4 * w, H4 = 4 * h;
  const long long HW4 = static_cast<long long>(H4) * W4;
  const long long b = p / HW4;
  const int r = static_cast<int>(p - b * HW4);
  const int y = r / W4, x = r - y * W4;
  const int yl = y >> 2, xl = x >> 2;
  const float* wp = wts + b * 9 * HW4 + r;
  const float* dp = disp + b * static_cast<long long>(h) * w;
  float wv[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) wv[k] = wp[k * HW4];
  if (SOFTMAX) {
    float m = wv[0];
#pragma unroll
    for (int k = 1; k < 9; ++k) m = fmaxf(m, wv[k]);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      wv[k] = expf(wv[k] - m);
      s += wv[k];
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) wv[k] = wv[k] / s;
  }
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = yl + k / 3 - 1, xx = xl + k % 3 - 1;
    const float nb = (yy >= 0 && yy < h && xx >= 0 && xx < w) ? dp[yy * w + xx] * scale : 0.f;
    acc += nb * wv[k];
  }
  out[p] = acc;
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// core/update.py:92-93: qin = cat[sigmoid(r) * h, x] for both GRUs
__global__ __launch_bounds__(kT) void gru_reset_kernel(const float* __restrict__ zr_s, const float* __restrict__ zr_l,
                                                       const float* __restrict__ h, const float* __restrict__ x,
                                                       float* __restrict__ qs, float* __restrict__ ql, int Hd, int Cx,
                                                       int HW, long long total) {
  const long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x;
  if (i >= total) return;
  const int Ct = Hd + Cx;
  const int hw = static_cast<int>(i % HW);
  const long long r = i / HW;
  const int c = static_cast<int>(r % Ct);
  const long long b = r / Ct;
  float vs, vl;
  if (c < Hd) {
    const float hv = h[(b * Hd + c) * HW + hw];
    vs = sigm(zr_s[(b * 2 * Hd + Hd + c) * HW + hw]) * hv;
    vl = sigm(zr_l[(b * 2 * Hd + Hd + c) * HW + hw]) * hv;
  } else {
    vs = vl = x[(b * Cx + (c - Hd)) * HW + hw];
  }
  qs[i] = vs;
  ql[i] = vl;
}

// core/update.py:91,94-95,117
__global__ __launch_bounds__(kT) void gru_blend_kernel(const float* __restrict__ zr_s, const float* __restrict__ zr_l,
                                                       const float* __restrict__ q_s, const float* __restrict__ q_l,
                                                       const float* h, const float* __restrict__ att, float* hout,
                                                       int Hd, int HW, long long total) {
  const long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x;
  if (i >= total) return;
  const int hw = static_cast<int>(i % HW);
  const long long r = i / HW;
  const int c = static_cast<int>(r % Hd);
  const long long b = r / Hd;
  const float hv = h[i];
  const float zs = sigm(zr_s[(b * 2 * Hd + c) * HW + hw]);
  const float zl = sigm(zr_l[(b * 2 * Hd + c) * HW + hw]);
  const float hs = (1.f - zs) * hv + zs * tanhf(q_s[i]);
  const float hl = (1.f - zl) * hv + zl * tanhf(q_l[i]);
  const float a = att[b * HW + hw];
  hout[i] = hs * a + hl * (1.f - a);
}

}  // namespace
}  // namespace fsmi

using namespace fsmi;

extern "C" {

int fsmi_disparity_regression(const float* prob, float* out, int B, int D, int H, int W, void* stream) {
  FSMI_CHECK_ARG(prob && out, "fsmi_disparity_regression: null pointer");
  FSMI_CHECK_ARG(B > 0 && D > 0 && H > 0 && W > 0, "fsmi_disparity_regression: bad shape");
  const long long P = static_cast<long long>(B) * H * W;
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_REG, s);
  hipLaunchKernelGGL(regression_kernel, dim3(ceil_div(P, 64)), dim3(64), 0, s, prob, out, D, H * W, P);
  return finish_launch("fsmi_disparity_regression");
}

int fsmi_softmax_regression(const float* logits, float* out, int B, int D, int H, int W, void* stream) {
  FSMI_CHECK_ARG(logits && out, "fsmi_softmax_regression: null pointer");
  FSMI_CHECK_ARG(B > 0 && D > 0 && H > 0 && W > 0, "fsmi_softmax_regression: bad shape");
  const long long P = static_cast<long long>(B) * H * W;
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_REG, s);
  // 64-thread blocks: one pixel per lane, so a 19k-pixel plane still spreads over every CU
  hipLaunchKernelGGL(softmax_regression_kernel, dim3(ceil_div(P, 64)), dim3(64), 0, s, logits, out, D, H * W, P);
  return finish_launch("fsmi_softmax_regression");
}

int fsmi_context_upsample(const float* disp, const float* w, float* out, int B, int h, int w_, void* stream) {
  FSMI_CHECK_ARG(disp && w && out, "fsmi_context_upsample: null pointer");
  FSMI_CHECK_ARG(B > 0 && h > 0 && w_ > 0, "fsmi_context_upsample: bad shape");
  const long long P = static_cast<long long>(B) * 16 * h * w_;
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_UPSAMPLE, s);
  hipLaunchKernelGGL(upsample_kernel<false>, dim3(ceil_div(P, kT)), dim3(kT), 0, s, disp, w, out, 1.0f, h, w_, P);
  return finish_launch("fsmi_context_upsample");
}

int fsmi_softmax_context_upsample(const float* disp, const float* logits, float* out, float scale, int B, int h,
                                  int w_, void* stream) {
  FSMI_CHECK_ARG(disp && logits && out, "fsmi_softmax_context_upsample: null pointer");
  FSMI_CHECK_ARG(B > 0 && h > 0 && w_ > 0, "fsmi_softmax_context_upsample: bad shape");
  const long long P = static_cast<long long>(B) * 16 * h * w_;
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_UPSAMPLE, s);
  hipLaunchKernelGGL(upsample_kernel<true>, dim3(ceil_div(P, kT)), dim3(kT), 0, s, disp, logits, out, scale, h, w_,
                     P);
  return finish_launch("fsmi_softmax_context_upsample");
}

int fsmi_gru_reset(const float* zr_s, const float* zr_l, const float* h, const float* x, float* qin_s, float* qin_l,
                   int B, int Hd, int Cx, int H, int W, void* stream) {
  FSMI_CHECK_ARG(zr_s && zr_l && h && x && qin_s && qin_l, "fsmi_gru_reset: null pointer");
  FSMI_CHECK_ARG(B > 0 && Hd > 0 && Cx > 0 && H > 0 && W > 0, "fsmi_gru_reset: bad shape");
  const long long total = static_cast<long long>(B) * (Hd + Cx) * H * W;
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_GRU_RESET, s);
  hipLaunchKernelGGL(gru_reset_kernel, dim3(ceil_div(total, kT)), dim3(kT), 0, s, zr_s, zr_l, h, x, qin_s, qin_l,
                     Hd, Cx, H * W, total);
  return finish_launch("fsmi_gru_reset");
}

int fsmi_gru_blend(const float* zr_s, const float* zr_l, const float* q_s, const float* q_l, const float* h,
                   const float* att, float* hout, int B, int Hd, int H, int W, void* stream) {
  FSMI_CHECK_ARG(zr_s && zr_l && q_s && q_l && h && att && hout, "fsmi_gru_blend: null pointer");
  FSMI_CHECK_ARG(B > 0 && Hd > 0 && H > 0 && W > 0, "fsmi_gru_blend: bad shape");
  const long long total = static_cast<long long>(B) * Hd * H * W;
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_GRU_BLEND, s);
  hipLaunchKernelGGL(gru_blend_kernel, dim3(ceil_div(total, kT)), dim3(kT), 0, s, zr_s, zr_l, q_s, q_l, h, att, hout,
                     Hd, H * W, total);
  return finish_launch("fsmi_gru_blend");
}

}  // extern "C"
