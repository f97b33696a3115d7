// Disparity transformer of the hourglass: the path
//   conv_patch (depthwise Conv3d k4 s4 + BatchNorm3d, core/foundation_stereo.py:85-88)
//   -> CostVolumeDisparityAttention (core/submodule.py:506-528: sin/cos PE + post-norm
//      encoder layers, FlashMultiheadAttention core/submodule.py:198-229 whose
//      flash_attn_func call is plain non-causal softmax(QK^T/sqrt(hd))V)
//   -> F.interpolate(scale_factor=4, trilinear, align_corners=False) + add
//      (core/foundation_stereo.py:117-120)
// as three gfx950 kernels.  The reference runs ~40 small launches here (4 layers x
// {3 projections, SDPA, out proj, 2 LayerNorms, 2 FFN linears, GELU, adds}) on sequences of
// only D4/4 <= 20 tokens x 28 channels; all of it is latency, not bandwidth or FLOPs.
//
// dt_encoder_kernel: one thread per token, a block holds S = 64 / L whole sequences (one
// wave).  The token's 28 features live in VGPRs; every weight index is a compile-time constant
// after unrolling and the layer base is uniform, so weights arrive as scalar loads (SGPR
// operands of v_fma) -- no LDS staging of weights.  K and V of the block's tokens go through
// LDS for the attention; softmax is online (running max / denominator) over the L keys.
#include "fsmi_common.h"

namespace fsmi {
namespace {

constexpr int kDtC = 28, kDtHeads = 4, kDtFF = 28;
constexpr int kDtMaxL = 64;
// per-layer packed parameters (nn.Linear weights are (out, in) row-major)
constexpr int kOffQ = 0, kOffK = kOffQ + kDtC * kDtC + kDtC, kOffV = kOffK + kDtC * kDtC + kDtC,
              kOffO = kOffV + kDtC * kDtC + kDtC, kOffLn1 = kOffO + kDtC * kDtC + kDtC,
              kOffF1 = kOffLn1 + 2 * kDtC, kOffF2 = kOffF1 + kDtFF * kDtC + kDtFF,
              kOffLn2 = kOffF2 + kDtC * kDtFF + kDtC, kLayerFloats = kOffLn2 + 2 * kDtC;

template <int NO, int NI>
__device__ __forceinline__ void linear(const float* __restrict__ p, const float (&x)[NI], float (&y)[NO]) {
#pragma unroll
  for (int o = 0; o < NO; ++o) {
    float s = p[NO * NI + o];                                 // bias after the weight block
#pragma unroll
    for (int i = 0; i < NI; ++i) s = fmaf(p[o * NI + i], x[i], s);
    y[o] = s;
  }
}

// x <- LayerNorm(x + r) with biased variance (nn.LayerNorm), weight / bias at p, p + C
template <int C>
__device__ __forceinline__ void add_layernorm(const float* __restrict__ p, float (&x)[C], const float (&r)[C],
                                              float eps) {
  float mean = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    x[c] += r[c];
    mean += x[c];
  }
  mean *= 1.f / C;
  float var = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float d = x[c] - mean;
    var = fmaf(d, d, var);
  }
  const float inv = 1.f / sqrtf(var * (1.f / C) + eps);
#pragma unroll
  for (int c = 0; c < C; ++c) x[c] = fmaf((x[c] - mean) * inv, p[c], p[C + c]);
}

__global__ __launch_bounds__(64) void dt_encoder_kernel(const float* __restrict__ x, float* __restrict__ out,
                                                        const float* __restrict__ params,
                                                        const float* __restrict__ pe, int B, int L, int HW,
                                                        int nlayers, float eps) {
  constexpr int C = kDtC, HD = kDtC / kDtHeads;
  __shared__ float kv[kDtMaxL][2 * C + 1];                   // +1: rows of different tokens spread banks
  const int S = 64 / L;                                      // whole sequences per block
  const int tid = threadIdx.x;
  const int s = tid % S, l = tid / S;                        // consecutive threads: consecutive pixels
  const long long seq = static_cast<long long>(blockIdx.x) * S + s;
  const bool live = l < L && seq < static_cast<long long>(B) * HW;
  const int b = live ? static_cast<int>(seq / HW) : 0;
  const int hw = live ? static_cast<int>(seq % HW) : 0;
  const long long cstride = static_cast<long long>(L) * HW;
  const float* xp = x + static_cast<long long>(b) * C * cstride + static_cast<long long>(l) * HW + hw;

  float t[C];
#pragma unroll
  for (int c = 0; c < C; ++c) t[c] = live ? xp[c * cstride] + pe[(live ? l : 0) * C + c] : 0.f;

  const float scale = 1.f / sqrtf(static_cast<float>(HD));
  for (int layer = 0; layer < nlayers; ++layer) {
    const float* __restrict__ p = params + static_cast<long long>(layer) * kLayerFloats;
    float q[C], r[C];
    linear<C, C>(p + kOffK, t, q);                           // K, V of this token into LDS
    linear<C, C>(p + kOffV, t, r);
    __syncthreads();                                         // previous layer's readers are done
#pragma unroll
    for (int c = 0; c < C; ++c) {
      kv[tid][c] = q[c];
      kv[tid][C + c] = r[c];
    }
    linear<C, C>(p + kOffQ, t, q);
    __syncthreads();
    // attention over the L tokens of this sequence (token j of it is thread j * S + s)
#pragma unroll
    for (int h = 0; h < kDtHeads; ++h) {
      float m = -INFINITY, den = 0.f, acc[HD];
#pragma unroll
      for (int e = 0; e < HD; ++e) acc[e] = 0.f;
      for (int j = 0; j < L; ++j) {
        const float* kr = kv[j * S + s];
        float sc = 0.f;
#pragma unroll
        for (int e = 0; e < HD; ++e) sc = fmaf(q[h * HD + e], kr[h * HD + e], sc);
        sc *= scale;
        const float mn = fmaxf(m, sc);
        const float corr = expf(m - mn), w = expf(sc - mn);
        den = fmaf(den, corr, w);
#pragma unroll
        for (int e = 0; e < HD; ++e) acc[e] = fmaf(acc[e], corr, w * kr[C + h * HD + e]);
        m = mn;
      }
      const float inv = 1.f / den;
#pragma unroll
      for (int e = 0; e < HD; ++e) r[h * HD + e] = acc[e] * inv;
    }
    linear<C, C>(p + kOffO, r, q);
    add_layernorm<C>(p + kOffLn1, t, q, eps);
    float f[kDtFF];
    linear<kDtFF, C>(p + kOffF1, t, f);
#pragma unroll
    for (int i = 0; i < kDtFF; ++i) f[i] = 0.5f * f[i] * (1.f + erff(f[i] * 0.70710678118654752f));   // exact GELU
    linear<C, kDtFF>(p + kOffF2, f, q);
    add_layernorm<C>(p + kOffLn2, t, q, eps);
  }
  if (live) {
    float* op = out + static_cast<long long>(b) * C * cstride + static_cast<long long>(l) * HW + hw;
#pragma unroll
    for (int c = 0; c < C; ++c) op[c * cstride] = t[c];
  }
}

// Depthwise Conv3d k4 s4 (no padding) with bias and eval BatchNorm folded into (scale, shift):
// out[b,c,d,h,w] = scale[c] * sum_{kd,kh,kw} w[c,kd,kh,kw] x[b,c,4d+kd,4h+kh,4w+kw] + shift[c].
// One thread per output voxel; each of its 16 input rows is one float4.
__global__ __launch_bounds__(256) void dt_patch_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, float* __restrict__ out,
                                                       int C, int Do, int Ho, int Wo, long long n) {
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const int wo = static_cast<int>(i % Wo);
  long long r = i / Wo;
  const int ho = static_cast<int>(r % Ho);
  r /= Ho;
  const int d = static_cast<int>(r % Do);
  const long long bc = r / Do;                                // b * C + c
  const int c = static_cast<int>(bc % C);
  const int Wi = 4 * Wo, Hi = 4 * Ho;
  const float* xp = x + ((bc * 4 * Do + 4 * d) * Hi + 4 * ho) * static_cast<long long>(Wi) + 4 * wo;
  const float* wp = w + c * 64;
  float s = 0.f;
#pragma unroll
  for (int kd = 0; kd < 4; ++kd)
#pragma unroll
    for (int kh = 0; kh < 4; ++kh) {
      const float4 v = *reinterpret_cast<const float4*>(xp + (static_cast<long long>(kd) * Hi + kh) * Wi);
      const float* ww = wp + kd * 16 + kh * 4;
      s = fmaf(ww[0], v.x, s);
      s = fmaf(ww[1], v.y, s);
      s = fmaf(ww[2], v.z, s);
      s = fmaf(ww[3], v.w, s);
    }
  out[i] = fmaf(s, scale[c], shift[c]);
}

// vol[b,c,z,y,x] += trilinear(t)(z,y,x), scale 4, align_corners=False (PyTorch's source index
// (o + 0.5) / 4 - 0.5 clamped at 0; the upper neighbour clamped to the last sample).
// One thread per 4 consecutive x outputs (one float4 of vol).
__device__ __forceinline__ void up4_coord(int o, int n, int& i0, int& i1, float& l1) {
  const float src = fmaxf((o + 0.5f) * 0.25f - 0.5f, 0.f);
  i0 = static_cast<int>(src);
  i1 = i0 + (i0 < n - 1 ? 1 : 0);
  l1 = src - static_cast<float>(i0);
}

__global__ __launch_bounds__(256) void dt_upsample4_add_kernel(const float* __restrict__ t, float* __restrict__ vol,
                                                               int D, int H, int W, long long n4) {
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n4) return;
  const int W4 = 4 * W, H4 = 4 * H, D4 = 4 * D;
  const int xq = static_cast<int>(i % W);                     // float4 index along x: outputs 4xq..4xq+3
  long long r = i / W;
  const int y = static_cast<int>(r % H4);
  r /= H4;
  const int z = static_cast<int>(r % D4);
  const long long bc = r / D4;
  int z0, z1, y0, y1;
  float lz, ly;
  up4_coord(z, D, z0, z1, lz);
  up4_coord(y, H, y0, y1, ly);
  const float* tp = t + bc * D * H * W;
  const float* p00 = tp + (static_cast<long long>(z0) * H + y0) * W;
  const float* p01 = tp + (static_cast<long long>(z0) * H + y1) * W;
  const float* p10 = tp + (static_cast<long long>(z1) * H + y0) * W;
  const float* p11 = tp + (static_cast<long long>(z1) * H + y1) * W;
  const float w00 = (1.f - lz) * (1.f - ly), w01 = (1.f - lz) * ly, w10 = lz * (1.f - ly), w11 = lz * ly;
  float4* vp = reinterpret_cast<float4*>(vol + ((bc * D4 + z) * H4 + y) * static_cast<long long>(W4)) + xq;
  float4 v = *vp;
  float o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int x0, x1;
    float lx;
    up4_coord(4 * xq + k, W, x0, x1, lx);
    // same association as PyTorch's upsample_trilinear3d: t0 * (h0 * (w0 a + w1 b) + ...) form
    const float a0 = (1.f - lx) * p00[x0] + lx * p00[x1];
    const float a1 = (1.f - lx) * p01[x0] + lx * p01[x1];
    const float b0 = (1.f - lx) * p10[x0] + lx * p10[x1];
    const float b1 = (1.f - lx) * p11[x0] + lx * p11[x1];
    o[k] = w00 * a0 + w01 * a1 + w10 * b0 + w11 * b1;
  }
  v.x += o[0];
  v.y += o[1];
  v.z += o[2];
  v.w += o[3];
  *vp = v;
}

}  // namespace
}  // namespace fsmi

using namespace fsmi;

extern "C" int fsmi_dt_layer_floats(void) { return kLayerFloats; }

extern "C" int fsmi_disparity_transformer(const float* x, float* out, const float* params, const float* pe, int B,
                                          int C, int L, int HW, int nheads, int ffdim, int nlayers, float eps,
                                          void* stream) {
  FSMI_CHECK_ARG(x && out && params && pe, "fsmi_disparity_transformer: null pointer");
  FSMI_CHECK_ARG(C == kDtC && nheads == kDtHeads && ffdim == kDtFF,
                 "fsmi_disparity_transformer: built for C=%d, %d heads, FFN %d (got %d, %d, %d)", kDtC, kDtHeads,
                 kDtFF, C, nheads, ffdim);
  FSMI_CHECK_ARG(L >= 1 && L <= kDtMaxL, "fsmi_disparity_transformer: sequence length %d (1..%d)", L, kDtMaxL);
  FSMI_CHECK_ARG(B >= 1 && HW >= 1 && nlayers >= 0, "fsmi_disparity_transformer: bad shape");
  hipStream_t s = as_stream(stream);
  LaunchTimer tm(FSMI_K_DT, s);
  const int S = 64 / L;
  const long long nseq = static_cast<long long>(B) * HW;
  hipLaunchKernelGGL(dt_encoder_kernel, dim3(ceil_div(nseq, S)), dim3(64), 0, s, x, out, params, pe, B, L, HW,
                     nlayers, eps);
  return finish_launch("fsmi_disparity_transformer");
}

extern "C" int fsmi_dt_patch_embed(const float* x, const float* w, const float* scale, const float* shift, float* out,
                                   int B, int C, int D, int H, int W, void* stream) {
  FSMI_CHECK_ARG(x && w && scale && shift && out, "fsmi_dt_patch_embed: null pointer");
  FSMI_CHECK_ARG(B > 0 && C > 0 && D >= 4 && H >= 4 && W >= 4, "fsmi_dt_patch_embed: bad shape");
  // the kernel strides the input by 4*Do planes / 4*Ho rows: a floor (as Conv3d k4 s4 does) would
  // need the true D / H as strides, so ragged sizes are refused instead of silently misread
  FSMI_CHECK_ARG(D % 4 == 0 && H % 4 == 0 && W % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0,
                 "fsmi_dt_patch_embed: D, H, W %% 4 == 0 and a 16-B aligned input required (D=%d H=%d W=%d)", D, H,
                 W);
  hipStream_t s = as_stream(stream);
  LaunchTimer tm(FSMI_K_DT, s);
  const int Do = D / 4, Ho = H / 4, Wo = W / 4;
  const long long n = static_cast<long long>(B) * C * Do * Ho * Wo;
  if (n == 0) return FSMI_OK;
  hipLaunchKernelGGL(dt_patch_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, s, x, w, scale, shift, out, C, Do, Ho,
                     Wo, n);
  return finish_launch("fsmi_dt_patch_embed");
}

extern "C" int fsmi_upsample4_add(const float* t, float* vol, int B, int C, int D, int H, int W, void* stream) {
  FSMI_CHECK_ARG(t && vol, "fsmi_upsample4_add: null pointer");
  FSMI_CHECK_ARG(B > 0 && C > 0 && D > 0 && H > 0 && W > 0, "fsmi_upsample4_add: bad shape");
  FSMI_CHECK_ARG(reinterpret_cast<uintptr_t>(vol) % 16 == 0, "fsmi_upsample4_add: volume must be 16-B aligned");
  hipStream_t s = as_stream(stream);
  LaunchTimer tm(FSMI_K_DT, s);
  const long long n4 = static_cast<long long>(B) * C * (4LL * D) * (4LL * H) * W;   // float4s of vol
  hipLaunchKernelGGL(dt_upsample4_add_kernel, dim3(ceil_div(n4, 256)), dim3(256), 0, s, t, vol, D, H, W, n4);
  return finish_launch("fsmi_upsample4_add");
}
