// Implicit-GEMM 2D convolution on fp32 MFMA for the refinement loop
// (the ConvGRU, motion encoder and heads,
// core/update.py:20-159).
//
// out[b, co0+co, h, w] = epilogue( sum_{tap, ci} Wt[co, ci, tap] * in[b, ci, h+dh, w+dw] )
// as a GEMM  OUT[Cout x P] = W[Cout x K] * X[K x P]  with K = KH*KW*Cin,
// P = B*H*W, NCHW activations (no layout transposes), stride 1, zero
// padding KH/2.  Zero-copy concatenation: the input is up to 4 channel
// segments (each its own NCHW tensor / channel slice), and the output may be
// a channel slice of a wider tensor.  Epilogue: +bias, activation
// (none/ReLU/GELU-erf), *alpha, *gamma[co], +residual -- the elementwise
// passes torch runs after MIOpen (bias add, clamp, scale, residual) fused.
//
// MFMA v_mfma_f32_32x32x2_f32 (exact fp32 fmaf chain):
//   A = weights, lane l: A[m = l&31][k = l>>5]  (LDS As[k][m])
//   B = pixels,  lane l: B[k = l>>5][n = l&31]  (LDS Bs[k][n])
//   D[m][n]: n = l&31 (pixel -> coalesced NCHW stores), m = (r&3)+8(r>>2)+4(l>>5).
// Block = 256 threads (4 waves) computing BM couts x BN pixels; K is walked
// in chunks of KC=16 channels of one tap, double-buffered through LDS with
// the next chunk's global loads in flight during the current chunk's MFMAs.
#include "fsmi_common.h"

namespace fsmi {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int KC = 16;
constexpr int kMaxSeg = 4;

struct ConvArgs {
  const float* seg_ptr[kMaxSeg];
  long long seg_bstride[kMaxSeg];  // batch stride (elements) of each segment tensor
  int seg_end[kMaxSeg];            // cumulative channel end of each segment
  int nseg, Cin;
  const float* wpk;                // [KH*KW*Cin][CoutP] packed, CoutP = roundup(Cout, 4), zero padded
  const float* bias;               // [Cout] or null
  const float* gamma;              // [Cout] or null
  const float* res;                // residual (B, Cout, H, W) slice or null
  long long res_bstride;
  float* out;
  long long out_bstride;
  int co0, Cout, CoutP, B, H, W, act;
  float alpha;
};

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

template <int KH, int KW, int BM, int BN, int WM>
__global__ __launch_bounds__(256) void conv2d_mfma_kernel(ConvArgs a) {
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / (32 * WM), TN = BN / (32 * WN);
  constexpr int PH = KH / 2, PW = KW / 2;
  constexpr int A_PER_T = KC * BM / 4 / 256;  // float4 loads of weights per thread per chunk
  constexpr int B_PER_T = KC * BN / 256;      // scalar loads of pixels per thread per chunk
  static_assert(A_PER_T >= 1 || KC * BM / 4 < 256, "tile");
  static_assert(256 % BN == 0 || BN % 256 == 0, "tile");
  __shared__ __attribute__((aligned(16))) float As[2][KC][BM];
  __shared__ __attribute__((aligned(16))) float Bs[2][KC][BN];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int HW = a.H * a.W;
  const long long P = static_cast<long long>(a.B) * HW;
  const int m0 = blockIdx.y * BM;
  const long long n0 = static_cast<long long>(blockIdx.x) * BN;

  // the pixel this thread stages for the B tile (fixed across chunks; see B_PER_T mapping)
  const int bn = tid % BN;
  const int bk0 = tid / BN;                         // first k row this thread stages
  constexpr int BK_STEP = 256 / BN;                 // k stride between its rows
  const long long pglob = n0 + bn;
  const bool pvalid = pglob < P;
  const int pb = pvalid ? static_cast<int>(pglob / HW) : 0;
  const int phw = pvalid ? static_cast<int>(pglob - static_cast<long long>(pb) * HW) : 0;
  const int ph = phw / a.W, pw = phw - (phw / a.W) * a.W;

  const int nck = (a.Cin + KC - 1) / KC;
  const int nchunks = KH * KW * nck;

  float ra[A_PER_T > 0 ? A_PER_T : 1][4];
  float rb[B_PER_T];

  auto load_chunk = [&](int ch) {
    const int tap = ch / nck;
    const int c0 = (ch - tap * nck) * KC;
    const int dh = tap / KW - PH, dw = tap % KW - PW;
    // weights: rows k = c0..c0+KC of tap, cols m0..m0+BM (float4)
#pragma unroll
    for (int u = 0; u < (A_PER_T > 0 ? A_PER_T : 1); ++u) {
      const int e = tid + 256 * u;
      const int k = e / (BM / 4), m4 = e - k * (BM / 4);
      const int ci = c0 + k, m = m0 + 4 * m4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if ((A_PER_T > 0 || e < KC * BM / 4) && ci < a.Cin && m < a.CoutP)
        v = *reinterpret_cast<const float4*>(a.wpk + (static_cast<size_t>(tap) * a.Cin + ci) * a.CoutP + m);
      ra[u][0] = v.x; ra[u][1] = v.y; ra[u][2] = v.z; ra[u][3] = v.w;
    }
    // pixels: channel rows k = bk0 + BK_STEP*u of this thread's pixel, shifted by the tap
    const int hh = ph + dh, ww = pw + dw;
    const bool inb = pvalid && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
    const int off = hh * a.W + ww;
#pragma unroll
    for (int u = 0; u < B_PER_T; ++u) {
      const int ci = c0 + bk0 + BK_STEP * u;
      float v = 0.f;
      if (inb && ci < a.Cin) {
        int s = 0, base = 0;
#pragma unroll
        for (int q = 0; q < kMaxSeg - 1; ++q)
          if (q < a.nseg - 1 && ci >= a.seg_end[q]) { s = q + 1; base = a.seg_end[q]; }
        v = a.seg_ptr[s][pb * a.seg_bstride[s] + static_cast<long long>(ci - base) * HW + off];
      }
      rb[u] = v;
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int u = 0; u < (A_PER_T > 0 ? A_PER_T : 1); ++u) {
      const int e = tid + 256 * u;
      if (A_PER_T > 0 || e < KC * BM / 4) {
        const int k = e / (BM / 4), m4 = e - k * (BM / 4);
        *reinterpret_cast<float4*>(&As[buf][k][4 * m4]) = make_float4(ra[u][0], ra[u][1], ra[u][2], ra[u][3]);
      }
    }
#pragma unroll
    for (int u = 0; u < B_PER_T; ++u) Bs[buf][bk0 + BK_STEP * u][bn] = rb[u];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int kl = lane >> 5, il = lane & 31;
  load_chunk(0);
  store_chunk(0);
  __syncthreads();
  for (int ch = 0; ch < nchunks; ++ch) {
    const int buf = ch & 1;
    if (ch + 1 < nchunks) load_chunk(ch + 1);
#pragma unroll
    for (int kk = 0; kk < KC; kk += 2) {
      float av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) av[i] = As[buf][kk + kl][(wm * TM + i) * 32 + il];
#pragma unroll
      for (int j = 0; j < TN; ++j) bv[j] = Bs[buf][kk + kl][(wn * TN + j) * 32 + il];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (ch + 1 < nchunks) store_chunk(buf ^ 1);
    __syncthreads();
  }

  // epilogue
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const long long p = n0 + (wn * TN + j) * 32 + il;
    if (p >= P) continue;
    const int b = static_cast<int>(p / HW);
    const int hw = static_cast<int>(p - static_cast<long long>(b) * HW);
    float* ob = a.out + b * a.out_bstride + hw;
    const float* rbp = a.res ? a.res + b * a.res_bstride + hw : nullptr;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        if (co >= a.Cout) continue;
        float v = acc[i][j][r];
        if (a.bias) v += a.bias[co];
        if (a.act == 1) v = fmaxf(v, 0.f);
        else if (a.act == 2) v = gelu_erf(v);
        v *= a.alpha;
        if (a.gamma) v *= a.gamma[co];
        if (rbp) v += rbp[static_cast<size_t>(co) * HW];
        ob[static_cast<size_t>(a.co0 + co) * HW] = v;
      }
    }
  }
}

template <int KH, int KW>
int launch_cfg(const ConvArgs& a, int cfg, hipStream_t s) {
  const long long P = static_cast<long long>(a.B) * a.H * a.W;
  switch (cfg) {
    case 0: {  // 128 x 128, waves 2 x 2
      dim3 grid(ceil_div(P, 128), ceil_div(a.Cout, 128));
      hipLaunchKernelGGL((conv2d_mfma_kernel<KH, KW, 128, 128, 2>), grid, dim3(256), 0, s, a);
      break;
    }
    case 1: {  // 64 x 128, waves 1 x 4
      dim3 grid(ceil_div(P, 128), ceil_div(a.Cout, 64));
      hipLaunchKernelGGL((conv2d_mfma_kernel<KH, KW, 64, 128, 1>), grid, dim3(256), 0, s, a);
      break;
    }
    case 2: {  // 32 x 128, waves 1 x 4
      dim3 grid(ceil_div(P, 128), ceil_div(a.Cout, 32));
      hipLaunchKernelGGL((conv2d_mfma_kernel<KH, KW, 32, 128, 1>), grid, dim3(256), 0, s, a);
      break;
    }
    default: {  // 128 x 64, waves 2 x 2 (few pixels)
      dim3 grid(ceil_div(P, 64), ceil_div(a.Cout, 128));
      hipLaunchKernelGGL((conv2d_mfma_kernel<KH, KW, 128, 64, 2>), grid, dim3(256), 0, s, a);
      break;
    }
  }
  return finish_launch("fsmi_conv2d");
}

// pick the largest tile that still puts >= ~2 blocks on every CU
int pick_cfg(long long P, int Cout) {
  auto blocks = [&](int bm, int bn) { return ceil_div(P, bn) * static_cast<long long>(ceil_div(Cout, bm)); };
  if (Cout > 64 && blocks(128, 128) >= 480) return 0;
  if (Cout > 64 && blocks(128, 64) >= 480) return 3;
  if (Cout > 32) return 1;
  return 2;
}

}  // namespace
}  // namespace fsmi

using namespace fsmi;

extern "C" int fsmi_conv2d(const float* const* seg_ptr, const int* seg_ch, const int* seg_ctot, int nseg,
                           const float* wpk, const float* bias, const float* gamma, const float* res, int res_ctot,
                           float* out, int out_ctot, int co0, int B, int Cout, int KH, int KW, int H, int W, int act,
                           float alpha, int cfg, void* stream) {
  FSMI_CHECK_ARG(seg_ptr && seg_ch && seg_ctot && wpk && out, "fsmi_conv2d: null pointer");
  FSMI_CHECK_ARG(nseg >= 1 && nseg <= kMaxSeg, "fsmi_conv2d: 1..%d input segments, got %d", kMaxSeg, nseg);
  FSMI_CHECK_ARG(B > 0 && Cout > 0 && H > 0 && W > 0, "fsmi_conv2d: bad shape");
  FSMI_CHECK_ARG((KH == 1 && KW == 1) || (KH == 3 && KW == 3) || (KH == 7 && KW == 7),
                 "fsmi_conv2d: kernel %dx%d unsupported (1x1, 3x3, 7x7)", KH, KW);
  FSMI_CHECK_ARG(act >= 0 && act <= 2, "fsmi_conv2d: act %d", act);
  FSMI_CHECK_ARG(co0 >= 0 && co0 + Cout <= out_ctot, "fsmi_conv2d: output slice [%d,%d) outside %d channels", co0,
                 co0 + Cout, out_ctot);
  ConvArgs a{};
  int cin = 0;
  const long long HW = static_cast<long long>(H) * W;
  for (int i = 0; i < nseg; ++i) {
    FSMI_CHECK_ARG(seg_ptr[i] && seg_ch[i] > 0 && seg_ctot[i] >= seg_ch[i], "fsmi_conv2d: bad segment %d", i);
    a.seg_ptr[i] = seg_ptr[i];
    a.seg_bstride[i] = static_cast<long long>(seg_ctot[i]) * HW;
    cin += seg_ch[i];
    a.seg_end[i] = cin;
  }
  a.nseg = nseg;
  a.Cin = cin;
  a.wpk = wpk;
  a.bias = bias;
  a.gamma = gamma;
  a.res = res;
  a.res_bstride = static_cast<long long>(res_ctot) * HW;
  a.out = out;
  a.out_bstride = static_cast<long long>(out_ctot) * HW;
  a.co0 = co0;
  a.Cout = Cout;
  a.CoutP = (Cout + 3) / 4 * 4;
  a.B = B;
  a.H = H;
  a.W = W;
  a.act = act;
  a.alpha = alpha;
  if (cfg < 0) cfg = pick_cfg(static_cast<long long>(B) * HW, Cout);
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_CONV2D, s);
  if (KH == 1) return launch_cfg<1, 1>(a, cfg, s);
  if (KH == 3) return launch_cfg<3, 3>(a, cfg, s);
  return launch_cfg<7, 7>(a, cfg, s);
}
