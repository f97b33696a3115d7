// Direct 3D convolution for the few-output-channel layers of the 3D filtering
// (SURVEY §8a row a3): the classifier's Conv3d(14 -> 1, k=7, pad 3)
// (core/foundation_stereo.py:175), which MIOpen runs at ~1 TFLOP/s on gfx950.
//
// Layout: (B, Cin, D, H, W) fp32 in, (B, Cout, D, H, W) out, weight (Cout, Cin, KS, KS, KS).
// Block = 256 threads -> output tile 4(d) x 8(h) x 32(w); thread = 4 consecutive
// w of one (d, h) for all COUT output channels.  Per input channel the
// (4+KS-1)x(8+KS-1)x(32+KS-1) halo tile is staged in LDS (zero padding baked
// in); each (kd, kh) row contributes 4 x KS x COUT FMAs from 4+KS-1 LDS reads.
// Weights are wave-uniform, so they come through scalar loads (SGPR operands).
// FP32 VALU: 2*Cin*KS^3*COUT flops per output, ~1 flop/B -> compute-bound.
#include "fsmi_common.h"

namespace fsmi {
namespace {

constexpr int kTD = 4, kTH = 8, kTW = 32;

template <int KS, int COUT>
__global__ __launch_bounds__(256) void conv3d_direct_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                                                            const float* __restrict__ bias, float* __restrict__ out,
                                                            int Cin, int D, int H, int W, int nTd, int nTh, int nTw) {
  constexpr int P = KS / 2;
  constexpr int ID = kTD + KS - 1, IH = kTH + KS - 1, IW = kTW + KS - 1;
  __shared__ float tile[ID * IH * IW];
  // XCD-aware order: consecutive tiles (w fastest, then h, then d) on one XCD, so the halos a tile
  // shares with its neighbours are L2 hits there (the round-robin default put every neighbour on
  // another XCD's L2: 7.3x the input fetched per launch)
  int bid = static_cast<int>(xcd_remap(blockIdx.x, gridDim.x));
  const int tw = bid % nTw; bid /= nTw;
  const int th = bid % nTh; bid /= nTh;
  const int td = bid % nTd;
  const int b = bid / nTd;
  const int d0 = td * kTD, h0 = th * kTH, w0 = tw * kTW;
  const int tid = threadIdx.x;
  const int wq = tid & 7, hy = (tid >> 3) & 7, dz = tid >> 6;  // 8 x 8 x 4
  const size_t plane = static_cast<size_t>(H) * W;
  const size_t vol = static_cast<size_t>(D) * plane;

  float acc[COUT][4];
#pragma unroll
  for (int o = 0; o < COUT; ++o)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[o][j] = 0.f;

  for (int c = 0; c < Cin; ++c) {
    const float* xc = x + (static_cast<size_t>(b) * Cin + c) * vol;
    __syncthreads();
    for (int e = tid; e < ID * IH * IW; e += 256) {
      const int iw = e % IW;
      const int r = e / IW;
      const int ih = r % IH, id = r / IH;
      const int dd = d0 + id - P, hh = h0 + ih - P, ww = w0 + iw - P;
      const bool ok = dd >= 0 && dd < D && hh >= 0 && hh < H && ww >= 0 && ww < W;
      tile[e] = ok ? xc[static_cast<size_t>(dd) * plane + static_cast<size_t>(hh) * W + ww] : 0.f;
    }
    __syncthreads();
    const float* wc = wt + static_cast<size_t>(c) * KS * KS * KS;
#pragma unroll 1
    for (int kd = 0; kd < KS; ++kd) {
#pragma unroll
      for (int kh = 0; kh < KS; ++kh) {
        const float* row = tile + ((dz + kd) * IH + (hy + kh)) * IW + wq * 4;
        float v[4 + KS - 1];
#pragma unroll
        for (int i = 0; i < 4 + KS - 1; ++i) v[i] = row[i];
#pragma unroll
        for (int o = 0; o < COUT; ++o) {
          const float* wr = wc + static_cast<size_t>(o) * Cin * KS * KS * KS + (kd * KS + kh) * KS;
#pragma unroll
          for (int kw = 0; kw < KS; ++kw) {
            const float wv = wr[kw];
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[o][j] += v[j + kw] * wv;
          }
        }
      }
    }
  }
  const int d = d0 + dz, h = h0 + hy;
  if (d >= D || h >= H) return;
#pragma unroll
  for (int o = 0; o < COUT; ++o) {
    const float bo = bias ? bias[o] : 0.f;
    float* dst = out + (static_cast<size_t>(b) * COUT + o) * vol + static_cast<size_t>(d) * plane +
                 static_cast<size_t>(h) * W;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int w = w0 + wq * 4 + j;
      if (w < W) dst[w] = acc[o][j] + bo;
    }
  }
}

}  // namespace
}  // namespace fsmi

using namespace fsmi;

extern "C" int fsmi_conv3d_direct(const float* x, const float* w, const float* bias, float* out, int B, int Cin,
                                  int Cout, int KS, int D, int H, int W, void* stream) {
  FSMI_CHECK_ARG(x && w && out, "fsmi_conv3d_direct: null pointer");
  FSMI_CHECK_ARG(B > 0 && Cin > 0 && D > 0 && H > 0 && W > 0, "fsmi_conv3d_direct: bad shape");
  FSMI_CHECK_ARG((KS == 7 && Cout == 1) || (KS == 3 && Cout == 1),
                 "fsmi_conv3d_direct: supports (KS, Cout) in {(7,1), (3,1)}, got (%d,%d)", KS, Cout);
  const int nTd = (D + kTD - 1) / kTD, nTh = (H + kTH - 1) / kTH, nTw = (W + kTW - 1) / kTW;
  const unsigned grid = static_cast<unsigned>(B) * nTd * nTh * nTw;
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_CONV3D, s);
  if (KS == 7)
    hipLaunchKernelGGL((conv3d_direct_kernel<7, 1>), dim3(grid), dim3(256), 0, s, x, w, bias, out, Cin, D, H, W, nTd,
                       nTh, nTw);
  else
    hipLaunchKernelGGL((conv3d_direct_kernel<3, 1>), dim3(grid), dim3(256), 0, s, x, w, bias, out, Cin, D, H, W, nTd,
                       nTh, nTw);
  return finish_launch("fsmi_conv3d_direct");
}
