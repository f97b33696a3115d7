// Direct 3D convolution for the few-output-channel layers of the 3D filtering
// (SURVEY §8a row a3): the classifier's Conv3d(14 -> 1, k=7, pad 3)
// (core/foundation_stereo.py:175), which MIOpen runs at ~1 TFLOP/s on gfx950.
//
// Layout: (B, Cin, D, H, W) fp32 in, (B, Cout, D, H, W) out, weight (Cout, Cin, KS, KS, KS).
// Block = 256 threads -> output tile 8(d) x 8(h) x 32(w); thread = 4 consecutive w of one h at two
// consecutive depths (2 dz, 2 dz + 1: dz = wave index, so every (kd, kh) is wave-uniform and the
// weights come through scalar loads as SGPR operands).  Per input channel the (8+KS-1) x (8+KS-1) x
// (32+KS-1) halo tile is staged in LDS (zero padding baked in); the next channel's halo is loaded
// into registers while this one is consumed.  A wave walks its KS+1 input planes once: each
// (plane, kh) row of 4+KS-1 LDS reads feeds both of its output depths (2 x 4 x KS FMAs; the 4-deep
// tile of round 2 read every row once per output depth).
// FP32 VALU: 2*Cin*KS^3*COUT flops per output, ~1 flop/B -> compute-bound.
#include "fsmi_common.h"

namespace fsmi {
namespace {

constexpr int kTD = 8, kTH = 8, kTW = 32;

template <int KS, int COUT>
__global__ __launch_bounds__(256) void conv3d_direct_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                                                            const float* __restrict__ bias, float* __restrict__ out,
                                                            int Cin, int D, int H, int W, int nTd, int nTh, int nTw) {
  constexpr int P = KS / 2;
  constexpr int ID = kTD + KS - 1, IH = kTH + KS - 1, IW = kTW + KS - 1;
  constexpr int NT = ID * IH * IW;
  constexpr int PER = (NT + 255) / 256;           // staged elements per thread
  __shared__ float tile[NT];
  // XCD-aware order, depth fastest: an XCD's contiguous run of tiles is whole depth columns of a few
  // (h, w) tiles, so the KS - 1 halo planes two depth tiles share and the halo rows of h neighbours
  // are hits in that XCD's L2 (w fastest re-fetched the depth halos: 1.9x the input per launch)
  int bid = static_cast<int>(xcd_remap(blockIdx.x, gridDim.x));
  const int td = bid % nTd; bid /= nTd;
  const int tw = bid % nTw; bid /= nTw;
  const int th = bid % nTh;
  const int b = bid / nTh;
  const int d0 = td * kTD, h0 = th * kTH, w0 = tw * kTW;
  const int tid = threadIdx.x;
  const int wq = tid & 7, hy = (tid >> 3) & 7;
  const int dz = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave index: output depths 2 dz, 2 dz + 1
  const size_t plane = static_cast<size_t>(H) * W;
  const size_t vol = static_cast<size_t>(D) * plane;

  // per-thread staging slots: offset into a channel's volume (or -1 for the zero padding)
  int off[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = tid + i * 256;
    const int iw = e % IW;
    const int r = e / IW;
    const int ih = r % IH, id = r / IH;
    const int dd = d0 + id - P, hh = h0 + ih - P, ww = w0 + iw - P;
    const bool ok = e < NT && dd >= 0 && dd < D && hh >= 0 && hh < H && ww >= 0 && ww < W;
    off[i] = ok ? (dd * H + hh) * W + ww : -1;      // < 2^31: the host checks D * H * W
  }
  float nxt[PER];
  auto fetch = [&](int c) {
    const float* xc = x + (static_cast<size_t>(b) * Cin + c) * vol;
#pragma unroll
    for (int i = 0; i < PER; ++i) nxt[i] = off[i] >= 0 ? xc[off[i]] : 0.f;
  };

  float acc[COUT][2][4];
#pragma unroll
  for (int o = 0; o < COUT; ++o)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[o][t][j] = 0.f;

  fetch(0);
  for (int c = 0; c < Cin; ++c) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (i < PER - 1 || tid + i * 256 < NT) tile[tid + i * 256] = nxt[i];
    __syncthreads();
    if (c + 1 < Cin) fetch(c + 1);                  // in flight under this channel's FMAs
    const float* wc = wt + static_cast<size_t>(c) * KS * KS * KS;
#pragma unroll 1
    for (int p = 0; p <= KS; ++p) {                 // input plane 2 dz + p of the tile
#pragma unroll
      for (int kh = 0; kh < KS; ++kh) {
        const float* row = tile + ((2 * dz + p) * IH + (hy + kh)) * IW + wq * 4;
        float v[4 + KS - 1];
#pragma unroll
        for (int i = 0; i < 4 + KS - 1; ++i) v[i] = row[i];
#pragma unroll
        for (int o = 0; o < COUT; ++o) {
          const float* wo = wc + static_cast<size_t>(o) * Cin * KS * KS * KS;
#pragma unroll
          for (int t = 0; t < 2; ++t) {             // output depth 2 dz + t reads this plane at kd = p - t
            const int kd = p - t;
            if (kd < 0 || kd >= KS) continue;
            const float* wr = wo + (kd * KS + kh) * KS;
#pragma unroll
            for (int kw = 0; kw < KS; ++kw) {
              const float wv = wr[kw];
#pragma unroll
              for (int j = 0; j < 4; ++j) acc[o][t][j] += v[j + kw] * wv;
            }
          }
        }
      }
    }
  }
  const int h = h0 + hy;
  if (h >= H) return;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int d = d0 + 2 * dz + t;
    if (d >= D) continue;
#pragma unroll
    for (int o = 0; o < COUT; ++o) {
      const float bo = bias ? bias[o] : 0.f;
      float* dst = out + (static_cast<size_t>(b) * COUT + o) * vol + static_cast<size_t>(d) * plane +
                   static_cast<size_t>(h) * W;
      const int w = w0 + wq * 4;
      if ((W & 3) == 0 && w + 3 < W) {
        *reinterpret_cast<float4*>(dst + w) =
            make_float4(acc[o][t][0] + bo, acc[o][t][1] + bo, acc[o][t][2] + bo, acc[o][t][3] + bo);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (w + j < W) dst[w + j] = acc[o][t][j] + bo;
      }
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
  FSMI_CHECK_ARG(static_cast<long long>(D) * H * W < (1ll << 31), "fsmi_conv3d_direct: volume too large");
  FSMI_CHECK_ARG((KS == 7 && Cout == 1) || (KS == 3 && Cout == 1),
                 "fsmi_conv3d_direct: supports (KS, Cout) in {(7,1), (3,1)}, got (%d,%d)", KS, Cout);
  const int nTd = (D + kTD - 1) / kTD, nTh = (H + kTH - 1) / kTH, nTw = (W + kTW - 1) / kTW;
  const unsigned grid = static_cast<unsigned>(B) * nTd * nTh * nTw;   // (b, h tile, w tile, d tile), d fastest
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
