// Split-precision ("3 x fp16") implicit-GEMM 2D convolution on the fp16 MFMA.
//
// Each fp32 operand is carried as two fp16 halves, x = hi + lo with
// hi = fp16(x), lo = fp16(x - hi) (22 significant bits together), and each
// product as  a_hi*b_hi + a_hi*b_lo + a_lo*b_hi  (the a_lo*b_lo term is below
// 2^-22 relative) accumulated in fp32 by v_mfma_f32_32x32x16_f16 -- 3 MFMAs at
// 16x the fp32-MFMA rate, i.e. ~5x fp32 throughput at ~fp32 accuracy.
// Measured end to end (emulated on the CPU oracle, cfg2 / 32 iterations):
// max |dd| = 1.4e-4 px vs the fp32 reference (pure fp16: 5e-3 px at cfg1).
//
// Same GEMM view and interface as conv2d.hip (OUT[Cout x P] = W[Cout x K] X[K x P],
// NCHW fp32 activations, multi-segment input, channel-offset output, fused
// epilogue), plus a power-of-two weight scale: weights are packed pre-split
// and multiplied by 2^wexp so their lo halves stay out of the fp16 subnormal
// range; the epilogue multiplies by 2^-wexp (exact).
//
// Fragments (v_mfma_f32_32x32x16_f16): lane l, r = l&31, h = l>>5 holds
//   A[m = r][k = 8h + j], B[k = 8h + j][n = r], j = 0..7 (one 16-B half8);
//   D[m][n]: n = l&31, m = (reg&3) + 8(reg>>2) + 4h.
// LDS rows are k-contiguous ([m][k] / [n][k], padded) so every fragment is
// one ds_read_b128.  Pixels are split on the fly while staging: each thread
// loads 8 channels of one pixel (coalesced across lanes) and writes the hi
// and lo half8 with two ds_write_b128.
#include "fsmi_common.h"

namespace fsmi {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

constexpr int XKC = 32;             // channels per K chunk (2 MFMA k-steps)
constexpr int XROW = XKC + 8;       // padded LDS row (halves)
constexpr int kXMaxSeg = 4;

struct ConvX3Args {
  const float* seg_ptr[kXMaxSeg];
  long long seg_bstride[kXMaxSeg];
  int seg_end[kXMaxSeg];
  int nseg, Cin, CinP;              // CinP = roundup(Cin, XKC)
  const _Float16* whi;              // [KH*KW][CinP/XKC][CoutP][XKC] (pre-split, pre-scaled)
  const _Float16* wlo;
  float wscale;                     // 2^-wexp
  const float* bias;
  const float* gamma;
  const float* res;
  long long res_bstride;
  float* out;
  long long out_bstride;
  int co0, Cout, CoutP, B, H, W, act;
  float alpha;
};

__device__ __forceinline__ float gelu_erf_x(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

template <int KH, int KW, int BM, int BN, int WM>
__global__ __launch_bounds__(256) void conv2d_x3_kernel(ConvX3Args a) {
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / (32 * WM), TN = BN / (32 * WN);
  constexpr int PH = KH / 2, PW = KW / 2;
  constexpr int A_PIECES = BM * XKC / 8;            // 16-B pieces per hi (or lo) weight tile
  constexpr int A_PER_T = (A_PIECES + 255) / 256;
  constexpr int B_TASKS = BN * (XKC / 8);           // (pixel, 8-channel group) tasks
  constexpr int B_PER_T = (B_TASKS + 255) / 256;
  __shared__ __attribute__((aligned(16))) _Float16 Ah[BM][XROW];
  __shared__ __attribute__((aligned(16))) _Float16 Al[BM][XROW];
  __shared__ __attribute__((aligned(16))) _Float16 Bh[BN][XROW];
  __shared__ __attribute__((aligned(16))) _Float16 Bl[BN][XROW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int HW = a.H * a.W;
  const long long P = static_cast<long long>(a.B) * HW;
  const int m0 = blockIdx.y * BM;
  const long long n0 = static_cast<long long>(blockIdx.x) * BN;
  const int nck = a.CinP / XKC;
  const int nchunks = KH * KW * nck;

  // per-task pixel coordinates (fixed across chunks)
  int tb[B_PER_T], th[B_PER_T], tw[B_PER_T], tn[B_PER_T], tg[B_PER_T];
  bool tv[B_PER_T];
#pragma unroll
  for (int u = 0; u < B_PER_T; ++u) {
    const int task = tid + 256 * u;
    tn[u] = task % BN;
    tg[u] = task / BN;                 // 8-channel group within the chunk
    const long long p = n0 + tn[u];
    tv[u] = task < B_TASKS && p < P;
    const int b = tv[u] ? static_cast<int>(p / HW) : 0;
    const int hw = tv[u] ? static_cast<int>(p - static_cast<long long>(b) * HW) : 0;
    tb[u] = b;
    th[u] = hw / a.W;
    tw[u] = hw - th[u] * a.W;
  }

  uint4 rah[A_PER_T], ral[A_PER_T];
  float rx[B_PER_T][8];

  auto load_chunk = [&](int ch) {
    const int tap = ch / nck;
    const int cc = ch - tap * nck;
    const size_t wbase = (static_cast<size_t>(tap) * nck + cc) * a.CoutP * XKC;
#pragma unroll
    for (int u = 0; u < A_PER_T; ++u) {
      const int e = tid + 256 * u;
      rah[u] = ral[u] = make_uint4(0, 0, 0, 0);
      if (e < A_PIECES) {
        const int m = e / (XKC / 8), q = e - m * (XKC / 8);
        if (m0 + m < a.CoutP) {
          const size_t off = wbase + static_cast<size_t>(m0 + m) * XKC + q * 8;
          rah[u] = *reinterpret_cast<const uint4*>(a.whi + off);
          ral[u] = *reinterpret_cast<const uint4*>(a.wlo + off);
        }
      }
    }
    const int dh = tap / KW - PH, dw = tap % KW - PW;
#pragma unroll
    for (int u = 0; u < B_PER_T; ++u) {
      const int hh = th[u] + dh, ww = tw[u] + dw;
      const bool inb = tv[u] && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
      const int off = hh * a.W + ww;
      const int cb = cc * XKC + tg[u] * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ci = cb + j;
        float v = 0.f;
        if (inb && ci < a.Cin) {
          int s = 0, base = 0;
#pragma unroll
          for (int q = 0; q < kXMaxSeg - 1; ++q)
            if (q < a.nseg - 1 && ci >= a.seg_end[q]) { s = q + 1; base = a.seg_end[q]; }
          v = a.seg_ptr[s][tb[u] * a.seg_bstride[s] + static_cast<long long>(ci - base) * HW + off];
        }
        rx[u][j] = v;
      }
    }
  };
  auto store_chunk = [&]() {
#pragma unroll
    for (int u = 0; u < A_PER_T; ++u) {
      const int e = tid + 256 * u;
      if (e < A_PIECES) {
        const int m = e / (XKC / 8), q = e - m * (XKC / 8);
        *reinterpret_cast<uint4*>(&Ah[m][q * 8]) = rah[u];
        *reinterpret_cast<uint4*>(&Al[m][q * 8]) = ral[u];
      }
    }
#pragma unroll
    for (int u = 0; u < B_PER_T; ++u) {
      if (tid + 256 * u < B_TASKS) {
        half8 hi, lo;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const _Float16 x16 = static_cast<_Float16>(rx[u][j]);
          hi[j] = x16;
          lo[j] = static_cast<_Float16>(rx[u][j] - static_cast<float>(x16));
        }
        *reinterpret_cast<half8*>(&Bh[tn[u]][tg[u] * 8]) = hi;
        *reinterpret_cast<half8*>(&Bl[tn[u]][tg[u] * 8]) = lo;
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int hsel = lane >> 5, rl = lane & 31;
  load_chunk(0);
  for (int ch = 0; ch < nchunks; ++ch) {
    store_chunk();
    __syncthreads();
    if (ch + 1 < nchunks) load_chunk(ch + 1);   // next chunk's global loads fly during the MFMAs
#pragma unroll
    for (int ks = 0; ks < XKC; ks += 16) {
      half8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = (wm * TM + i) * 32 + rl;
        ah[i] = *reinterpret_cast<const half8*>(&Ah[m][ks + 8 * hsel]);
        al[i] = *reinterpret_cast<const half8*>(&Al[m][ks + 8 * hsel]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = (wn * TN + j) * 32 + rl;
        bh[j] = *reinterpret_cast<const half8*>(&Bh[n][ks + 8 * hsel]);
        bl[j] = *reinterpret_cast<const half8*>(&Bl[n][ks + 8 * hsel]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
    __syncthreads();
  }

#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const long long p = n0 + (wn * TN + j) * 32 + rl;
    if (p >= P) continue;
    const int b = static_cast<int>(p / HW);
    const int hw = static_cast<int>(p - static_cast<long long>(b) * HW);
    float* ob = a.out + b * a.out_bstride + hw;
    const float* rbp = a.res ? a.res + b * a.res_bstride + hw : nullptr;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hsel;
        if (co >= a.Cout) continue;
        float v = acc[i][j][r] * a.wscale;
        if (a.bias) v += a.bias[co];
        if (a.act == 1) v = fmaxf(v, 0.f);
        else if (a.act == 2) v = gelu_erf_x(v);
        v *= a.alpha;
        if (a.gamma) v *= a.gamma[co];
        if (rbp) v += rbp[static_cast<size_t>(co) * HW];
        ob[static_cast<size_t>(a.co0 + co) * HW] = v;
      }
    }
  }
}

template <int KH, int KW>
int launch_x3(const ConvX3Args& a, int cfg, hipStream_t s) {
  const long long P = static_cast<long long>(a.B) * a.H * a.W;
  switch (cfg) {
    case 0: {
      dim3 grid(ceil_div(P, 128), ceil_div(a.Cout, 128));
      hipLaunchKernelGGL((conv2d_x3_kernel<KH, KW, 128, 128, 2>), grid, dim3(256), 0, s, a);
      break;
    }
    case 1: {
      dim3 grid(ceil_div(P, 128), ceil_div(a.Cout, 64));
      hipLaunchKernelGGL((conv2d_x3_kernel<KH, KW, 64, 128, 1>), grid, dim3(256), 0, s, a);
      break;
    }
    case 2: {
      dim3 grid(ceil_div(P, 128), ceil_div(a.Cout, 32));
      hipLaunchKernelGGL((conv2d_x3_kernel<KH, KW, 32, 128, 1>), grid, dim3(256), 0, s, a);
      break;
    }
    default: {
      dim3 grid(ceil_div(P, 64), ceil_div(a.Cout, 128));
      hipLaunchKernelGGL((conv2d_x3_kernel<KH, KW, 128, 64, 2>), grid, dim3(256), 0, s, a);
      break;
    }
  }
  return finish_launch("fsmi_conv2d_x3");
}

int pick_cfg_x3(long long P, int Cout) {
  auto blocks = [&](int bm, int bn) { return ceil_div(P, bn) * static_cast<long long>(ceil_div(Cout, bm)); };
  if (Cout > 64 && blocks(128, 128) >= 480) return 0;
  if (Cout > 64 && blocks(128, 64) >= 240) return 3;
  if (Cout > 32) return 1;
  return 2;
}

}  // namespace
}  // namespace fsmi

using namespace fsmi;

extern "C" int fsmi_conv2d_x3(const float* const* seg_ptr, const int* seg_ch, const int* seg_ctot, int nseg,
                              const void* whi, const void* wlo, int wexp, const float* bias, const float* gamma,
                              const float* res, int res_ctot, float* out, int out_ctot, int co0, int B, int Cout,
                              int KH, int KW, int H, int W, int act, float alpha, int cfg, void* stream) {
  FSMI_CHECK_ARG(seg_ptr && seg_ch && seg_ctot && whi && wlo && out, "fsmi_conv2d_x3: null pointer");
  FSMI_CHECK_ARG(nseg >= 1 && nseg <= kXMaxSeg, "fsmi_conv2d_x3: 1..%d input segments, got %d", kXMaxSeg, nseg);
  FSMI_CHECK_ARG(B > 0 && Cout > 0 && H > 0 && W > 0, "fsmi_conv2d_x3: bad shape");
  FSMI_CHECK_ARG((KH == 1 && KW == 1) || (KH == 3 && KW == 3) || (KH == 7 && KW == 7),
                 "fsmi_conv2d_x3: kernel %dx%d unsupported (1x1, 3x3, 7x7)", KH, KW);
  FSMI_CHECK_ARG(act >= 0 && act <= 2, "fsmi_conv2d_x3: act %d", act);
  FSMI_CHECK_ARG(co0 >= 0 && co0 + Cout <= out_ctot, "fsmi_conv2d_x3: output slice outside the tensor");
  ConvX3Args a{};
  int cin = 0;
  const long long HW = static_cast<long long>(H) * W;
  for (int i = 0; i < nseg; ++i) {
    FSMI_CHECK_ARG(seg_ptr[i] && seg_ch[i] > 0 && seg_ctot[i] >= seg_ch[i], "fsmi_conv2d_x3: bad segment %d", i);
    a.seg_ptr[i] = seg_ptr[i];
    a.seg_bstride[i] = static_cast<long long>(seg_ctot[i]) * HW;
    cin += seg_ch[i];
    a.seg_end[i] = cin;
  }
  a.nseg = nseg;
  a.Cin = cin;
  a.CinP = (cin + XKC - 1) / XKC * XKC;
  a.whi = static_cast<const _Float16*>(whi);
  a.wlo = static_cast<const _Float16*>(wlo);
  a.wscale = ldexpf(1.f, -wexp);
  a.bias = bias;
  a.gamma = gamma;
  a.res = res;
  a.res_bstride = static_cast<long long>(res_ctot) * HW;
  a.out = out;
  a.out_bstride = static_cast<long long>(out_ctot) * HW;
  a.co0 = co0;
  a.Cout = Cout;
  a.CoutP = (Cout + 31) / 32 * 32;
  a.B = B;
  a.H = H;
  a.W = W;
  a.act = act;
  a.alpha = alpha;
  if (cfg < 0) cfg = pick_cfg_x3(static_cast<long long>(B) * HW, Cout);
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_CONV2D, s);
  if (KH == 1) return launch_x3<1, 1>(a, cfg, s);
  if (KH == 3) return launch_x3<3, 3>(a, cfg, s);
  return launch_x3<7, 7>(a, cfg, s);
}
