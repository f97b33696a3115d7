// Halo-tiled split-precision ("3 x fp16") convolution for the refinement loop.
//
// conv2d_x3.hip streams an im2col view: for a 3x3 layer every pixel is staged
// 9 times and the full weight matrix once per pixel tile (~2.8 GB of on-chip
// traffic for one 512->512 layer at 120x160).  Here a block owns a 2D pixel
// tile (TR rows x 32 columns of one image) and BM output channels:
//   * per 32-channel chunk the (TR+2) x 34 input halo is loaded ONCE, split
//     into fp16 hi/lo and kept in LDS for all 9 taps (fragments for tap
//     (dh,dw) are the halo rows/cols shifted by (dh,dw));
//   * per tap the BM x 32 weight slice (pre-split, pre-packed) goes through a
//     double-buffered LDS slot whose next fill is in flight during the MFMAs;
//   * blocks are ordered cout-tile-major over an XCD-aware remap, so each XCD
//     works on one cout slice and keeps its weights in its 4 MB L2.
// MFMA v_mfma_f32_32x32x16_f16, three per product (lo*hi, hi*lo, hi*hi), fp32
// accumulation; fragment maps as in conv2d_x3.hip.  Epilogue identical to
// fsmi_conv2d (bias, ReLU/GELU, alpha, gamma, residual, channel-offset store).
#include "fsmi_common.h"

namespace fsmi {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

constexpr int HKC = 32;            // channels per chunk
constexpr int HROW = HKC + 8;      // padded LDS row (halves): conflict-free ds_read_b128 at 80-B stride
constexpr int kHMaxSeg = 4;

struct HaloArgs {
  const float* seg_ptr[kHMaxSeg];
  long long seg_bstride[kHMaxSeg];
  int seg_end[kHMaxSeg];
  int nseg, Cin, CinP;
  const _Float16* whi;             // [taps][CinP/32][CoutP][32]
  const _Float16* wlo;
  float wscale;
  const float* bias;
  const float* gamma;
  const float* res;
  long long res_bstride;
  float* out;
  long long out_bstride;
  int co0, Cout, CoutP, B, H, W, act;
  float alpha;
  int nrt, nct, npix, nco;         // row tiles, col tiles, pixel tiles (B*nrt*nct), cout tiles
  int nsplit, kpc;                 // split-K factor, channel chunks per split
  float* ws;                       // [nsplit][B][Cout][H*W] partial sums when nsplit > 1
};

__device__ __forceinline__ float gelu_erf_h(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

template <int KS, int BM, int TR, int WM>
__global__ __launch_bounds__(256) void conv_halo_x3_kernel(HaloArgs a) {
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM / 32, TN = TR / WN;
  constexpr int PD = KS / 2;
  constexpr int HR = TR + KS - 1, HC = 32 + KS - 1, NHP = HR * HC;
  constexpr int NTAP = KS * KS;
  constexpr int W_PIECES = BM * HKC / 8;           // 16-B pieces per hi (or lo) weight slice
  constexpr int W_PER_T = (W_PIECES + 255) / 256;
  constexpr int X_TASKS = NHP * (HKC / 8);
  constexpr int X_PER_T = (X_TASKS + 255) / 256;
  __shared__ __attribute__((aligned(16))) _Float16 Xh[NHP][HROW];
  __shared__ __attribute__((aligned(16))) _Float16 Xl[NHP][HROW];
  __shared__ __attribute__((aligned(16))) _Float16 Wh[2][BM][HROW];
  __shared__ __attribute__((aligned(16))) _Float16 Wl[2][BM][HROW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int hsel = lane >> 5, rl = lane & 31;
  // cout-tile-major logical order over an XCD-aware remap: an XCD's blocks share weights in its L2
  const unsigned item = xcd_remap(blockIdx.x, gridDim.x);
  const int cs = item / a.npix;             // (cout tile, split) pair
  const int ptile = item - cs * a.npix;
  const int ctile = cs / a.nsplit, split = cs - ctile * a.nsplit;
  const int m0 = ctile * BM;
  const int b = ptile / (a.nrt * a.nct);
  const int prem = ptile - b * a.nrt * a.nct;
  const int r0 = (prem / a.nct) * TR, c0 = (prem % a.nct) * 32;
  const int HW = a.H * a.W;
  const int nck = a.CinP / HKC;

  uint4 rwh[W_PER_T], rwl[W_PER_T];
  auto load_w = [&](int cc, int tap) {
    const size_t base = (static_cast<size_t>(tap) * nck + cc) * a.CoutP * HKC;
#pragma unroll
    for (int u = 0; u < W_PER_T; ++u) {
      const int e = tid + 256 * u;
      rwh[u] = rwl[u] = make_uint4(0, 0, 0, 0);
      if (e < W_PIECES) {
        const int m = e / (HKC / 8), q = e - m * (HKC / 8);
        if (m0 + m < a.CoutP) {
          const size_t off = base + static_cast<size_t>(m0 + m) * HKC + q * 8;
          rwh[u] = *reinterpret_cast<const uint4*>(a.whi + off);
          rwl[u] = *reinterpret_cast<const uint4*>(a.wlo + off);
        }
      }
    }
  };
  auto store_w = [&](int buf) {
#pragma unroll
    for (int u = 0; u < W_PER_T; ++u) {
      const int e = tid + 256 * u;
      if (e < W_PIECES) {
        const int m = e / (HKC / 8), q = e - m * (HKC / 8);
        *reinterpret_cast<uint4*>(&Wh[buf][m][q * 8]) = rwh[u];
        *reinterpret_cast<uint4*>(&Wl[buf][m][q * 8]) = rwl[u];
      }
    }
  };
  // halo chunk -> registers (issued a whole chunk ahead), then split into LDS
  float xv[X_PER_T][8];
  auto load_halo = [&](int cc) {
#pragma unroll
    for (int u = 0; u < X_PER_T; ++u) {
      const int task = tid + 256 * u;
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[u][j] = 0.f;
      if (task < X_TASKS) {
        const int hp = task % NHP, g = task / NHP;
        const int hr = hp / HC, hc = hp - hr * HC;
        const int hh = r0 + hr - PD, ww = c0 + hc - PD;
        const int ci0 = cc * HKC + g * 8;
        if (hh >= 0 && hh < a.H && ww >= 0 && ww < a.W && ci0 < a.Cin) {
          int s = 0, base = 0;   // segments are multiples of 8 channels: one lookup per group
#pragma unroll
          for (int q = 0; q < kHMaxSeg - 1; ++q)
            if (q < a.nseg - 1 && ci0 >= a.seg_end[q]) { s = q + 1; base = a.seg_end[q]; }
          const float* src = a.seg_ptr[s] + b * a.seg_bstride[s] + static_cast<long long>(ci0 - base) * HW +
                             hh * a.W + ww;
          const int nv = min(8, a.Cin - ci0);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < nv) xv[u][j] = src[static_cast<size_t>(j) * HW];
        }
      }
    }
  };
  auto store_halo = [&]() {
#pragma unroll
    for (int u = 0; u < X_PER_T; ++u) {
      const int task = tid + 256 * u;
      if (task < X_TASKS) {
        const int hp = task % NHP, g = task / NHP;
        half8 hi, lo;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const _Float16 x16 = static_cast<_Float16>(xv[u][j]);
          hi[j] = x16;
          lo[j] = static_cast<_Float16>(xv[u][j] - static_cast<float>(x16));
        }
        *reinterpret_cast<half8*>(&Xh[hp][g * 8]) = hi;
        *reinterpret_cast<half8*>(&Xl[hp][g * 8]) = lo;
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

  // split-K: this block reduces channel chunks [cc_begin, cc_end)
  const int cc_begin = split * a.kpc;
  const int cc_end = min(nck, cc_begin + a.kpc);
  int step = 0;
  load_w(cc_begin, 0);
  load_halo(cc_begin);
  for (int cc = cc_begin; cc < cc_end; ++cc) {
    __syncthreads();               // every wave is done with the previous chunk's halo
    store_halo();
    if (cc + 1 < cc_end) load_halo(cc + 1);   // in flight during this chunk's taps
#pragma unroll 1
    for (int tap = 0; tap < NTAP; ++tap, ++step) {
      const int buf = step & 1;
      store_w(buf);
      __syncthreads();             // halo (first tap) and this tap's weights visible
      if (tap + 1 < NTAP) load_w(cc, tap + 1);
      else if (cc + 1 < cc_end) load_w(cc + 1, 0);
      const int dh = tap / KS, dw = tap % KS;
#pragma unroll
      for (int ks = 0; ks < HKC; ks += 16) {
        half8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int m = (wm * TM + i) * 32 + rl;
          ah[i] = *reinterpret_cast<const half8*>(&Wh[buf][m][ks + 8 * hsel]);
          al[i] = *reinterpret_cast<const half8*>(&Wl[buf][m][ks + 8 * hsel]);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int hp = ((wn * TN + j) + dh) * HC + rl + dw;
          bh[j] = *reinterpret_cast<const half8*>(&Xh[hp][ks + 8 * hsel]);
          bl[j] = *reinterpret_cast<const half8*>(&Xl[hp][ks + 8 * hsel]);
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
    }
  }

  // epilogue: n = lane&31 is the pixel column, rows of the tile on j
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int hh = r0 + wn * TN + j, ww = c0 + rl;
    if (hh >= a.H || ww >= a.W) continue;
    const int hw = hh * a.W + ww;
    if (a.nsplit > 1) {            // raw partial sums; conv_split_reduce_kernel applies the epilogue
      float* wp = a.ws + (static_cast<size_t>(split) * a.B + b) * a.Cout * HW + hw;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hsel;
          if (co < a.Cout) wp[static_cast<size_t>(co) * HW] = acc[i][j][r] * a.wscale;
        }
      continue;
    }
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
        else if (a.act == 2) v = gelu_erf_h(v);
        v *= a.alpha;
        if (a.gamma) v *= a.gamma[co];
        if (rbp) v += rbp[static_cast<size_t>(co) * HW];
        ob[static_cast<size_t>(a.co0 + co) * HW] = v;
      }
    }
  }
}

// Sums the split-K partials in split order (deterministic) and applies the epilogue.
__global__ __launch_bounds__(256) void conv_split_reduce_kernel(HaloArgs a) {
  const long long HW = static_cast<long long>(a.H) * a.W;
  const long long n = static_cast<long long>(a.B) * a.Cout * HW;
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const int hw = static_cast<int>(i % HW);
  const int co = static_cast<int>((i / HW) % a.Cout);
  const int b = static_cast<int>(i / (HW * a.Cout));
  float v = 0.f;
  for (int sp = 0; sp < a.nsplit; ++sp) v += a.ws[sp * n + i];
  if (a.bias) v += a.bias[co];
  if (a.act == 1) v = fmaxf(v, 0.f);
  else if (a.act == 2) v = gelu_erf_h(v);
  v *= a.alpha;
  if (a.gamma) v *= a.gamma[co];
  if (a.res) v += a.res[b * a.res_bstride + co * HW + hw];
  a.out[b * a.out_bstride + (a.co0 + co) * HW + hw] = v;
}

// Vector form (H*W % 4 == 0): one (b, co) plane per blockIdx.y, float4 per thread,
// all nsplit partial loads in flight before the ordered sum.
__global__ __launch_bounds__(256) void conv_split_reduce4_kernel(HaloArgs a) {
  const int HW = a.H * a.W;
  const int hw = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (hw >= HW) return;
  const int plane = blockIdx.y, co = plane % a.Cout, b = plane / a.Cout;
  const size_t n = static_cast<size_t>(a.B) * a.Cout * HW;
  const float* src = a.ws + static_cast<size_t>(plane) * HW + hw;
  float4 p[8];
#pragma unroll
  for (int sp = 0; sp < 8; ++sp)
    if (sp < a.nsplit) p[sp] = *reinterpret_cast<const float4*>(src + sp * n);
  float4 v = p[0];
#pragma unroll
  for (int sp = 1; sp < 8; ++sp)
    if (sp < a.nsplit) { v.x += p[sp].x; v.y += p[sp].y; v.z += p[sp].z; v.w += p[sp].w; }
  const float bb = a.bias ? a.bias[co] : 0.f;
  float r[4] = {v.x + bb, v.y + bb, v.z + bb, v.w + bb};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (a.act == 1) r[k] = fmaxf(r[k], 0.f);
    else if (a.act == 2) r[k] = gelu_erf_h(r[k]);
    r[k] *= a.alpha;
    if (a.gamma) r[k] *= a.gamma[co];
  }
  if (a.res) {
    const float4 q = *reinterpret_cast<const float4*>(a.res + b * a.res_bstride + static_cast<size_t>(co) * HW + hw);
    r[0] += q.x; r[1] += q.y; r[2] += q.z; r[3] += q.w;
  }
  *reinterpret_cast<float4*>(a.out + b * a.out_bstride + static_cast<size_t>(a.co0 + co) * HW + hw) =
      make_float4(r[0], r[1], r[2], r[3]);
}

template <int KS, int BM, int TR, int WM>
void tile_counts(HaloArgs& a) {
  a.nrt = (a.H + TR - 1) / TR;
  a.nct = (a.W + 31) / 32;
  a.npix = a.B * a.nrt * a.nct;
  a.nco = (a.Cout + BM - 1) / BM;
}

template <int KS, int BM, int TR, int WM>
int launch_halo(HaloArgs a, hipStream_t s) {
  const unsigned grid = static_cast<unsigned>(a.npix) * a.nco * a.nsplit;
  hipLaunchKernelGGL((conv_halo_x3_kernel<KS, BM, TR, WM>), dim3(grid), dim3(256), 0, s, a);
  if (a.nsplit > 1) {
    const int HW = a.H * a.W;
    const bool vec = HW % 4 == 0 && a.nsplit <= 8 && reinterpret_cast<uintptr_t>(a.out) % 16 == 0 &&
                     reinterpret_cast<uintptr_t>(a.ws) % 16 == 0 &&
                     (!a.res || reinterpret_cast<uintptr_t>(a.res) % 16 == 0);
    if (vec) {
      hipLaunchKernelGGL(conv_split_reduce4_kernel, dim3((HW / 4 + 255) / 256, a.B * a.Cout), dim3(256), 0, s, a);
    } else {
      const long long n = static_cast<long long>(a.B) * a.Cout * HW;
      hipLaunchKernelGGL(conv_split_reduce_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s,
                         a);
    }
  }
  return finish_launch("fsmi_conv2d_halo_x3");
}

}  // namespace
}  // namespace fsmi

using namespace fsmi;

extern "C" int fsmi_conv2d_halo_x3(const float* const* seg_ptr, const int* seg_ch, const int* seg_ctot, int nseg,
                                   const void* whi, const void* wlo, int wexp, const float* bias, const float* gamma,
                                   const float* res, int res_ctot, float* out, int out_ctot, int co0, int B, int Cout,
                                   int KS, int H, int W, int act, float alpha, int cfg, int nsplit, float* ws,
                                   long long ws_floats, void* stream) {
  FSMI_CHECK_ARG(seg_ptr && seg_ch && seg_ctot && whi && wlo && out, "fsmi_conv2d_halo_x3: null pointer");
  FSMI_CHECK_ARG(nseg >= 1 && nseg <= kHMaxSeg, "fsmi_conv2d_halo_x3: 1..%d segments, got %d", kHMaxSeg, nseg);
  FSMI_CHECK_ARG(B > 0 && Cout > 0 && H > 0 && W > 0, "fsmi_conv2d_halo_x3: bad shape");
  FSMI_CHECK_ARG(KS == 1 || KS == 3, "fsmi_conv2d_halo_x3: kernel %d unsupported (1, 3)", KS);
  FSMI_CHECK_ARG(act >= 0 && act <= 2, "fsmi_conv2d_halo_x3: act %d", act);
  FSMI_CHECK_ARG(co0 >= 0 && co0 + Cout <= out_ctot, "fsmi_conv2d_halo_x3: output slice outside the tensor");
  HaloArgs a{};
  int cin = 0;
  const long long HW = static_cast<long long>(H) * W;
  for (int i = 0; i < nseg; ++i) {
    FSMI_CHECK_ARG(seg_ptr[i] && seg_ch[i] > 0 && seg_ctot[i] >= seg_ch[i], "fsmi_conv2d_halo_x3: bad segment %d",
                   i);
    FSMI_CHECK_ARG(i == nseg - 1 || seg_ch[i] % 8 == 0,
                   "fsmi_conv2d_halo_x3: inner segments must be multiples of 8 channels (segment %d: %d)", i,
                   seg_ch[i]);
    a.seg_ptr[i] = seg_ptr[i];
    a.seg_bstride[i] = static_cast<long long>(seg_ctot[i]) * HW;
    cin += seg_ch[i];
    a.seg_end[i] = cin;
  }
  a.nseg = nseg;
  a.Cin = cin;
  a.CinP = (cin + HKC - 1) / HKC * HKC;
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
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_CONV2D, s);
  if (cfg < 0) cfg = (Cout > 64) ? 1 : 0;
  if (cfg == 1) tile_counts<3, 128, 4, 2>(a);
  else tile_counts<3, 64, 8, 1>(a);
  // split-K when the output tiles alone cannot fill 256 CUs x 2 resident blocks
  const int nck = a.CinP / HKC;
  const long long per_split = static_cast<long long>(B) * Cout * H * W;
  if (nsplit < 0) {
    // measured on the cfg2 loop layers (tools/conv_bench.py --nsplit): 3x3 layers are best
    // near ~1200 blocks (~2.3 rounds of the 512 resident slots), 1x1 layers -- a quarter of
    // the MFMA work per chunk, so the extra reduce pass weighs more -- near ~400
    const int base = a.npix * a.nco;
    nsplit = max(1, (KS == 3 ? 1200 : 400) / base);
    nsplit = min(nsplit, min(8, nck / 2 > 0 ? nck / 2 : 1));      // keep >= 2 chunks per split
    if (!ws) nsplit = 1;
    else if (per_split * nsplit > ws_floats) nsplit = static_cast<int>(max(1LL, ws_floats / per_split));
  }
  nsplit = max(1, min(nsplit, nck));
  a.kpc = (nck + nsplit - 1) / nsplit;
  a.nsplit = (nck + a.kpc - 1) / a.kpc;                    // no empty splits
  FSMI_CHECK_ARG(a.nsplit == 1 || (ws && per_split * a.nsplit <= ws_floats),
                 "fsmi_conv2d_halo_x3: split-K %d needs %lld workspace floats", a.nsplit, per_split * a.nsplit);
  a.ws = ws;
  if (KS == 3) return cfg == 1 ? launch_halo<3, 128, 4, 2>(a, s) : launch_halo<3, 64, 8, 1>(a, s);
  return cfg == 1 ? launch_halo<1, 128, 4, 2>(a, s) : launch_halo<1, 64, 8, 1>(a, s);
}
