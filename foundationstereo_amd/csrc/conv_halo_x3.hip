// Halo-tiled split-precision ("3 x fp16") convolution for the refinement loop.
//
// conv2d_x3.hip streams an im2col view: for a 3x3 layer every pixel is staged
// 9 times and the full weight matrix once per pixel tile (~2.8 GB of on-chip
// traffic for one 512->512 layer at 120x160).  Here a block owns a 2D pixel
// tile (TR rows x 32 columns of one image) and BM output channels:
//   * per 32-channel chunk the (TR+2) x 34 input halo is loaded ONCE, split
//     into fp16 hi/lo and kept in LDS for all 9 taps (fragments for tap
//     (dh,dw) are the halo rows/cols shifted by (dh,dw));
//   * weights (pre-split, pre-packed) either go per tap through a double-
//     buffered LDS slot whose next fill is in flight during the MFMAs
//     (conv_halo_x3_kernel, cfg 0/1: one barrier per tap), or each wave loads
//     its own A fragments from L2 into a double-buffered register set one tap
//     ahead (conv_halo_wreg_kernel, cfg 2/3: LDS holds only the halo, two
//     barriers per 32-channel chunk);
//   * blocks are ordered cout-tile-major over an XCD-aware remap, so each XCD
//     works on one cout slice and keeps its weights in its 4 MB L2.
// MFMA v_mfma_f32_32x32x16_f16, three per product (lo*hi, hi*lo, hi*hi), fp32
// accumulation; fragment maps as in conv2d_x3.hip.  Epilogue identical to
// fsmi_conv2d (bias, ReLU/GELU, alpha, gamma, residual, channel-offset store).
#include <cstdlib>
#include <type_traits>

#include "fsmi_common.h"

namespace fsmi {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x8 __attribute__((ext_vector_type(8)));

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
  int res_pre;                     // residual added before the activation (ResNet block tail)
  // 3D: NCDHW tensors with D depth planes; a KD x KS x KS kernel is the sum over kd of 2D
  // convs on plane d + kd - PDD.  2D: D = KD = 1.
  int D, KD, PDD;
  long long cstride;               // channel stride = D*H*W
  int nrt, nct, npix, nco;         // row tiles, col tiles, pixel tiles (B*D*nrt*nct), cout tiles
  int nsplit, kpc;                 // split-K factor, (kd, channel chunk) pairs per split
  float* ws;                       // [nsplit][B][Cout][D*H*W] partial sums when nsplit > 1
  unsigned long long* ts;          // debug (fsmi_debug_conv_timestamps): per-block wall-clock stamps
  int dbg;                         // ablation (FSMI_CONV_DBG): 1 weights from one line, 2 no halo reloads
  // SelectiveConvGRU gate epilogues (act 3..5), core/update.py:83-95,117; all (B, gHd, H, W)
  // except gatt (B, 1, H, W)
  const float* gh;                 // hidden state h
  float* gz;                       // z = sigmoid(z_pre): written by act 3, read by act 4 / 5
  const float* gatt;               // att
  float* grh;                      // sigmoid(r_pre) * h, written by act 3
  int gHd;
};

__device__ __forceinline__ float gelu_erf_h(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float sigm_h(float x) { return 1.f / (1.f + expf(-x)); }

// Final value of output channel co at (b, sp) -- sp = d*H*W + h*W + w -- from the raw conv sum v
// (already x wscale).
//  act 0/1/2/6: out[b, co0+co] = res + gamma * alpha * act(v + bias)   (none / ReLU / GELU-erf /
//               LeakyReLU 0.01); with res_pre: gamma * alpha * act(v + bias + res)
//  act 3 (convz|convr):  co <  Hd: z[b,co] = sigmoid(v + bias);
//                        co >= Hd: rh[b,co-Hd] = sigmoid(v + bias) * h[b,co-Hd]
//  act 4 (small convq):  out[b,co0+co] = ((1-z)h + z tanh(v + bias)) * att
//  act 5 (large convq):  out[b,co0+co] += ((1-z)h + z tanh(v + bias)) * (1 - att)
// RESPRE: compile the res_pre (ResNet tail) path; the 2D conv kernels instantiate without it --
// with the branch present their epilogue needs ~100 more VGPRs (occupancy 2 -> 1).
// Every tensor arrives as its own __restrict__ parameter: a caller that runs a whole batch of
// elements inside ONE call of a function taking them so lets the compiler issue all the batch's
// loads (bias, residual, gate state) ahead of its stores.  Read through the HaloArgs fields
// (which may alias the output) each load waited behind the previous element's store, and a
// tile's epilogue paid one L2 round trip per element: 20-56 % of a block's lifetime on the
// nsplit = 1 layers (tools/conv_phases.py).
template <bool RESPRE>
__device__ __forceinline__ void store_el(const HaloArgs& a, float v, int co, int b, long long hw,
                                         float* __restrict__ out, const float* __restrict__ bias,
                                         const float* __restrict__ gamma, const float* __restrict__ res,
                                         const float* __restrict__ gh, float* __restrict__ gz,
                                         const float* __restrict__ gatt, float* __restrict__ grh) {
  const long long HW = a.cstride;
  if (bias) v += bias[co];
  if (a.act >= 3 && a.act <= 5) {
    const size_t g = (static_cast<size_t>(b) * a.gHd + (co % a.gHd)) * HW + hw;
    if (a.act == 3) {
      const float sg = sigm_h(v);
      if (co < a.gHd) gz[g] = sg;
      else grh[g] = sg * gh[g];
      return;
    }
    const float z = gz[g], hv = gh[g], at = gatt[static_cast<size_t>(b) * HW + hw];
    const float hn = (1.f - z) * hv + z * tanhf(v);
    float* o = out + b * a.out_bstride + static_cast<long long>(a.co0 + co) * HW + hw;
    if (a.act == 4) *o = hn * at;
    else *o = *o + hn * (1.f - at);
    return;
  }
  float* o = out + b * a.out_bstride + static_cast<long long>(a.co0 + co) * HW + hw;
  if (RESPRE && a.res_pre) {       // ResNet tail: act(v + bias + res)
    v += res[b * a.res_bstride + static_cast<long long>(co) * HW + hw];
    *o = a.act == 1 ? fmaxf(v, 0.f) : (a.act == 6 ? (v >= 0.f ? v : 0.01f * v) : v);
    return;
  }
  if (a.act == 1) v = fmaxf(v, 0.f);
  else if (a.act == 2) v = gelu_erf_h(v);
  else if (a.act == 6) v = v >= 0.f ? v : 0.01f * v;
  v *= a.alpha;
  if (gamma) v *= gamma[co];
  if (res) v += res[b * a.res_bstride + static_cast<long long>(co) * HW + hw];
  *o = v;
}

template <bool RESPRE = true>
__device__ __forceinline__ void store_out(const HaloArgs& a, float v, int co, int b, long long hw) {
  store_el<RESPRE>(a, v, co, b, hw, a.out, a.bias, a.gamma, a.res, a.gh, a.gz, a.gatt, a.grh);
}

// One 16-element accumulator fragment (couts cb + (r&3) + 8(r>>2)) at one pixel, activation ACT
// fixed at compile time and one restrict scope: the fragment's bias / gamma / residual / gate
// loads are issued together, then 16 branch-free finishes and stores.  (The generic store_el per
// element compiled to ~400 instructions per fragment with a wait per element: 20-56 % of a
// block's lifetime went to the epilogue on the nsplit = 1 layers, tools/conv_phases.py.)
template <int ACT, bool RESPRE>
__device__ __forceinline__ void store_frag(const HaloArgs& a, const f32x16& v, int cb, int b, long long hw,
                                           float* __restrict__ out, const float* __restrict__ bias,
                                           const float* __restrict__ gamma, const float* __restrict__ res,
                                           const float* __restrict__ gh, float* __restrict__ gz,
                                           const float* __restrict__ gatt, float* __restrict__ grh) {
  const long long HW = a.cstride;
  float bv[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) bv[r] = bias ? bias[min(cb + (r & 3) + 8 * (r >> 2), a.Cout - 1)] : 0.f;
  if constexpr (ACT >= 3 && ACT <= 5) {
    const float at = ACT == 3 ? 0.f : gatt[static_cast<size_t>(b) * HW + hw];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = cb + (r & 3) + 8 * (r >> 2);
      if (co >= a.Cout) continue;
      const float x = v[r] * a.wscale + bv[r];
      const size_t g = (static_cast<size_t>(b) * a.gHd + (co % a.gHd)) * HW + hw;
      if constexpr (ACT == 3) {
        const float sg = sigm_h(x);
        if (co < a.gHd) gz[g] = sg;
        else grh[g] = sg * gh[g];
      } else {
        const float z = gz[g];
        const float hn = (1.f - z) * gh[g] + z * tanhf(x);
        float* o = out + b * a.out_bstride + static_cast<long long>(a.co0 + co) * HW + hw;
        if constexpr (ACT == 4) *o = hn * at;
        else *o = *o + hn * (1.f - at);
      }
    }
    return;
  } else {
    float gv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) gv[r] = gamma ? gamma[min(cb + (r & 3) + 8 * (r >> 2), a.Cout - 1)] : 1.f;
    const bool pre = RESPRE && a.res_pre;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = cb + (r & 3) + 8 * (r >> 2);
      if (co >= a.Cout) continue;
      float x = v[r] * a.wscale + bv[r];
      const float rv = res ? res[b * a.res_bstride + static_cast<long long>(co) * HW + hw] : 0.f;
      if (pre) x += rv;            // ResNet tail: act(conv + bias + res)
      if constexpr (ACT == 1) x = fmaxf(x, 0.f);
      else if constexpr (ACT == 2) x = gelu_erf_h(x);
      else if constexpr (ACT == 6) x = x >= 0.f ? x : 0.01f * x;
      if (!pre) x = x * a.alpha * gv[r] + rv;
      out[b * a.out_bstride + static_cast<long long>(a.co0 + co) * HW + hw] = x;
    }
  }
}

// 4 consecutive pixels of one channel, one restrict scope
__device__ __forceinline__ void store4(const HaloArgs& a, const float (&v)[4], int co, int b, long long hw,
                                       float* __restrict__ out, const float* __restrict__ bias,
                                       const float* __restrict__ gamma, const float* __restrict__ res,
                                       const float* __restrict__ gh, float* __restrict__ gz,
                                       const float* __restrict__ gatt, float* __restrict__ grh) {
#pragma unroll
  for (int k = 0; k < 4; ++k) store_el<true>(a, v[k], co, b, hw + k, out, bias, gamma, res, gh, gz, gatt, grh);
}

// ---------------------------------------------------------------- shared pieces

// Input-halo staging for a TR x 32 pixel tile: task = (halo pixel, 8-channel
// group); per task a packed descriptor (clamped pixel offset << 3 | in-image << 2
// | group) computed once per block; a chunk is loaded into registers one chunk
// ahead and split into fp16 hi/lo when stored to LDS.
template <int KS, int TR>
struct HaloStage {
  static constexpr int PD = KS / 2, HR = TR + KS - 1, HC = 32 + KS - 1, NHP = HR * HC;
  static constexpr int X_TASKS = NHP * (HKC / 8), X_PER_T = (X_TASKS + 255) / 256;
  int desc[X_PER_T];
  f32x8 xv[X_PER_T];

  __device__ __forceinline__ void init(const HaloArgs& a, int tid, int r0, int c0) {
#pragma unroll
    for (int u = 0; u < X_PER_T; ++u) {
      const int task = min(tid + 256 * u, X_TASKS - 1);
      const int hp = task % NHP, g = task / NHP;
      const int hr = hp / HC, hc = hp - hr * HC;
      const int hh = r0 + hr - PD, ww = c0 + hc - PD;
      const bool in = hh >= 0 && hh < a.H && ww >= 0 && ww < a.W && tid + 256 * u < X_TASKS;
      const int pix = min(max(hh, 0), a.H - 1) * a.W + min(max(ww, 0), a.W - 1);
      desc[u] = (pix << 3) | (in ? 4 : 0) | g;
    }
  }

  // chunk cc of depth plane d (zeros outside [0, D))
  __device__ __forceinline__ void load(const HaloArgs& a, int b, int cc, int d = 0) {
    const long long HW = a.cstride;
    const bool full = (cc + 1) * HKC <= a.Cin;     // block-uniform: only the last chunk is ragged
    const bool plane_ok = d >= 0 && d < a.D;
    const long long poff = static_cast<long long>(min(max(d, 0), a.D - 1)) * a.H * a.W;
#pragma unroll
    for (int u = 0; u < X_PER_T; ++u) {
      const int g = desc[u] & 3, pix = desc[u] >> 3;
      const int ci0 = cc * HKC + g * 8;
      const int cic = min(ci0, a.Cin - 1);
      // segment of this 8-channel group (segments hold multiples of 8 channels): a select
      // chain over constant indices, so the kernarg arrays are never indexed per lane
      const float* sp = a.seg_ptr[0];
      long long sb = a.seg_bstride[0];
      int base = 0;
#pragma unroll
      for (int q = 1; q < kHMaxSeg; ++q) {
        const bool in_q = q < a.nseg && cic >= a.seg_end[q - 1];
        sp = in_q ? a.seg_ptr[q] : sp;
        sb = in_q ? a.seg_bstride[q] : sb;
        base = in_q ? a.seg_end[q - 1] : base;
      }
      const float* src = sp + b * sb + static_cast<long long>(cic - base) * HW + poff + pix;
      const bool ok = (desc[u] & 4) && plane_ok;
      f32x8 v;
      if (full) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = src[static_cast<size_t>(j) * HW];
      } else {
        const int nv = a.Cin - ci0;                // may be <= 0 in the padded tail
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float t = src[static_cast<size_t>(max(0, min(j, nv - 1))) * HW];
          v[j] = j < nv ? t : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[u][j] = ok ? v[j] : 0.f;
    }
  }

  __device__ __forceinline__ void store(_Float16 (*Xh)[HROW], _Float16 (*Xl)[HROW], int tid) const {
#pragma unroll
    for (int u = 0; u < X_PER_T; ++u) {
      const int task = tid + 256 * u;
      if (X_TASKS % 256 == 0 || task < X_TASKS) {
        const int hp = task % NHP, g = task / NHP;
        const half8 hi = __builtin_convertvector(xv[u], half8);
        const half8 lo = __builtin_convertvector(xv[u] - __builtin_convertvector(hi, f32x8), half8);
        *reinterpret_cast<half8*>(&Xh[hp][g * 8]) = hi;
        *reinterpret_cast<half8*>(&Xl[hp][g * 8]) = lo;
      }
    }
  }
};

struct TileCoord {
  int m0, b, d0, r0, c0, split;
};

// Tile t (cout tile = t / npix, pixel tile = t % npix; D3: depth fastest) -> coordinates
template <int BM, int TR, bool D3>
__device__ __forceinline__ TileCoord tile_coord(const HaloArgs& a, int ctile, int ptile) {
  TileCoord t;
  t.split = 0;
  t.m0 = ctile * BM;
  const int per_plane = a.nrt * a.nct;
  int prem;
  if constexpr (D3) {
    // depth fastest: blocks of consecutive output depths at one (row, col) tile run together on
    // one XCD, so the KD input planes each of them reads are shared in that XCD's L2 (depth-
    // slowest order re-fetched them from HBM: 10x the input for a (17,1,1) conv)
    t.d0 = ptile % a.D;
    const int rest = ptile / a.D;
    t.b = rest / per_plane;
    prem = rest - t.b * per_plane;
  } else {
    t.b = ptile / per_plane;
    t.d0 = 0;
    prem = ptile - t.b * per_plane;
  }
  t.r0 = (prem / a.nct) * TR;
  t.c0 = (prem % a.nct) * 32;
  return t;
}

// cout-tile-major logical order over an XCD-aware remap: an XCD's blocks share weights in its L2
template <int BM, int TR, bool D3>
__device__ __forceinline__ TileCoord decode_tile(const HaloArgs& a) {
  const unsigned item = xcd_remap(blockIdx.x, gridDim.x);
  const int cs = item / a.npix;                    // (cout tile, split) pair
  const int ptile = item - cs * a.npix;
  const int ctile = cs / a.nsplit;
  TileCoord t = tile_coord<BM, TR, D3>(a, ctile, ptile);
  t.split = cs - ctile * a.nsplit;
  return t;
}

template <int TM, int TN>
__device__ __forceinline__ void mma3(f32x16 (&acc)[TM][TN], const half8 (&ah)[TM], const half8 (&al)[TM],
                                     const half8 (&bh)[TN], const half8 (&bl)[TN]) {
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
    }
}

// Non-split epilogue of the block's tile with the activation fixed at compile time
template <int ACT, int TM, int TN, bool D3>
__device__ __forceinline__ void epi_tile(const HaloArgs& a, const f32x16 (&acc)[TM][TN], const TileCoord& t, int wm,
                                         int wn, int lane) {
  const int hsel = lane >> 5, rl = lane & 31;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int hh = t.r0 + wn * TN + j, ww = t.c0 + rl;
    if (hh >= a.H || ww >= a.W) continue;
    const long long hw = static_cast<long long>(t.d0) * a.H * a.W + hh * a.W + ww;
#pragma unroll
    for (int i = 0; i < TM; ++i)
      store_frag<ACT, D3>(a, acc[i][j], t.m0 + (wm * TM + i) * 32 + 4 * hsel, t.b, hw, a.out, a.bias, a.gamma, a.res,
                          a.gh, a.gz, a.gatt, a.grh);
  }
}

// n = lane&31 is the pixel column, tile row wn*TN + j; D row map of the 32x32 MFMA
template <int TM, int TN, bool D3>
__device__ __forceinline__ void conv_epilogue(const HaloArgs& a, const f32x16 (&acc)[TM][TN], const TileCoord& t,
                                              int wm, int wn, int lane, bool partial) {
  const int hsel = lane >> 5, rl = lane & 31;
  const long long HW = a.cstride;
  if (partial) {                   // raw partial sums into ws slot t.split; a reduce applies the epilogue
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int hh = t.r0 + wn * TN + j, ww = t.c0 + rl;
      if (hh >= a.H || ww >= a.W) continue;
      const long long hw = static_cast<long long>(t.d0) * a.H * a.W + hh * a.W + ww;
      float* wp = a.ws + (static_cast<size_t>(t.split) * a.B + t.b) * a.Cout * HW + hw;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = t.m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hsel;
          if (co < a.Cout) wp[static_cast<size_t>(co) * HW] = acc[i][j][r] * a.wscale;
        }
    }
    return;
  }
  switch (a.act) {                 // uniform: one specialised tile epilogue per activation
    case 1: epi_tile<1, TM, TN, D3>(a, acc, t, wm, wn, lane); break;
    case 2: epi_tile<2, TM, TN, D3>(a, acc, t, wm, wn, lane); break;
    case 3: epi_tile<3, TM, TN, D3>(a, acc, t, wm, wn, lane); break;
    case 4: epi_tile<4, TM, TN, D3>(a, acc, t, wm, wn, lane); break;
    case 5: epi_tile<5, TM, TN, D3>(a, acc, t, wm, wn, lane); break;
    case 6: epi_tile<6, TM, TN, D3>(a, acc, t, wm, wn, lane); break;
    default: epi_tile<0, TM, TN, D3>(a, acc, t, wm, wn, lane); break;
  }
}

// ---------------------------------------------------------------- cfg 0/1: weights through LDS

template <int KS, int BM, int TR, int WM, bool D3>
__global__ __launch_bounds__(256) void conv_halo_x3_kernel(HaloArgs a) {
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM / 32, TN = TR / WN;
  constexpr int NTAP = KS * KS;
  constexpr int W_PIECES = BM * HKC / 8;           // 16-B pieces per hi (or lo) weight slice
  constexpr int W_PER_T = W_PIECES / 256;
  static_assert(W_PIECES % 256 == 0, "weight pieces must tile the block");
  using HS = HaloStage<KS, TR>;
  __shared__ __attribute__((aligned(16))) _Float16 Xh[HS::NHP][HROW];
  __shared__ __attribute__((aligned(16))) _Float16 Xl[HS::NHP][HROW];
  __shared__ __attribute__((aligned(16))) _Float16 Wh[2][BM][HROW];
  __shared__ __attribute__((aligned(16))) _Float16 Wl[2][BM][HROW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int hsel = lane >> 5, rl = lane & 31;
  const TileCoord tc = decode_tile<BM, TR, D3>(a);
  const int m0 = tc.m0;
  const int nck = a.CinP / HKC;
  const int nq = D3 ? a.KD * nck : nck;            // chunks = (kd, 32-channel chunk) pairs, kd major

  const bool w_full = m0 + BM <= a.CoutP;          // block-uniform: only the last cout tile is ragged
  uint4 rwh[W_PER_T], rwl[W_PER_T];
  auto load_w = [&](int cc, int tap) {
    const size_t base = D3 ? (static_cast<size_t>((cc / nck) * NTAP + tap) * nck + cc % nck) * a.CoutP * HKC
                           : (static_cast<size_t>(tap) * nck + cc) * a.CoutP * HKC;
    const _Float16* ph = a.whi + base;
    const _Float16* pl = a.wlo + base;
    if (w_full) {
#pragma unroll
      for (int u = 0; u < W_PER_T; ++u) {
        const int e = tid + 256 * u;
        const int off = (m0 + e / (HKC / 8)) * HKC + (e % (HKC / 8)) * 8;
        rwh[u] = *reinterpret_cast<const uint4*>(ph + off);
        rwl[u] = *reinterpret_cast<const uint4*>(pl + off);
      }
    } else {
#pragma unroll
      for (int u = 0; u < W_PER_T; ++u) {
        const int e = tid + 256 * u;
        const int row = m0 + e / (HKC / 8);
        const int off = min(row, a.CoutP - 1) * HKC + (e % (HKC / 8)) * 8;   // clamped, then zeroed
        const uint4 h = *reinterpret_cast<const uint4*>(ph + off);
        const uint4 l = *reinterpret_cast<const uint4*>(pl + off);
        const bool ok = row < a.CoutP;             // per component: a uint4 ternary goes via scratch
        rwh[u] = make_uint4(ok ? h.x : 0u, ok ? h.y : 0u, ok ? h.z : 0u, ok ? h.w : 0u);
        rwl[u] = make_uint4(ok ? l.x : 0u, ok ? l.y : 0u, ok ? l.z : 0u, ok ? l.w : 0u);
      }
    }
  };
  auto store_w = [&](int buf) {
#pragma unroll
    for (int u = 0; u < W_PER_T; ++u) {
      const int e = tid + 256 * u;
      const int m = e / (HKC / 8), q = e % (HKC / 8);
      *reinterpret_cast<uint4*>(&Wh[buf][m][q * 8]) = rwh[u];
      *reinterpret_cast<uint4*>(&Wl[buf][m][q * 8]) = rwl[u];
    }
  };
  HS hs;
  hs.init(a, tid, tc.r0, tc.c0);

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // split-K: this block reduces chunks [cc_begin, cc_end)
  const int cc_begin = tc.split * a.kpc;
  const int cc_end = min(nq, cc_begin + a.kpc);
  int step = 0;
  load_w(cc_begin, 0);
  if constexpr (D3) hs.load(a, tc.b, cc_begin % nck, tc.d0 + cc_begin / nck - a.PDD);
  else hs.load(a, tc.b, cc_begin);
  for (int cc = cc_begin; cc < cc_end; ++cc) {
    __syncthreads();               // every wave is done with the previous chunk's halo
    hs.store(Xh, Xl, tid);
    if (cc + 1 < cc_end) {
      if constexpr (D3) hs.load(a, tc.b, (cc + 1) % nck, tc.d0 + (cc + 1) / nck - a.PDD);
      else hs.load(a, tc.b, cc + 1);
    }   // in flight during this chunk's taps
#pragma unroll 1
    for (int tap = 0; tap < NTAP; ++tap, ++step) {
      const int buf = step & 1;
      store_w(buf);
      __syncthreads();             // halo (first tap) and this tap's weights visible
      // next slice; past the end it re-loads the last one (unconditional, never used)
      const bool wrap = tap + 1 == NTAP;
      load_w(wrap ? min(cc + 1, cc_end - 1) : cc, wrap ? 0 : tap + 1);
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
          const int hp = ((wn * TN + j) + dh) * HS::HC + rl + dw;
          bh[j] = *reinterpret_cast<const half8*>(&Xh[hp][ks + 8 * hsel]);
          bl[j] = *reinterpret_cast<const half8*>(&Xl[hp][ks + 8 * hsel]);
        }
        mma3<TM, TN>(acc, ah, al, bh, bl);
      }
    }
  }
  conv_epilogue<TM, TN, D3>(a, acc, tc, wm, wn, lane, a.nsplit > 1);
}

// ---------------------------------------------------------------- cfg 2/3: weights in registers

template <int KS, int BM, int TR, int WM, bool D3>
__global__ __launch_bounds__(256) void conv_halo_wreg_kernel(HaloArgs a) {
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM / 32, TN = TR / WN;
  constexpr int NTAP = KS * KS;
  using HS = HaloStage<KS, TR>;
  __shared__ __attribute__((aligned(16))) _Float16 Xh[HS::NHP][HROW];
  __shared__ __attribute__((aligned(16))) _Float16 Xl[HS::NHP][HROW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int hsel = lane >> 5, rl = lane & 31;
  const int nck = a.CinP / HKC;
  const int nq = D3 ? a.KD * nck : nck;            // chunks = (kd, 32-channel chunk) pairs, kd major
  unsigned long long* tsb = a.ts ? a.ts + static_cast<size_t>(blockIdx.x) * 40 : nullptr;
  if (tsb && tid == 0) tsb[0] = wall_clock64();

  // one segment: chunks [cc_begin, cc_end) of tile tc; partial: raw sums into ws slot tc.split
  auto segment = [&](const TileCoord& tc, int cc_begin, int cc_end, bool partial) {
    // this lane's A-fragment rows (rows past Cout only feed outputs the epilogue drops:
    // clamped so every address is mapped, no zeroing needed)
    int wrow[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) wrow[i] = min(tc.m0 + (wm * TM + i) * 32 + rl, a.CoutP - 1) * HKC + 8 * hsel;
    half8 wf[2][TM][2][2];         // [buffer][i][k half][hi, lo]
    auto load_wf = [&](auto buf_c, int cc, int tap) {
      constexpr int buf = decltype(buf_c)::value;
      size_t base = D3 ? (static_cast<size_t>((cc / nck) * NTAP + tap) * nck + cc % nck) * a.CoutP * HKC
                       : (static_cast<size_t>(tap) * nck + cc) * a.CoutP * HKC;
      if (a.dbg & 1) base = 0;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          wf[buf][i][k][0] = *reinterpret_cast<const half8*>(a.whi + base + wrow[i] + 16 * k);
          wf[buf][i][k][1] = *reinterpret_cast<const half8*>(a.wlo + base + wrow[i] + 16 * k);
        }
    };
    HS hs;
    hs.init(a, tid, tc.r0, tc.c0);

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // tap t of a chunk uses register buffer (t + P) & 1, P = chunk parity; each tap prefetches the next
    auto chunk = [&](auto par_c, int cc) {
      constexpr int P = decltype(par_c)::value;
#pragma unroll
      for (int tap = 0; tap < NTAP; ++tap) {
        const bool last = tap + 1 == NTAP;
        if (((tap + P) & 1) == 0) {
          load_wf(std::integral_constant<int, 1>(), last ? min(cc + 1, cc_end - 1) : cc, last ? 0 : tap + 1);
        } else {
          load_wf(std::integral_constant<int, 0>(), last ? min(cc + 1, cc_end - 1) : cc, last ? 0 : tap + 1);
        }
        // issue the next tap's loads before this tap's MFMAs: unfenced, the scheduler sinks them
        // below the last MFMA and reuses the current buffer's registers -- a single buffer whose
        // L2 round trip every tap then waits on
        __builtin_amdgcn_sched_barrier(0);
        const int dh = tap / KS, dw = tap % KS;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          half8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            ah[i] = wf[(tap + P) & 1][i][k][0];
            al[i] = wf[(tap + P) & 1][i][k][1];
          }
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int hp = ((wn * TN + j) + dh) * HS::HC + rl + dw;
            bh[j] = *reinterpret_cast<const half8*>(&Xh[hp][16 * k + 8 * hsel]);
            bl[j] = *reinterpret_cast<const half8*>(&Xl[hp][16 * k + 8 * hsel]);
          }
          mma3<TM, TN>(acc, ah, al, bh, bl);
        }
        // keep the one-tap-ahead structure: without this fence the scheduler hoists every
        // tap's loads of the unrolled chunk to its top (500 registers, 1 wave per SIMD)
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    auto stage = [&](int cc) {
      __syncthreads();             // every wave is done with the previous chunk's halo
      if (tsb && tid == 0 && cc - cc_begin < 36) tsb[1 + cc - cc_begin] = wall_clock64();
      hs.store(Xh, Xl, tid);
      if (cc + 1 < cc_end && !(a.dbg & 2)) {
        if constexpr (D3) hs.load(a, tc.b, (cc + 1) % nck, tc.d0 + (cc + 1) / nck - a.PDD);
        else hs.load(a, tc.b, cc + 1);
      }   // in flight during this chunk's taps
      __syncthreads();
    };
    load_wf(std::integral_constant<int, 0>(), cc_begin, 0);
    if constexpr (D3) hs.load(a, tc.b, cc_begin % nck, tc.d0 + cc_begin / nck - a.PDD);
    else hs.load(a, tc.b, cc_begin);
    // chunks in pairs so every register-buffer index is static (parity 0, then 1)
    int cc = cc_begin;
    for (; cc + 1 < cc_end; cc += 2) {
      stage(cc);
      chunk(std::integral_constant<int, 0>(), cc);
      stage(cc + 1);
      chunk(std::integral_constant<int, 1>(), cc + 1);
    }
    if (cc < cc_end) {
      stage(cc);
      chunk(std::integral_constant<int, 0>(), cc);
    }
    if (tsb && tid == 0) tsb[37] = wall_clock64();
    conv_epilogue<TM, TN, D3>(a, acc, tc, wm, wn, lane, partial);
    if (tsb && tid == 0) {
      tsb[38] = wall_clock64();
      tsb[39] = (static_cast<unsigned long long>(cc_end - cc_begin) << 32) | blockIdx.x;
    }
  };

  const TileCoord tc = decode_tile<BM, TR, D3>(a);
  const int c0 = tc.split * a.kpc;
  segment(tc, c0, min(nq, c0 + a.kpc), a.nsplit > 1);
}

// Sums the split-K partials in split order (deterministic) and applies the epilogue.
__global__ __launch_bounds__(256) void conv_split_reduce_kernel(HaloArgs a) {
  const long long SP = a.cstride;
  const long long n = static_cast<long long>(a.B) * a.Cout * SP;
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const long long sp = i % SP;
  const int co = static_cast<int>((i / SP) % a.Cout);
  const int b = static_cast<int>(i / (SP * a.Cout));
  float v = 0.f;
  for (int k = 0; k < a.nsplit; ++k) v += a.ws[k * n + i];
  store_out(a, v, co, b, sp);
}

// Vector form (D*H*W % 4 == 0): one (b, co) channel per blockIdx.y, float4 partial loads, all
// nsplit of them in flight before the ordered sum.
__global__ __launch_bounds__(256) void conv_split_reduce4_kernel(HaloArgs a) {
  const long long SP = a.cstride;
  const long long hw = (static_cast<long long>(blockIdx.x) * 256 + threadIdx.x) * 4;
  if (hw >= SP) return;
  const int plane = blockIdx.y, co = plane % a.Cout, b = plane / a.Cout;
  const size_t n = static_cast<size_t>(a.B) * a.Cout * SP;
  const float* src = a.ws + static_cast<size_t>(plane) * SP + hw;
  float4 p[8];
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (k < a.nsplit) p[k] = *reinterpret_cast<const float4*>(src + k * n);
  float4 v = p[0];
#pragma unroll
  for (int k = 1; k < 8; ++k)
    if (k < a.nsplit) { v.x += p[k].x; v.y += p[k].y; v.z += p[k].z; v.w += p[k].w; }
  if ((a.act <= 2 || a.act == 6) && !a.res) {      // plain epilogue: vector store
    const float bb = a.bias ? a.bias[co] : 0.f;
    const float gg = a.gamma ? a.gamma[co] : 1.f;
    float r[4] = {v.x + bb, v.y + bb, v.z + bb, v.w + bb};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (a.act == 1) r[k] = fmaxf(r[k], 0.f);
      else if (a.act == 2) r[k] = gelu_erf_h(r[k]);
      else if (a.act == 6) r[k] = r[k] >= 0.f ? r[k] : 0.01f * r[k];
      r[k] *= a.alpha;
      if (a.gamma) r[k] *= gg;
    }
    *reinterpret_cast<float4*>(a.out + b * a.out_bstride + static_cast<size_t>(a.co0 + co) * SP + hw) =
        make_float4(r[0], r[1], r[2], r[3]);
    return;
  }
  const float sv[4] = {v.x, v.y, v.z, v.w};
  store4(a, sv, co, b, hw, a.out, a.bias, a.gamma, a.res, a.gh, a.gz, a.gatt, a.grh);
}

template <int KS, int BM, int TR, int WM>
void tile_counts(HaloArgs& a) {
  a.nrt = (a.H + TR - 1) / TR;
  a.nct = (a.W + 31) / 32;
  a.npix = a.B * a.D * a.nrt * a.nct;
  a.nco = (a.Cout + BM - 1) / BM;
}

// D3OK false: 2D-only tile (its volume variant spills -- 464 B/lane for 128x8x32 -- and faulted)
template <int KS, int BM, int TR, int WM, bool WREG, bool D3OK = true>
int launch_halo(HaloArgs a, hipStream_t s) {
  const bool d3 = a.D > 1 || a.KD > 1;
  const unsigned grid = static_cast<unsigned>(a.npix) * a.nco * a.nsplit;
  if constexpr (WREG && !D3OK) {
    FSMI_CHECK_ARG(!d3, "fsmi_conv_halo: tile %dx%dx32 is 2D only", BM, TR);
    hipLaunchKernelGGL((conv_halo_wreg_kernel<KS, BM, TR, WM, false>), dim3(grid), dim3(256), 0, s, a);
  } else if constexpr (WREG) {
    if (d3) hipLaunchKernelGGL((conv_halo_wreg_kernel<KS, BM, TR, WM, true>), dim3(grid), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((conv_halo_wreg_kernel<KS, BM, TR, WM, false>), dim3(grid), dim3(256), 0, s, a);
  } else {
    if (d3) hipLaunchKernelGGL((conv_halo_x3_kernel<KS, BM, TR, WM, true>), dim3(grid), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((conv_halo_x3_kernel<KS, BM, TR, WM, false>), dim3(grid), dim3(256), 0, s, a);
  }
  if (a.nsplit > 1) {
    const long long SP = a.cstride;
    const bool vec = SP % 4 == 0 && a.nsplit <= 8 && reinterpret_cast<uintptr_t>(a.out) % 16 == 0 &&
                     reinterpret_cast<uintptr_t>(a.ws) % 16 == 0 &&
                     (!a.res || reinterpret_cast<uintptr_t>(a.res) % 16 == 0);
    if (vec) {
      hipLaunchKernelGGL(conv_split_reduce4_kernel, dim3(static_cast<unsigned>((SP / 4 + 255) / 256), a.B * a.Cout),
                         dim3(256), 0, s, a);
    } else {
      const long long n = static_cast<long long>(a.B) * a.Cout * SP;
      hipLaunchKernelGGL(conv_split_reduce_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s,
                         a);
    }
  }
  return finish_launch("fsmi_conv2d_halo_x3");
}

}  // namespace
}  // namespace fsmi

using namespace fsmi;

namespace {

unsigned long long* g_conv_ts = nullptr;

// Shared host side of both entry points: validates, fills HaloArgs (gate fields preset by the
// caller), picks tiles and split-K, launches.
int run_halo(HaloArgs& a, const char* what, const float* const* seg_ptr, const int* seg_ch, const int* seg_ctot,
             int nseg, const void* whi, const void* wlo, int wexp, const float* bias, float* out, int out_ctot,
             int co0, int B, int Cout, int KS, int H, int W, int cfg, int nsplit, float* ws, long long ws_floats,
             void* stream, int D = 1, int KD = 1) {
  FSMI_CHECK_ARG(seg_ptr && seg_ch && seg_ctot && whi && wlo, "%s: null pointer", what);
  FSMI_CHECK_ARG(nseg >= 1 && nseg <= kHMaxSeg, "%s: 1..%d segments, got %d", what, kHMaxSeg, nseg);
  FSMI_CHECK_ARG(B > 0 && Cout > 0 && H > 0 && W > 0, "%s: bad shape", what);
  FSMI_CHECK_ARG(KS == 1 || KS == 3, "%s: kernel %d unsupported (1, 3)", what, KS);
  FSMI_CHECK_ARG(D >= 1 && KD >= 1 && KD % 2 == 1, "%s: depth %d / depth kernel %d (odd)", what, D, KD);
  FSMI_CHECK_ARG(a.act == 3 || (out && co0 >= 0 && co0 + Cout <= out_ctot), "%s: output slice outside the tensor",
                 what);
  int cin = 0;
  const long long HW = static_cast<long long>(D) * H * W;     // channel stride
  a.D = D;
  a.KD = KD;
  a.PDD = KD / 2;
  a.cstride = HW;
  for (int i = 0; i < nseg; ++i) {
    FSMI_CHECK_ARG(seg_ptr[i] && seg_ch[i] > 0 && seg_ctot[i] >= seg_ch[i], "%s: bad segment %d", what, i);
    FSMI_CHECK_ARG(i == nseg - 1 || seg_ch[i] % 8 == 0,
                   "%s: inner segments must be multiples of 8 channels (segment %d: %d)", what, i, seg_ch[i]);
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
  a.out = out;
  a.out_bstride = static_cast<long long>(out_ctot) * HW;
  a.co0 = co0;
  a.Cout = Cout;
  a.CoutP = (Cout + 31) / 32 * 32;
  a.B = B;
  a.H = H;
  a.W = W;
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_CONV2D, s);
  // default tiles, measured per layer shape (tools/conv_bench.py --all-cfg): 3x3 layers run best
  // with register-resident weights and two pixel fragments per wave (cfg 3; cfg 2 / 5 for narrow
  // outputs); 1x1 layers -- one tap per chunk, too little MFMA work to cover a load issued a
  // chunk ahead -- with one fragment per wave, which buys a third resident wave per SIMD (cfg 4)
  if (cfg < 0) {
    if (Cout <= 32) cfg = 6;
    else if (KS == 3) cfg = Cout > 64 ? 3 : (a.Cin <= 64 ? 5 : 2);
    else cfg = Cout > 64 ? 4 : 5;
  }
  FSMI_CHECK_ARG(cfg >= 0 && cfg <= 9, "%s: cfg %d (0..9)", what, cfg);
  switch (cfg) {                                  // tile = couts x (rows x 32 px)
    case 0: case 2: tile_counts<3, 64, 8, 1>(a); break;
    case 1: case 3: tile_counts<3, 128, 4, 2>(a); break;
    case 4: tile_counts<3, 128, 2, 2>(a); break;
    case 5: tile_counts<3, 64, 4, 1>(a); break;
    case 6: tile_counts<3, 32, 8, 1>(a); break;
    case 8: tile_counts<3, 128, 8, 2>(a); break;
    case 9: tile_counts<3, 256, 4, 4>(a); break;
    default: tile_counts<3, 32, 4, 1>(a); break;
  }
  const int nck = KD * a.CinP / HKC;               // split-K runs over (kd, channel chunk) pairs
  const long long per_split = static_cast<long long>(B) * Cout * HW;
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
                 "%s: split-K %d needs %lld workspace floats", what, a.nsplit, per_split * a.nsplit);
  a.ws = ws;
  a.ts = g_conv_ts;
  static const int conv_dbg = [] {
    const char* e = std::getenv("FSMI_CONV_DBG");
    return e ? std::atoi(e) : 0;
  }();
  a.dbg = conv_dbg;
  if (KS == 3) {
    switch (cfg) {
      case 0: return launch_halo<3, 64, 8, 1, false>(a, s);
      case 1: return launch_halo<3, 128, 4, 2, false>(a, s);
      case 2: return launch_halo<3, 64, 8, 1, true>(a, s);
      case 3: return launch_halo<3, 128, 4, 2, true>(a, s);
      case 4: return launch_halo<3, 128, 2, 2, true>(a, s);
      case 5: return launch_halo<3, 64, 4, 1, true>(a, s);
      case 6: return launch_halo<3, 32, 8, 1, true>(a, s);
      case 8: return launch_halo<3, 128, 8, 2, true, false>(a, s);
      case 9: return launch_halo<3, 256, 4, 4, true, false>(a, s);
      default: return launch_halo<3, 32, 4, 1, true>(a, s);
    }
  }
  switch (cfg) {
    case 0: return launch_halo<1, 64, 8, 1, false>(a, s);
    case 1: return launch_halo<1, 128, 4, 2, false>(a, s);
    case 2: return launch_halo<1, 64, 8, 1, true>(a, s);
    case 3: return launch_halo<1, 128, 4, 2, true>(a, s);
    case 4: return launch_halo<1, 128, 2, 2, true>(a, s);
    case 5: return launch_halo<1, 64, 4, 1, true>(a, s);
    case 6: return launch_halo<1, 32, 8, 1, true>(a, s);
    case 8: return launch_halo<1, 128, 8, 2, true, false>(a, s);
    case 9: return launch_halo<1, 256, 4, 4, true, false>(a, s);
    default: return launch_halo<1, 32, 4, 1, true>(a, s);
  }
}

}  // namespace

// Debug: while buf is non-NULL every halo conv launch records, per block, thread 0's wall clock
// (100 MHz) at start [0], at each chunk's staging barrier [1..36], before / after the epilogue
// [37] / [38] and (chunks << 32 | block) [39] into buf[block * 40 ..] (tools/conv_phases.py).
extern "C" int fsmi_debug_conv_timestamps(unsigned long long* buf) {
  g_conv_ts = buf;
  return FSMI_OK;
}

extern "C" int fsmi_conv2d_halo_x3(const float* const* seg_ptr, const int* seg_ch, const int* seg_ctot, int nseg,
                                   const void* whi, const void* wlo, int wexp, const float* bias, const float* gamma,
                                   const float* res, int res_ctot, float* out, int out_ctot, int co0, int B, int Cout,
                                   int KS, int H, int W, int act, float alpha, int cfg, int nsplit, float* ws,
                                   long long ws_floats, void* stream) {
  FSMI_CHECK_ARG(out, "fsmi_conv2d_halo_x3: null output");
  FSMI_CHECK_ARG((act >= 0 && act <= 2) || act == 6, "fsmi_conv2d_halo_x3: act %d (0, 1, 2, 6)", act);
  HaloArgs a{};
  a.act = act;
  a.alpha = alpha;
  a.gamma = gamma;
  a.res = res;
  a.res_bstride = static_cast<long long>(res_ctot) * H * W;
  return run_halo(a, "fsmi_conv2d_halo_x3", seg_ptr, seg_ch, seg_ctot, nseg, whi, wlo, wexp, bias, out, out_ctot,
                  co0, B, Cout, KS, H, W, cfg, nsplit, ws, ws_floats, stream);
}

extern "C" int fsmi_conv2d_halo_x3_gate(const float* const* seg_ptr, const int* seg_ch, const int* seg_ctot,
                                        int nseg, const void* whi, const void* wlo, int wexp, const float* bias,
                                        int mode, const float* h, float* z, const float* att, float* rh, int Hd,
                                        float* out, int out_ctot, int co0, int B, int Cout, int KS, int H, int W,
                                        int cfg, int nsplit, float* ws, long long ws_floats, void* stream) {
  FSMI_CHECK_ARG(mode >= 0 && mode <= 2, "fsmi_conv2d_halo_x3_gate: mode %d (0 zr, 1 small, 2 large)", mode);
  FSMI_CHECK_ARG(h && z && Hd > 0, "fsmi_conv2d_halo_x3_gate: null h / z");
  FSMI_CHECK_ARG(mode != 0 || (rh && Cout == 2 * Hd), "fsmi_conv2d_halo_x3_gate: zr needs rh and Cout == 2*Hd");
  FSMI_CHECK_ARG(mode == 0 || (att && out && Cout == Hd), "fsmi_conv2d_halo_x3_gate: blend needs att, out, Cout == Hd");
  HaloArgs a{};
  a.act = 3 + mode;
  a.alpha = 1.f;
  a.gh = h;
  a.gz = z;
  a.gatt = att;
  a.grh = rh;
  a.gHd = Hd;
  return run_halo(a, "fsmi_conv2d_halo_x3_gate", seg_ptr, seg_ch, seg_ctot, nseg, whi, wlo, wexp, bias, out,
                  out_ctot, co0, B, Cout, KS, H, W, cfg, nsplit, ws, ws_floats, stream);
}

extern "C" int fsmi_conv3d_halo_x3(const float* x, int Cin, const void* whi, const void* wlo, int wexp,
                                   const float* bias, const float* res, float* out, int B, int Cout, int D, int H,
                                   int W, int KD, int KS, int act, int res_pre, int cfg, int nsplit, float* ws,
                                   long long ws_floats, void* stream) {
  FSMI_CHECK_ARG(x && out && Cin > 0, "fsmi_conv3d_halo_x3: null pointer / channels");
  FSMI_CHECK_ARG(act == 0 || act == 1 || act == 6, "fsmi_conv3d_halo_x3: act %d (0 none, 1 ReLU, 6 LeakyReLU)", act);
  HaloArgs a{};
  a.act = act;
  a.alpha = 1.f;
  a.res = res;
  a.res_pre = res_pre;
  a.res_bstride = static_cast<long long>(Cout) * D * H * W;
  const float* seg[1] = {x};
  const int ch[1] = {Cin}, tot[1] = {Cin};
  return run_halo(a, "fsmi_conv3d_halo_x3", seg, ch, tot, 1, whi, wlo, wexp, bias, out, Cout, 0, B, Cout, KS, H, W,
                  cfg, nsplit, ws, ws_floats, stream, D, KD);
}
