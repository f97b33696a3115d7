// EdgeNeXt inverted-bottleneck MLP in one kernel (DispHead's two EdgeNextConvEncoder blocks,
// core/submodule.py:578-591 via core/update.py:24-31):
//     out = res + gamma * (W2 . gelu(W1 . x + b1) + b2)          x = dwconv(input), per pixel
// with W1 (4C x C) and W2 (C x 4C) the pwconv1 / pwconv2 Linear layers.
//
// The two-kernel form (pwconv1 with a GELU epilogue, then pwconv2 with the gamma / residual
// epilogue) writes the 4C-channel GELU map to HBM and reads it back (2 x 39 MB per block at cfg2),
// and each 1x1 kernel re-splits its input into fp16 hi / lo per cout tile.  Here a block owns
// PX = 64 consecutive pixels of one image and all channels:
//   * x tile (C x 64 fp32) -> one split into an LDS [pixel][channel] hi / lo image, scaled by the
//     exact power of two that puts the tile's max |x| in [2^14, 2^15) (no headroom guess: the whole
//     tile is known before the split, so nothing can overflow fp16);
//   * GEMM 1 on MFMA (3 products per MAC, as the conv tiles): 8 waves x (64 hidden x 64 px),
//     bias + exact GELU on the accumulators, then the block's max |h| and one split of the hidden
//     tile into a second, 4C-wide hi / lo image that overwrites the first (same LDS);
//   * GEMM 2: 8 waves x (32 out x 32 px), K = 4C, two accumulators per wave (even / odd k-steps)
//     so consecutive MFMAs are independent; epilogue res + gamma * (v + b2), stored once.
// One block of 8 waves per CU (139 KB of LDS).  A 4-wave variant staging the hidden map a quarter at
// a time (75 KB, two blocks per CU) was faster alone (40 vs 50 us at cfg2) but slower in the step
// (48.0-48.6 vs 47.8 ms): its longer-lived blocks hold CUs the concurrent streams' convs need.
// HBM traffic per pixel: x, res and out, C floats each -- the hidden map never leaves the CU.
// Weights: the halo kernels' pre-split packing (ops.PackedConv, [cin chunk][cout][32] hi / lo, rows
// scaled by 2^wexp[co] with (2^-wexp, bias) pairs), read from L2 one chunk ahead.
#include "conv_halo.h"

namespace fsmi {
namespace {

constexpr int kMlpPX = 64;
constexpr int kMlpWaves = 8;

struct MlpArgs {
  const float* x;                  // (B, C, HW): dwconv output
  const float* res;                // (B, C, HW): block input (may alias out)
  float* out;                      // (B, C, HW)
  const _Float16* w1h;             // [C/32][E][32]
  const _Float16* w1l;
  const float2* sb1;               // E pairs (2^-wexp, b1)
  const _Float16* w2h;             // [E/32][C][32]
  const _Float16* w2l;
  const float2* sb2;               // C pairs (2^-wexp, b2)
  const float* gamma;              // C or nullptr
  int B, HW, tiles;
  unsigned long long* ts;          // debug (fsmi_debug_conv_timestamps): 8 phase stamps per block
  unsigned long long* clk;         // in-kernel launch clock (nullptr: off)
};

// gelu_erf_h (conv_halo.h, FSMI_GELU_FAST) on two values at once: the same operations in the same
// order on <2 x float>, so the fma / mul / add chains issue as packed v_pk_* instructions (two per
// lane per issue) and every result is bit-identical to the scalar form.  The GELU of the 4C x 64
// hidden tile is the kernel's largest VALU phase (~30 operations per element, more issue cycles per
// block than its MFMAs).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 gelu_erf_h2(f32x2 x) {
#if FSMI_GELU_FAST
  const f32x2 z = x * 0.70710678118654752f;
  const f32x2 t = z * z;
  f32x2 p = 7.847259258e-05f;
  p = fma2(p, t, -8.008189034e-04f);
  p = fma2(p, t, 5.188099109e-03f);
  p = fma2(p, t, -2.685369179e-02f);
  p = fma2(p, t, 1.128358245e-01f);
  p = fma2(p, t, -3.761262596e-01f);
  p = fma2(p, t, 1.128379107e+00f);
  const f32x2 small = z * p;
  const f32x2 az = {fminf(fabsf(z.x), 4.f), fminf(fabsf(z.y), 4.f)};
  f32x2 r = 1.498133884e-06f;
  r = fma2(r, az, -4.378752783e-05f);
  r = fma2(r, az, 5.791864241e-04f);
  r = fma2(r, az, -4.594380967e-03f);
  r = fma2(r, az, 2.443690039e-02f);
  r = fma2(r, az, -9.241911769e-02f);
  r = fma2(r, az, 2.575692832e-01f);
  r = fma2(r, az, -5.418152213e-01f);
  r = fma2(r, az, 8.737412691e-01f);
  r = fma2(r, az, -1.082139969e+00f);
  r = fma2(r, az, 9.922678471e-01f);
  const f32x2 m = -t * 1.4426950408889634f;
  const f32x2 e = {__builtin_amdgcn_exp2f(m.x), __builtin_amdgcn_exp2f(m.y)};
  const f32x2 g = fma2(-e, r, 1.f);
  const f32x2 big = {copysignf(g.x, z.x), copysignf(g.y, z.y)};
  const f32x2 erf = {fabsf(z.x) < 1.f ? small.x : big.x, fabsf(z.y) < 1.f ? small.y : big.y};
  return 0.5f * x * (1.f + erf);
#else
  return f32x2{gelu_erf_h(x.x), gelu_erf_h(x.y)};
#endif
}

// max over the block of per-thread values v >= 0 (8 waves); one barrier
__device__ __forceinline__ float block_max8(float v, float* red, int lane, int wave) {
  const float m = wave_max(v);
  if (lane == 0) red[wave] = m;
  __syncthreads();
  const float4 r0 = *reinterpret_cast<const float4*>(red);
  const float4 r1 = *reinterpret_cast<const float4*>(red + 4);
  return fmaxf(fmaxf(fmaxf(r0.x, r0.y), fmaxf(r0.z, r0.w)), fmaxf(fmaxf(r1.x, r1.y), fmaxf(r1.z, r1.w)));
}

// phase stamp k of this block (lane 0 of wave FSMI_MLP_STAMP_WAVE) when the debug buffer is set
#ifndef FSMI_MLP_STAMP_WAVE
#define FSMI_MLP_STAMP_WAVE 0
#endif
__device__ __forceinline__ void mlp_stamp(const MlpArgs& a, int k) {
  if (a.ts && threadIdx.x == 64 * FSMI_MLP_STAMP_WAVE) a.ts[static_cast<size_t>(blockIdx.x) * 8 + k] = wall_clock64();
}


template <int C>
__global__ __launch_bounds__(512) void edgenext_mlp_kernel(MlpArgs a) {
  FSMI_TIMELINE_CLOCK(a.clk);
  constexpr int E = 4 * C, PX = kMlpPX;
  constexpr int XR = C + 8, HR = E + 8;            // padded LDS rows (halves): 16-B aligned, 4-bank skew
  constexpr int NKX = C / HKC, NKH = E / HKC;      // 32-channel chunks of x / of the hidden map
  constexpr int TM1 = E / 32 / kMlpWaves;          // GEMM 1 row fragments per wave (all 64 px: 2 cols)
  static_assert(C % HKC == 0 && TM1 >= 1 && C / 32 * 2 == kMlpWaves, "edgenext_mlp: C = 128");
  // hi image then lo image; the x images (PX x XR) alias the front of the hidden images
  __shared__ __attribute__((aligned(16))) _Float16 img[2 * PX * HR];
  __shared__ __attribute__((aligned(16))) float red[kMlpWaves];
  __shared__ __attribute__((aligned(16))) float2 lsb1[E];      // GEMM 1 epilogue (2^-wexp, b1)
  __shared__ __attribute__((aligned(16))) float2 lsb2[C];      // GEMM 2 epilogue (2^-wexp, b2)
  __shared__ __attribute__((aligned(16))) float lg[C];         // gamma
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hsel = lane >> 5, rl = lane & 31;
  const int b = blockIdx.x / a.tiles;
  const int p0 = (blockIdx.x - b * a.tiles) * PX;
  const long long HW = a.HW;
  mlp_stamp(a, 0);

  // W1 fragments of the first two chunks, issued first: their L2 round trip overlaps the x tile's
  const int hrow0 = wave * 32 * TM1;
  half8 w1f[2][TM1][2][2];                         // [ring slot][i][k half][hi, lo]
  auto load_w1 = [&](int slot, int c) FSMI_HALO_INL {
#pragma unroll
    for (int i = 0; i < TM1; ++i)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const size_t o = (static_cast<size_t>(c) * E + hrow0 + i * 32 + rl) * HKC + 16 * k + 8 * hsel;
        w1f[slot][i][k][0] = *reinterpret_cast<const half8*>(a.w1h + o);
        w1f[slot][i][k][1] = *reinterpret_cast<const half8*>(a.w1l + o);
      }
  };
  load_w1(0, 0);
  if (NKX > 1) load_w1(1, 1);
  // epilogue coefficients to LDS (visible after the first barrier below)
  for (int e = tid; e < E; e += 512) lsb1[e] = a.sb1[e];
  if (tid < C) {
    lsb2[tid] = a.sb2[tid];
    lg[tid] = a.gamma ? a.gamma[tid] : 1.f;
  }

  // ---- x tile -> scaled hi / lo [pixel][channel] image
  _Float16(*Xh)[XR] = reinterpret_cast<_Float16(*)[XR]>(img);
  _Float16(*Xl)[XR] = reinterpret_cast<_Float16(*)[XR]>(img + PX * XR);
  constexpr int XT = PX * (C / 8) / 512;           // 8-channel tasks per thread
  f32x8 xv[XT];
  float mx = 0.f;
#pragma unroll
  for (int u = 0; u < XT; ++u) {
    const int task = u * 512 + tid, px = task % PX, g = task / PX;
    const bool ok = p0 + px < HW;        // tail pixels load the last one (no branch) and drop it
    const float* src = a.x + (static_cast<size_t>(b) * C + 8 * g) * HW + min(p0 + px, static_cast<int>(HW) - 1);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float v = src[static_cast<size_t>(t) * HW];
      xv[u][t] = ok ? v : 0.f;
      mx = fmaxf(mx, fabsf(xv[u][t]));
    }
  }
  const int sx = __builtin_amdgcn_readfirstlane(chunk_exp(block_max8(mx, red, lane, wave)));
  mlp_stamp(a, 1);
  const float xs = exp2i(sx == kNoExp ? 0 : sx);
#pragma unroll
  for (int u = 0; u < XT; ++u) {
    const int task = u * 512 + tid, px = task % PX, g = task / PX;
    const f32x8 v = xv[u] * xs;
    const half8 hi = __builtin_convertvector(v, half8);
    *reinterpret_cast<half8*>(&Xh[px][8 * g]) = hi;
    if constexpr (FSMI_NPROD == 3)
      *reinterpret_cast<half8*>(&Xl[px][8 * g]) = __builtin_convertvector(v - __builtin_convertvector(hi, f32x8), half8);
  }
  __syncthreads();

  // ---- GEMM 1: hidden rows [wave * 32 * TM1, +32 * TM1) x 64 px, K = C
  f32x16 acc1[TM1][2];
#pragma unroll
  for (int i = 0; i < TM1; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc1[i][j][r] = 0.f;
  {
#pragma unroll
    for (int c = 0; c < NKX; ++c) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        half8 ah[TM1], al[TM1], bh[2], bl[2];
#pragma unroll
        for (int i = 0; i < TM1; ++i) {
          ah[i] = w1f[c & 1][i][k][0];
          al[i] = w1f[c & 1][i][k][1];
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          bh[j] = *reinterpret_cast<const half8*>(&Xh[j * 32 + rl][c * HKC + 16 * k + 8 * hsel]);
          if constexpr (FSMI_NPROD == 3) bl[j] = *reinterpret_cast<const half8*>(&Xl[j * 32 + rl][c * HKC + 16 * k + 8 * hsel]);
        }
        mma3<TM1, 2>(acc1, ah, al, bh, bl);
      }
      if (c + 2 < NKX) load_w1(c & 1, c + 2);
    }
  }
  // W2 fragments of the first kRing chunks of GEMM 2, issued before the GELU (whose VALU hides them)
  const int m2 = wave & 3, n2 = wave >> 2;
  constexpr int kRing = 3;
  half8 w2f[kRing][2][2];                          // [ring slot][k half][hi, lo]
  auto load_w2 = [&](int slot, int c) FSMI_HALO_INL {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const size_t o = (static_cast<size_t>(c) * C + m2 * 32 + rl) * HKC + 16 * k + 8 * hsel;
      w2f[slot][k][0] = *reinterpret_cast<const half8*>(a.w2h + o);
      w2f[slot][k][1] = *reinterpret_cast<const half8*>(a.w2l + o);
    }
  };
#pragma unroll
  for (int c = 0; c < kRing; ++c) load_w2(c, c);
  mlp_stamp(a, 2);
  // bias + GELU in place; row of element r of fragment i: hrow0 + 32 i + (r & 3) + 8 (r >> 2) + 4 hsel
  const float xinv = exp2i(sx == kNoExp ? 0 : -sx);
  float hm = 0.f;
#pragma unroll
  for (int i = 0; i < TM1; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float2 q = lsb1[hrow0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hsel];
      // the two pixel fragments' elements share the row's coefficients: one packed GELU
      const f32x2 v = fma2(f32x2{acc1[i][0][r], acc1[i][1][r]}, q.x * xinv, q.y);
      const f32x2 h = gelu_erf_h2(v);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        acc1[i][j][r] = (p0 + j * 32 + rl < HW) ? h[j] : 0.f;     // tail pixels: no effect on the max
        hm = fmaxf(hm, fabsf(acc1[i][j][r]));
      }
    }
  // the barrier inside block_max8 also retires every wave's reads of the x image, which the
  // hidden image overwrites next
  mlp_stamp(a, 3);
  const int sh = __builtin_amdgcn_readfirstlane(chunk_exp(block_max8(hm, red, lane, wave)));
  mlp_stamp(a, 4);
  const float hs = exp2i(sh == kNoExp ? 0 : sh);
  _Float16(*Hh)[HR] = reinterpret_cast<_Float16(*)[HR]>(img);
  _Float16(*Hl)[HR] = reinterpret_cast<_Float16(*)[HR]>(img + PX * HR);
#pragma unroll
  for (int i = 0; i < TM1; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {             // rows hrow0 + 32 i + 8 q4 + 4 hsel + (0..3)
        typedef float f32x4 __attribute__((ext_vector_type(4)));
        typedef _Float16 half4 __attribute__((ext_vector_type(4)));
        f32x4 v;
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = acc1[i][j][4 * q4 + t] * hs;
        const half4 hi = __builtin_convertvector(v, half4);
        const int px = j * 32 + rl, row = hrow0 + 32 * i + 8 * q4 + 4 * hsel;
        *reinterpret_cast<half4*>(&Hh[px][row]) = hi;
        if constexpr (FSMI_NPROD == 3)
          *reinterpret_cast<half4*>(&Hl[px][row]) = __builtin_convertvector(v - __builtin_convertvector(hi, f32x4), half4);
      }
  __syncthreads();

  mlp_stamp(a, 5);
  // ---- GEMM 2: out rows [32 m2, +32) x px [32 n2, +32), K = E; even / odd k-steps accumulate apart;
  // weights kRing chunks ahead in registers (one chunk's 6 MFMAs are ~200 cycles, an L2 trip ~700)
  f32x16 acc2[2][1][1];
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc2[e][0][0][r] = 0.f;
#pragma unroll
  for (int c = 0; c < NKH; ++c) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      half8 ah[1] = {w2f[c % kRing][k][0]}, al[1] = {w2f[c % kRing][k][1]}, bh[1], bl[1];
      bh[0] = *reinterpret_cast<const half8*>(&Hh[n2 * 32 + rl][c * HKC + 16 * k + 8 * hsel]);
      if constexpr (FSMI_NPROD == 3) bl[0] = *reinterpret_cast<const half8*>(&Hl[n2 * 32 + rl][c * HKC + 16 * k + 8 * hsel]);
      mma3<1, 1>(acc2[k], ah, al, bh, bl);
    }
    if (c + kRing < NKH) load_w2(c % kRing, c + kRing);
  }
  mlp_stamp(a, 6);
  // epilogue: out = res + gamma * (v * 2^-wexp * 2^-sh + b2)
  const int px = p0 + n2 * 32 + rl;
  if (px < HW) {
    const float hinv = exp2i(sh == kNoExp ? 0 : -sh);
    const size_t base = static_cast<size_t>(b) * C * HW + px;
    float rv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) rv[r] = a.res[base + static_cast<size_t>(m2 * 32 + (r & 3) + 8 * (r >> 2) + 4 * hsel) * HW];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = m2 * 32 + (r & 3) + 8 * (r >> 2) + 4 * hsel;
      const float2 q = lsb2[co];
      const float g = lg[co];
      const float v = (acc2[0][0][0][r] + acc2[1][0][0][r]) * (q.x * hinv) + q.y;
      a.out[base + static_cast<size_t>(co) * HW] = rv[r] + g * v;
    }
  }
  mlp_stamp(a, 7);
}


}  // namespace
}  // namespace fsmi

using namespace fsmi;

extern unsigned long long* g_conv_ts;   // conv_halo_x3.hip: fsmi_debug_conv_timestamps

extern "C" int fsmi_edgenext_mlp(const float* x, const float* res, float* out, const void* w1hi, const void* w1lo,
                                 const float* sb1, const void* w2hi, const void* w2lo, const float* sb2,
                                 const float* gamma, int B, int C, int E, int H, int W, void* stream) {
  FSMI_CHECK_ARG(x && res && out && w1hi && w1lo && sb1 && w2hi && w2lo && sb2, "fsmi_edgenext_mlp: null pointer");
  FSMI_CHECK_ARG(C == 128 && E == 4 * C, "fsmi_edgenext_mlp: built for C = 128, E = 4C (C=%d, E=%d)", C, E);
  FSMI_CHECK_ARG(B > 0 && H > 0 && W > 0, "fsmi_edgenext_mlp: bad shape");
  FSMI_CHECK_ARG(x != out, "fsmi_edgenext_mlp: out must not alias x");
  MlpArgs a;
  a.x = x;
  a.res = res;
  a.out = out;
  a.w1h = static_cast<const _Float16*>(w1hi);
  a.w1l = static_cast<const _Float16*>(w1lo);
  a.sb1 = reinterpret_cast<const float2*>(sb1);
  a.w2h = static_cast<const _Float16*>(w2hi);
  a.w2l = static_cast<const _Float16*>(w2lo);
  a.sb2 = reinterpret_cast<const float2*>(sb2);
  a.gamma = gamma;
  a.B = B;
  a.HW = H * W;
  a.tiles = (a.HW + kMlpPX - 1) / kMlpPX;
  a.ts = g_conv_ts;
  hipStream_t s = as_stream(stream);
  a.clk = clock_slot(FSMI_K_CONV2D, s, 8ll * B * a.tiles, "edgenext_mlp", true);
  LaunchTimer t(FSMI_K_CONV2D, s);
  hipLaunchKernelGGL(edgenext_mlp_kernel<128>, dim3(static_cast<unsigned>(B * a.tiles)), dim3(512), 0, s, a);
  return finish_launch("fsmi_edgenext_mlp");
}
