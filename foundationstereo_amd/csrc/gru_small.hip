// SelectiveConvGRU's small (1x1) GRU branch in one kernel (core/update.py:83-95, RaftConvGRU with
// kernel_size 1, weighted by att as at :117):
//     z = sigmoid(convz(hx)),  r = sigmoid(convr(hx)),  q = tanh(convq(cat[r * h, x]))
//     out = ((1 - z) h + z q) * att
// with hx = relu(conv1(cat[x, h])) (K channels, K = Hd + Cx) and x = conv0's output (Cx channels).
//
// The two-launch form (the zr conv with a gate epilogue writing z and r*h, then the q conv reading
// [r*h, x] as two segments with the blend epilogue) ran both 1x1 convs on 3x3 halo tiles at 3-13 % of
// the MFMA rate (`conv_halo_pipe_kernel<1,256,5,4>`, 21 VALU per MFMA) and moved z and r*h
// through HBM.  Here a block owns PX = 64 consecutive pixels of one image, as edgenext_mlp.hip:
//   * the hx tile (K x 64 fp32) -> one split into an LDS [pixel][channel] hi / lo image, scaled by the
//     exact power of two that puts the tile's max |hx| in [2^14, 2^15) (the whole tile is known before
//     the split: nothing can overflow fp16);
//   * GEMM 1 on MFMA (3 products per MAC): wave (m, n) computes z rows [32 m, +32) AND r rows
//     [Hd + 32 m, +32) of pixel fragment n, so the gate, r * h and -- after GEMM 2 -- the blend of
//     those (channel, pixel) elements all stay in that wave's registers (h, att loaded once);
//   * GEMM 2's input image [r*h | x] overwrites the hx image: r*h from the waves' registers, x from
//     HBM (loaded under GEMM 1), one exact exponent for the pair; wave (m, n) computes q rows
//     [32 m, +32) of pixel fragment n, two accumulators (even / odd k-steps) so consecutive MFMAs are
//     independent, and writes ((1 - z) h + z tanh(q)) * att once.
// One block of 8 waves per CU (136 KB of LDS at K = 512).  Weights: the halo kernels' pre-split
// packing (ops.PackedConv, [cin chunk][cout][32] hi / lo, rows scaled by 2^wexp[co], (2^-wexp, bias)
// pairs), read from L2 kRing chunks ahead.  HBM traffic per pixel: hx, x, h, att in, out once.
#include "conv_halo.h"

namespace fsmi {
namespace {

constexpr int kGsPX = 64;
constexpr int kGsHd = 128;

struct GruSmallArgs {
  const float* hx;                 // (B, K, HW): conv1 output
  const float* xc;                 // (B, K - Hd, HW): conv0 output (the GRU's x)
  const float* h;                  // (B, Hd, HW)
  const float* att;                // (B, 1, HW)
  float* out;                      // (B, Hd, HW)
  const _Float16* wzh;             // [K/32][2 Hd][32]: convz | convr stacked
  const _Float16* wzl;
  const float2* sbz;               // 2 Hd pairs (2^-wexp, bias)
  const _Float16* wqh;             // [K/32][Hd][32]: convq, input order [r*h, x]
  const _Float16* wql;
  const float2* sbq;               // Hd pairs
  int B, HW, tiles;
  unsigned long long* clk;         // in-kernel launch clock (timeline build)
};

// max over the block of per-thread values v >= 0 (8 waves); one barrier
__device__ __forceinline__ float gs_block_max(float v, float* red, int lane, int wave) {
  const float m = wave_max(v);
  if (lane == 0) red[wave] = m;
  __syncthreads();
  const float4 r0 = *reinterpret_cast<const float4*>(red);
  const float4 r1 = *reinterpret_cast<const float4*>(red + 4);
  return fmaxf(fmaxf(fmaxf(r0.x, r0.y), fmaxf(r0.z, r0.w)), fmaxf(fmaxf(r1.x, r1.y), fmaxf(r1.z, r1.w)));
}

template <int K>
__global__ __launch_bounds__(512) void gru_small_kernel(GruSmallArgs a) {
  FSMI_TIMELINE_CLOCK(a.clk);
  constexpr int Hd = kGsHd, PX = kGsPX, NK = K / HKC, XR = K + 8, CX = K - Hd;
  constexpr int XT = PX * (K / 8) / 512;           // 8-channel hx tasks per thread
  constexpr int CT = PX * (CX / 8) / 512;          // 8-channel x tasks per thread
  static_assert(K % HKC == 0 && CX > 0 && PX * (K / 8) % 512 == 0 && PX * (CX / 8) % 512 == 0, "gru_small: K");
  __shared__ __attribute__((aligned(16))) _Float16 img[2 * PX * XR];   // hi image, then lo image
  __shared__ __attribute__((aligned(16))) float red[8];
  __shared__ __attribute__((aligned(16))) float2 lsbz[2 * Hd];
  __shared__ __attribute__((aligned(16))) float2 lsbq[Hd];
  _Float16(*Xh)[XR] = reinterpret_cast<_Float16(*)[XR]>(img);
  _Float16(*Xl)[XR] = reinterpret_cast<_Float16(*)[XR]>(img + PX * XR);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hsel = lane >> 5, rl = lane & 31;
  const int m = wave & 3, n = wave >> 2;           // rows [32 m, +32) of z / r / q, pixel fragment n
  const int b = blockIdx.x / a.tiles;
  const int p0 = (blockIdx.x - b * a.tiles) * PX;
  const int HW = a.HW;
  const int px = p0 + 32 * n + rl;                 // this lane's pixel in both epilogues
  const bool pok = px < HW;
  const int pxc = min(px, HW - 1);

  // GEMM 1 weights (z and r fragments of rows 32 m ..), kRing chunks ahead; issued first so their L2
  // round trip overlaps the hx tile's
  constexpr int kRing = 3;
  half8 w1f[kRing][2][2][2];                       // [slot][z / r][k half][hi, lo]
  auto load_w1 = [&](int slot, int c) FSMI_HALO_INL {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const size_t o = (static_cast<size_t>(c) * 2 * Hd + i * Hd + 32 * m + rl) * HKC + 16 * k + 8 * hsel;
        w1f[slot][i][k][0] = *reinterpret_cast<const half8*>(a.wzh + o);
        w1f[slot][i][k][1] = *reinterpret_cast<const half8*>(a.wzl + o);
      }
  };
#pragma unroll
  for (int c = 0; c < kRing && c < NK; ++c) load_w1(c, c);
  for (int e = tid; e < 2 * Hd; e += 512) lsbz[e] = a.sbz[e];
  if (tid < Hd) lsbq[tid] = a.sbq[tid];

  // ---- hx tile -> scaled hi / lo [pixel][channel] image
  f32x8 xv[XT];
  float mx = 0.f;
#pragma unroll
  for (int u = 0; u < XT; ++u) {
    const int task = u * 512 + tid, p = task % PX, g = task / PX;
    const bool ok = p0 + p < HW;                   // tail pixels load the last one and drop it
    const float* src = a.hx + (static_cast<size_t>(b) * K + 8 * g) * HW + min(p0 + p, HW - 1);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float v = src[static_cast<size_t>(t) * HW];
      xv[u][t] = ok ? v : 0.f;
      mx = fmaxf(mx, fabsf(xv[u][t]));
    }
  }
  // the epilogues' h (rows of this wave's fragments, this lane's pixel) and att
  float hv[16];
#pragma unroll
  for (int r = 0; r < 16; ++r)
    hv[r] = a.h[(static_cast<size_t>(b) * Hd + 32 * m + (r & 3) + 8 * (r >> 2) + 4 * hsel) * HW + pxc];
  const float at = a.att[static_cast<size_t>(b) * HW + pxc];
  const int sx = __builtin_amdgcn_readfirstlane(chunk_exp(gs_block_max(mx, red, lane, wave)));
  {
    const float xs = exp2i(sx == kNoExp ? 0 : sx);
#pragma unroll
    for (int u = 0; u < XT; ++u) {
      const int task = u * 512 + tid, p = task % PX, g = task / PX;
      const f32x8 v = xv[u] * xs;
      const half8 hi = __builtin_convertvector(v, half8);
      *reinterpret_cast<half8*>(&Xh[p][8 * g]) = hi;
      if constexpr (FSMI_NPROD == 3)
        *reinterpret_cast<half8*>(&Xl[p][8 * g]) = __builtin_convertvector(v - __builtin_convertvector(hi, f32x8), half8);
    }
  }
  __syncthreads();

  // the x tile (GEMM 2's rows [Hd, K)) into registers: its HBM round trip runs under GEMM 1
  f32x8 cv[CT];
#pragma unroll
  for (int u = 0; u < CT; ++u) {
    const int task = u * 512 + tid, p = task % PX, g = task / PX;
    const bool ok = p0 + p < HW;
    const float* src = a.xc + (static_cast<size_t>(b) * CX + 8 * g) * HW + min(p0 + p, HW - 1);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float v = src[static_cast<size_t>(t) * HW];
      cv[u][t] = ok ? v : 0.f;
    }
  }

  // ---- GEMM 1: z rows [32 m, +32) and r rows [Hd + 32 m, +32) x pixel fragment n, K = hx channels
  f32x16 acc1[2][1];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc1[i][0][r] = 0.f;
#pragma unroll
  for (int c = 0; c < NK; ++c) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      half8 ah[2], al[2], bh[1], bl[1];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ah[i] = w1f[c % kRing][i][k][0];
        al[i] = w1f[c % kRing][i][k][1];
      }
      bh[0] = *reinterpret_cast<const half8*>(&Xh[32 * n + rl][c * HKC + 16 * k + 8 * hsel]);
      if constexpr (FSMI_NPROD == 3) bl[0] = *reinterpret_cast<const half8*>(&Xl[32 * n + rl][c * HKC + 16 * k + 8 * hsel]);
      mma3<2, 1>(acc1, ah, al, bh, bl);
    }
    if (c + kRing < NK) load_w1(c % kRing, c + kRing);
  }

  // GEMM 2 weights (q rows 32 m ..), kRing chunks ahead, issued before the gate math hides them
  half8 w2f[kRing][2][2];                          // [slot][k half][hi, lo]
  auto load_w2 = [&](int slot, int c) FSMI_HALO_INL {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const size_t o = (static_cast<size_t>(c) * Hd + 32 * m + rl) * HKC + 16 * k + 8 * hsel;
      w2f[slot][k][0] = *reinterpret_cast<const half8*>(a.wqh + o);
      w2f[slot][k][1] = *reinterpret_cast<const half8*>(a.wql + o);
    }
  };
#pragma unroll
  for (int c = 0; c < kRing && c < NK; ++c) load_w2(c, c);

  // ---- gates: z = sigmoid(.), r * h (store_el act 3's arithmetic)
  const float xinv = exp2i(sx == kNoExp ? 0 : -sx);
  float zv[16], rh[16];
  float mr = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int co = 32 * m + (r & 3) + 8 * (r >> 2) + 4 * hsel;
    const float2 qz = lsbz[co], qr = lsbz[Hd + co];
    zv[r] = sigm_h(acc1[0][0][r] * xinv * qz.x + qz.y);
    rh[r] = pok ? sigm_h(acc1[1][0][r] * xinv * qr.x + qr.y) * hv[r] : 0.f;
    mr = fmaxf(mr, fabsf(rh[r]));
  }
#pragma unroll
  for (int u = 0; u < CT; ++u)
#pragma unroll
    for (int t = 0; t < 8; ++t) mr = fmaxf(mr, fabsf(cv[u][t]));
  // the barrier inside gs_block_max also retires every wave's GEMM 1 reads of the hx image
  const int s2 = __builtin_amdgcn_readfirstlane(chunk_exp(gs_block_max(mr, red, lane, wave)));
  {
    const float ys = exp2i(s2 == kNoExp ? 0 : s2);
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    typedef _Float16 half4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {               // r*h rows 32 m + 8 q4 + 4 hsel + (0..3)
      f32x4 v;
#pragma unroll
      for (int t = 0; t < 4; ++t) v[t] = rh[4 * q4 + t] * ys;
      const half4 hi = __builtin_convertvector(v, half4);
      const int row = 32 * m + 8 * q4 + 4 * hsel;
      *reinterpret_cast<half4*>(&Xh[32 * n + rl][row]) = hi;
      if constexpr (FSMI_NPROD == 3)
        *reinterpret_cast<half4*>(&Xl[32 * n + rl][row]) = __builtin_convertvector(v - __builtin_convertvector(hi, f32x4), half4);
    }
#pragma unroll
    for (int u = 0; u < CT; ++u) {                 // x rows Hd + 8 g ..
      const int task = u * 512 + tid, p = task % PX, g = task / PX;
      const f32x8 v = cv[u] * ys;
      const half8 hi = __builtin_convertvector(v, half8);
      *reinterpret_cast<half8*>(&Xh[p][Hd + 8 * g]) = hi;
      if constexpr (FSMI_NPROD == 3)
        *reinterpret_cast<half8*>(&Xl[p][Hd + 8 * g]) = __builtin_convertvector(v - __builtin_convertvector(hi, f32x8), half8);
    }
  }
  __syncthreads();

  // ---- GEMM 2: q rows [32 m, +32) x pixel fragment n, K = [r*h, x]
  f32x16 acc2[2][1][1];
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc2[e][0][0][r] = 0.f;
#pragma unroll
  for (int c = 0; c < NK; ++c) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      half8 ah[1] = {w2f[c % kRing][k][0]}, al[1] = {w2f[c % kRing][k][1]}, bh[1], bl[1];
      bh[0] = *reinterpret_cast<const half8*>(&Xh[32 * n + rl][c * HKC + 16 * k + 8 * hsel]);
      if constexpr (FSMI_NPROD == 3) bl[0] = *reinterpret_cast<const half8*>(&Xl[32 * n + rl][c * HKC + 16 * k + 8 * hsel]);
      mma3<1, 1>(acc2[k], ah, al, bh, bl);
    }
    if (c + kRing < NK) load_w2(c % kRing, c + kRing);
  }

  // ---- blend (store_el act 4's arithmetic): out = ((1 - z) h + z tanh(q)) * att
  if (pok) {
    const float yinv = exp2i(s2 == kNoExp ? 0 : -s2);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = 32 * m + (r & 3) + 8 * (r >> 2) + 4 * hsel;
      const float2 qq = lsbq[co];
      const float v = (acc2[0][0][0][r] + acc2[1][0][0][r]) * yinv * qq.x + qq.y;
      const float hn = (1.f - zv[r]) * hv[r] + zv[r] * tanhf(v);
      a.out[(static_cast<size_t>(b) * Hd + co) * HW + px] = hn * at;
    }
  }
}

}  // namespace
}  // namespace fsmi

using namespace fsmi;

extern "C" int fsmi_gru_small(const float* hx, const float* xc, const float* h, const float* att, float* out,
                              const void* wzhi, const void* wzlo, const float* sbz, const void* wqhi,
                              const void* wqlo, const float* sbq, int B, int K, int Hd, int H, int W, void* stream) {
  FSMI_CHECK_ARG(hx && xc && h && att && out && wzhi && wzlo && sbz && wqhi && wqlo && sbq,
                 "fsmi_gru_small: null pointer");
  FSMI_CHECK_ARG(Hd == kGsHd, "fsmi_gru_small: built for Hd = %d (got %d)", kGsHd, Hd);
  FSMI_CHECK_ARG(K == 384 || K == 512, "fsmi_gru_small: K = %d (384 or 512: hidden 128 + x 256 / 384)", K);
  FSMI_CHECK_ARG(B > 0 && H > 0 && W > 0, "fsmi_gru_small: bad shape");
  FSMI_CHECK_ARG(out != h && out != hx && out != xc && out != att, "fsmi_gru_small: out must not alias an input");
  GruSmallArgs a;
  a.hx = hx;
  a.xc = xc;
  a.h = h;
  a.att = att;
  a.out = out;
  a.wzh = static_cast<const _Float16*>(wzhi);
  a.wzl = static_cast<const _Float16*>(wzlo);
  a.sbz = reinterpret_cast<const float2*>(sbz);
  a.wqh = static_cast<const _Float16*>(wqhi);
  a.wql = static_cast<const _Float16*>(wqlo);
  a.sbq = reinterpret_cast<const float2*>(sbq);
  a.B = B;
  a.HW = H * W;
  a.tiles = (a.HW + kGsPX - 1) / kGsPX;
  hipStream_t s = as_stream(stream);
  a.clk = clock_slot(FSMI_K_CONV2D, s, 8ll * B * a.tiles, "gru_small", true);
  LaunchTimer t(FSMI_K_CONV2D, s);
  const dim3 grid(static_cast<unsigned>(B * a.tiles));
  if (K == 512) hipLaunchKernelGGL(gru_small_kernel<512>, grid, dim3(512), 0, s, a);
  else hipLaunchKernelGGL(gru_small_kernel<384>, grid, dim3(512), 0, s, a);
  return finish_launch("fsmi_gru_small");
}
