// Pointwise (1x1) split-precision convolution with a multi-stage LDS-DMA input ring (cfg 24-26).
//
// A 1x1 layer gives the halo kernel one tap of MFMA work per 32-channel chunk, too little to
// cover the chunk's global round trip with one chunk of prefetch: the loop's 1x1 layers ran at
// 60-130 TFLOP/s against 230-300 for the 3x3 layers (tools/conv_census.py).  Here:
//   * a block owns BM output channels x PX consecutive pixels of one image (a 1x1 conv needs no
//     halo, so the pixel tile is a run of the flattened H*W plane: every channel row of a chunk
//     is PX contiguous floats);
//   * the input chunks go global -> LDS by LDS-DMA (global_load_lds_dwordx4: no VGPR staging,
//     one 1-KiB wave instruction per two 128-pixel rows) into an NS-deep ring, NS-1 chunks in
//     flight while one is consumed; one explicit vmcnt wait + barrier per chunk;
//   * each wave splits its own B fragments into fp16 hi / lo straight from the fp32 ring (8
//     ds_read_b32 per fragment and k half), the weights are register-resident one chunk ahead
//     (as conv_halo_wreg_kernel), three MFMAs per product;
//   * range mode 2 (conv_halo.h): the block exponent is fixed from the first chunk with 8 bits of
//     headroom; a value beyond fp16's range sets the range flag;
//   * same split-K partials / reduce pass and the same epilogues (store_frag) as the halo tiles.
// Entry: run_halo (conv_halo_x3.hip) with cfg 24-26; KS = 1, 2D, H*W % 4 == 0, 16-B aligned segments.
#include "conv_halo.h"

#ifndef FSMI_PW_TWOBAR
#define FSMI_PW_TWOBAR 0                           // 1: the round-2 schedule (a second barrier per chunk)
#endif
#ifndef FSMI_PW_WLD_ADJ
#define FSMI_PW_WLD_ADJ 0
#endif


namespace fsmi {
namespace {

// s_waitcnt with only vmcnt = N (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[15:14])
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt 0..63");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ void wait_lgkm0() {     // lgkmcnt = 0, vmcnt / expcnt untouched
  __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (3 << 14));
}

// One LDS-DMA wave instruction: 16 B per lane from src to LDS dst + 16 * lane (dst wave-uniform).
// Inline asm, so the compiler neither counts it nor guards the ring's LDS reads with its own
// vmcnt(0) (it cannot tell the ring slots apart); every wait on it is explicit (wait_vmcnt).
// M0 is compiler-reserved (an "m0" clobber is ignored), so the statement saves and restores it, and
// the M0 write -> LDS-DMA hazard needs one wait state (s_nop 0) inside the string.  Without both,
// a DMA could use a stale M0 (another ring slot) or leave the compiler's M0 clobbered: rare wrong
// partial sums in the split-K pointwise tests (round 4: 1 of ~40 runs; fixed here).
__device__ __forceinline__ void dma16(gcfptr src, float* dst) {
  typedef __attribute__((address_space(3))) float lds_float;
  const unsigned lds = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(reinterpret_cast<size_t>((lds_float*)dst)));
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}

// a bare workgroup barrier: __syncthreads()' release fence would wait for vmcnt(0), i.e. for
// every LDS-DMA chunk in flight, and serialise the ring; the waits are explicit instead
__device__ __forceinline__ void bar() { asm volatile("s_barrier" ::: "memory"); }

// COOP (cfg 27-29): the block splits each chunk ONCE -- every thread converts 8 channels of one
// pixel of the fp32 ring slot into fp16 hi / lo and stores them to a double-buffered [pixel][channel]
// image (the halo tiles' 80-B rows: conflict-free ds_read_b128 B fragments) -- instead of every wave
// splitting the B fragments it reads (WM waves re-split the same pixels: 2 x at cfg 24, 4 x for a
// 256-cout tile).  Two barriers per chunk; two or three blocks per CU overlap one block's split with
// another's MFMAs.
template <int BM, int PX, int WM, int NS, bool COOP = false>
__global__ __launch_bounds__(256) void conv_pw_kernel(HaloArgs a) {
  FSMI_TIMELINE_CLOCK(a.clk);
  constexpr int WN = 4 / WM, TM = BM / WM / 32, TN = PX / WN / 32;
  constexpr int CHF = HKC * PX;                    // floats per chunk: 32 channel rows x PX pixels
  constexpr int OPS = CHF / (4 * 256);             // DMA instructions per wave per chunk (16 B a lane)
  static_assert(TM >= 1 && TN >= 1 && OPS >= 1 && CHF % 1024 == 0 && NS >= 3, "pw tile");
  static_assert(!COOP || PX * (HKC / 8) % 256 == 0, "coop split: whole 8-channel tasks per thread");
  __shared__ __attribute__((aligned(16))) float ring[NS][CHF];
  __shared__ __attribute__((aligned(16))) float red[4];
  __shared__ __attribute__((aligned(16))) _Float16 Xh[COOP ? 2 : 1][COOP ? PX : 1][HROW];
  __shared__ __attribute__((aligned(16))) _Float16 Xl[COOP ? 2 : 1][COOP ? PX : 1][HROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM, hsel = lane >> 5, rl = lane & 31;
  const long long HW = a.cstride;
  const int nck = a.CinP / HKC;

  // tile: (cout tile, split) major over an XCD-aware remap; a.nct pixel tiles per image
  const unsigned item = xcd_remap(blockIdx.x, gridDim.x);
  const int cs = item / a.npix, ptile = item - cs * a.npix;
  const int ctile = cs / a.nsplit, split = cs - ctile * a.nsplit;
  const int m0 = ctile * BM;
  const int b = ptile / a.nct;
  const long long px0 = static_cast<long long>(ptile - b * a.nct) * PX;
  const int c_begin = split * a.kpc, c_end = min(nck, c_begin + a.kpc), n = c_end - c_begin;
  __shared__ EpiCoef<BM> ecoef;                    // visible to the epilogue after the ring's barriers
  if (a.nsplit == 1) ecoef.fill(a, m0, tid, 256);

  // this lane's DMA elements: op o moves flat quad (wave * OPS + o) * 64 + lane of the chunk
  int drow[OPS];
  long long dpix[OPS];
#pragma unroll
  for (int o = 0; o < OPS; ++o) {
    const int e = ((wave * OPS + o) * 64 + lane) * 4;
    drow[o] = e / PX;
    dpix[o] = min(px0 + e % PX, HW - 4);           // a tile tail past the plane re-reads its last quad
  }
  SegBases seg;
  seg.init(a, b, HW);
  auto dma = [&](int c, int slot) FSMI_HALO_INL {
#pragma unroll
    for (int o = 0; o < OPS; ++o) {
      const int ci = min(c * HKC + drow[o], a.Cin - 1);   // channels past Cin: any valid row (zeroed below)
      dma16(seg.chan(a, ci, HW) + dpix[o], &ring[slot][(wave * OPS + o) * 256]);
    }
  };

  int wrow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) wrow[i] = min(m0 + (wm * TM + i) * 32 + rl, a.CoutP - 1) * HKC + 8 * hsel;
  half8 wf[2][TM][2][2];                           // [buffer][i][k half][hi, lo]
  // global loads one load_wf issues: the explicit vmcnt waits below count them.  The one-product
  // build loads no lo halves -- left to the compiler, the unused lo loads were dropped and the
  // waits, still counting 4 * TM, let a chunk's LDS-DMA be read before it landed (round 4: garbage
  // in convc1's output in the fast build, one run in three)
  // (FSMI_PW_WLD_ADJ: a deliberately wrong count, only for tests/test_dma_waits.py's negative build)
  constexpr int WLD = (FSMI_NPROD == 3 ? 4 : 2) * TM + FSMI_PW_WLD_ADJ;
  auto load_wf = [&](auto buf_c, int c) FSMI_HALO_INL {
    constexpr int buf = decltype(buf_c)::value;
    const size_t base = static_cast<size_t>(c) * a.CoutP * HKC;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        wf[buf][i][k][0] = *reinterpret_cast<const half8*>(a.whi + base + wrow[i] + 16 * k);
        if constexpr (FSMI_NPROD == 3) wf[buf][i][k][1] = *reinterpret_cast<const half8*>(a.wlo + base + wrow[i] + 16 * k);
        else wf[buf][i][k][1] = wf[buf][i][k][0];
      }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  bool pix_ok[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) pix_ok[j] = px0 + (wn * TN + j) * 32 + rl < HW;

  float scale = 1.f;
  int sx = kNoExp;
  bool ovf = false;
  // chunk q (buffer parity P): prefetch weights q+1 and chunk q+NS-1, wait for chunk q and
  // weights q (the 2*OPS + WLD younger memory ops may stay in flight), barrier, MFMAs, barrier.
  // LAST (the odd tail step, q = n - 1): its weight prefetch would be dead code -- the compiler
  // drops it -- so it issues none and its wait counts none.  The n == 1 tail follows the prologue
  // directly, with only the (NS - 2) clamped DMA groups after chunk 0's; the static check
  // (tests/test_dma_waits.py) found the round-4 tail waiting for WLD loads that did not exist there.
  auto step = [&](auto par_c, auto last_c, int q) FSMI_HALO_INL {
    constexpr int P = decltype(par_c)::value;
    constexpr bool LAST = decltype(last_c)::value;
    constexpr int W = LAST ? 0 : WLD;
    const int c = c_begin + q;
    if constexpr (!LAST) load_wf(std::integral_constant<int, P ^ 1>(), min(c + 1, c_end - 1));
#if FSMI_PW_TWOBAR
    dma(min(c + NS - 1, c_end - 1), (q + NS - 1) % NS);
    wait_vmcnt<2 * OPS + W>();                     // this wave's part of chunk q has landed
    bar();                                         // ... and every wave's
#else
    // one barrier per chunk: chunk q's DMA is waited for (chunks q+1 .. q+NS-2 and the weights just
    // issued may stay in flight), the barrier makes every wave's part visible AND retires every
    // wave's reads of chunk q-1's slot, which chunk q+NS-1 then refills
    wait_vmcnt<(NS - 2) * OPS + W>();
    bar();
    dma(min(c + NS - 1, c_end - 1), (q + NS - 1) % NS);
#endif
    const float* xs = ring[q % NS];
    // block exponent (range mode 2) from the first chunk holding a nonzero value (an all-zero first
    // chunk would leave scale 1 and drop small later values to fp16 subnormals)
    if (sx == kNoExp) {
      float m = 0.f;
#pragma unroll
      for (int u = 0; u < CHF / 1024; ++u) {
        const float4 v = *reinterpret_cast<const float4*>(xs + (u * 256 + tid) * 4);
        const int row = ((u * 256 + tid) * 4) / PX;
        const bool okc = c * HKC + row < a.Cin;
        m = fmaxf(m, okc ? fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))) : 0.f);
      }
      m = wave_max(m);
      if (lane == 0) red[wave] = m;
      wait_lgkm0();
      bar();
      sx = __builtin_amdgcn_readfirstlane(chunk_exp<kRangeHeadroom>(red4_max(red)));
      scale = exp2i(sx == kNoExp ? 0 : sx);
    }
    if constexpr (COOP) {
      // the block's one split of chunk q: task = (8-channel group g, pixel), ring rows g*8 .. g*8+7
#pragma unroll
      for (int u = 0; u < PX * (HKC / 8) / 256; ++u) {
        const int task = u * 256 + tid, px = task % PX, gq = task / PX;
        const int nvalid = a.Cin - c * HKC - 8 * gq;
        const bool pok = px0 + px < HW;
        f32x8 x;
        float mx = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const float v = xs[(8 * gq + t) * PX + px];
          x[t] = (t < nvalid && pok) ? v * scale : 0.f;
          mx = fmaxf(mx, fabsf(x[t]));
        }
        ovf |= mx >= 65504.f;
        const half8 hi = __builtin_convertvector(x, half8);
        *reinterpret_cast<half8*>(&Xh[P][px][8 * gq]) = hi;
        if constexpr (FSMI_NPROD == 3)
          *reinterpret_cast<half8*>(&Xl[P][px][8 * gq]) = __builtin_convertvector(x - __builtin_convertvector(hi, f32x8), half8);
      }
      wait_lgkm0();
      bar();                                       // the split image of chunk q is complete
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      half8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        ah[i] = wf[P][i][k][0];
        al[i] = wf[P][i][k][1];
      }
      if constexpr (COOP) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int pl = (wn * TN + j) * 32 + rl;
          bh[j] = *reinterpret_cast<const half8*>(&Xh[P][pl][16 * k + 8 * hsel]);
          if constexpr (FSMI_NPROD == 3) bl[j] = *reinterpret_cast<const half8*>(&Xl[P][pl][16 * k + 8 * hsel]);
        }
        mma3<TM, TN>(acc, ah, al, bh, bl);
        continue;
      }
      const int ci0 = 16 * k + 8 * hsel;
      const int nvalid = a.Cin - c * HKC - ci0;    // channels of this lane's 8 that exist
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int pl = (wn * TN + j) * 32 + rl;
        f32x8 x;
        float mx = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const float v = xs[(ci0 + t) * PX + pl];
          x[t] = (t < nvalid && pix_ok[j]) ? v * scale : 0.f;
          mx = fmaxf(mx, fabsf(x[t]));
        }
        ovf |= mx >= 65504.f;
        bh[j] = __builtin_convertvector(x, half8);
        if constexpr (FSMI_NPROD == 3) bl[j] = __builtin_convertvector(x - __builtin_convertvector(bh[j], f32x8), half8);
      }
      mma3<TM, TN>(acc, ah, al, bh, bl);
    }
#if FSMI_PW_TWOBAR
    wait_lgkm0();
    bar();                                         // every wave is done with slot q % NS
#endif
  };
  // prologue: weights of the first chunk, then NS - 1 chunks in flight; the chunk loop sits inside
  // the same branch, so every path to a ring wait passes the prologue's DMAs
  if (n > 0) {
    load_wf(std::integral_constant<int, 0>(), c_begin);
#pragma unroll
    for (int s = 0; s < NS - 1; ++s) dma(min(c_begin + s, c_end - 1), s);
    using F = std::false_type;
    int q = 0;
    for (; q + 1 < n; q += 2) {
      step(std::integral_constant<int, 0>(), F(), q);
      step(std::integral_constant<int, 1>(), F(), q + 1);
    }
    if (q < n) step(std::integral_constant<int, 0>(), std::true_type(), q);
  }
  wait_vmcnt<0>();                                 // the tail's clamped prefetches land before exit
  flag_overflow(a, ovf);

  const float xinv = exp2i(sx == kNoExp ? 0 : -sx);
  if (a.nsplit > 1) {                              // raw partials (packed units) into ws slot `split`
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (!pix_ok[j]) continue;
      const long long hw = px0 + (wn * TN + j) * 32 + rl;
      float* wp = a.ws + (static_cast<size_t>(split) * a.B + b) * a.Cout * HW + hw;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hsel;
          if (co < a.Cout) wp[static_cast<size_t>(co) * HW] = acc[i][j][r] * xinv;
        }
    }
    return;
  }
  auto epi = [&](auto act_c) FSMI_HALO_INL {
    constexpr int ACT = decltype(act_c)::value;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (!pix_ok[j]) continue;
      const long long hw = px0 + (wn * TN + j) * 32 + rl;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int cl = (wm * TM + i) * 32 + 4 * hsel;
        FragCoef cf;               // per-cout coefficients from LDS (conv_halo.h EpiCoef)
        frag_coef_lds<ACT>(xinv, cl, ecoef.sb, ecoef.g, cf);
        store_frag_c<ACT, false>(a, acc[i][j], cf, m0 + cl, b, hw, 0, a.out, a.res, a.gh, a.gz, a.gatt, a.grh);
      }
    }
  };
  switch (a.act) {
    case 1: epi(std::integral_constant<int, 1>()); break;
    case 2: epi(std::integral_constant<int, 2>()); break;
    case 3: epi(std::integral_constant<int, 3>()); break;
    case 4: epi(std::integral_constant<int, 4>()); break;
    case 5: epi(std::integral_constant<int, 5>()); break;
    case 6: epi(std::integral_constant<int, 6>()); break;
    case 7: epi(std::integral_constant<int, 7>()); break;
    default: epi(std::integral_constant<int, 0>()); break;
  }
}

}  // namespace

namespace halo {

// cfg 24: 128 couts x 128 px (2 x 2 fragments per wave), 3-deep ring; 25: 128 x 64 (2 x 1), 4 deep;
// 26: 64 x 128 (2 x 1, waves along the pixels), 3 deep.  The block-split (COOP) tiles: 27: 256 x 64
// (2 x 2 per wave, waves along the couts), 4 deep; 28: 128 x 64 (2 x 1), 4 deep; 29: 128 x 128
// (2 x 2), 3 deep.  Deeper rings (6 / 8 chunks, 64-96 KB of
// LDS) measured 5-40 % slower on every cfg2 1x1 shape (tools/pw_bench.py), so the chunk round
// trip is not what bounds these layers.  Tile geometry (a.nct = pixel tiles per image, a.npix, a.nco) is set by
// the caller (pw_tile).
int launch_pw(int cfg, const HaloArgs& a, hipStream_t s) {
  const unsigned grid = static_cast<unsigned>(a.npix) * a.nco * a.nsplit;
  switch (cfg) {
    case 24: hipLaunchKernelGGL((conv_pw_kernel<128, 128, 2, 3>), dim3(grid), dim3(256), 0, s, a); break;
    case 25: hipLaunchKernelGGL((conv_pw_kernel<128, 64, 2, 4>), dim3(grid), dim3(256), 0, s, a); break;
    case 26: hipLaunchKernelGGL((conv_pw_kernel<64, 128, 1, 3>), dim3(grid), dim3(256), 0, s, a); break;
    case 27: hipLaunchKernelGGL((conv_pw_kernel<256, 64, 4, 4, true>), dim3(grid), dim3(256), 0, s, a); break;
    case 28: hipLaunchKernelGGL((conv_pw_kernel<128, 64, 2, 4, true>), dim3(grid), dim3(256), 0, s, a); break;
    case 29: hipLaunchKernelGGL((conv_pw_kernel<128, 128, 2, 3, true>), dim3(grid), dim3(256), 0, s, a); break;
    default: set_error("fsmi_conv_halo: pointwise tile %d (24..29)", cfg); return FSMI_ERR_ARG;
  }
  return finish_launch("fsmi_conv_halo");
}

void pw_tile(int cfg, HaloArgs& a) {
  const int BM = cfg == 26 ? 64 : cfg == 27 ? 256 : 128, PX = (cfg == 25 || cfg == 27 || cfg == 28) ? 64 : 128;
  const long long HW = a.cstride;
  a.nrt = 1;
  a.nct = static_cast<int>((HW + PX - 1) / PX);
  a.npix = a.B * a.nct;
  a.nco = (a.Cout + BM - 1) / BM;
}

}  // namespace halo
}  // namespace fsmi
