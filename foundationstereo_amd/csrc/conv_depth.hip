// Depth-blocked (KD, 1, 1) volume convolution: the disparity-axis conv of Conv3dNormActReduced
// (core/submodule.py:89-114, kernel_disp = 17; hourglass conv1..3, agg_0 / agg_1, conv_out,
// core/foundation_stereo.py:45-123), on the same split-precision MFMA ("3 x fp16") as the halo
// convs (conv_halo.h), with their epilogue (folded BatchNorm, ReLU / LeakyReLU, ResNet tail,
// FeatureAtt gate).
//
// On the generic volume tile (conv_halo.h, KS = 1, KD = 17) an output depth d stages KD input
// planes, each feeding ONE tap: every input plane is staged 17 times and a staged 16-KB chunk
// carries 6 MFMAs per wave (56 TFLOP/s on conv_out at cfg2).  Here a block owns DB = 16
// consecutive output depths of a 2 x 32 pixel tile and walks the DB + KD - 1 input planes that
// window covers once each: staged plane p feeds every output j with tap kd = p - (d0 + j) + KD/2
// in [0, KD), up to 8 per wave -- (DB + KD - 1) / DB = 2 stagings per output instead of KD.
//
//   * waves: (pixel row r = wave & 1, output-depth half jh = wave >> 1); a wave accumulates 8 output
//     depths of one 32-pixel row for a 32-cout tile (8 x 16 accumulator registers);
//   * the (KD x 32 cout x 32 cin) hi / lo weight slab of the current 32-channel chunk lives in LDS
//     for the whole plane walk (68 KB, 16-B slots XOR-swizzled by row so the A-fragment reads are
//     conflict-free without padding); each (plane, output) pair reads its tap's A fragments from it;
//   * the plane tile (64 px x 32 ch) is staged like the halo tile (HaloStage<1, 2>: loaded one plane
//     ahead into registers, split into fp16 hi / lo with the block exponent); 78 KB of LDS in all,
//     two blocks per CU;
//   * range: the exact block max of every staged plane; the block exponent follows it in both
//     directions (hysteresis 8 bits), accumulators rescaled by exact powers of two -- each plane is
//     split at ~22 bits relative to its own maximum (conv_halo.h, chunk_exp);
//   * blocks: cout tile slowest, then (b, row tile, col tile), depth tile fastest, over the XCD
//     remap -- the depth tiles of one pixel column share their overlapping planes in one L2.
#include "conv_halo.h"

namespace fsmi {
namespace {

constexpr int kDepthDB = 16;        // output depths per block
constexpr int kDepthTR = 2;        // pixel rows per block (x 32 columns)

// swizzled 16-B slot of (row, logical slot s in 0..3) in a 64-B weight row: lanes 0-15 of an
// A-fragment read (rows 0..15, one slot) then touch 16 distinct (bank quarter, slot) pairs
__device__ __forceinline__ int wslot(int row, int s) { return s ^ ((row >> 2) & 3); }

template <int KD>
__global__ __launch_bounds__(256) void conv_depth_kernel(HaloArgs a) {

  constexpr int DB = kDepthDB, TR = kDepthTR, JW = DB / 2, PD = KD / 2;
  static_assert(JW == 8, "the A-fragment ring holds 8 taps: 8 outputs per wave");
  using HS = HaloStage<1, TR>;
  __shared__ __attribute__((aligned(16))) _Float16 Wh[KD][32][32];
  __shared__ __attribute__((aligned(16))) _Float16 Wl[KD][32][32];
  __shared__ __attribute__((aligned(16))) _Float16 Xh[HS::NHP][HROW];
  __shared__ __attribute__((aligned(16))) _Float16 Xl[HS::NHP][HROW];
  __shared__ __attribute__((aligned(16))) float red[4];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = wave & 1, jh = wave >> 1;
  const int hsel = lane >> 5, rl = lane & 31;

  // block -> (cout tile, b, row tile, col tile, depth tile), depth fastest
  const unsigned item = xcd_remap(blockIdx.x, gridDim.x);
  const int ndt = (a.D + DB - 1) / DB;
  int rest = static_cast<int>(item);
  const int dt = rest % ndt; rest /= ndt;
  const int ct = rest % a.nct; rest /= a.nct;
  const int rt = rest % a.nrt; rest /= a.nrt;
  const int b = rest % a.B;
  const int m0 = (rest / a.B) * 32;
  const int d0 = dt * DB, r0 = rt * TR, c0 = ct * 32;
  const int nck = a.CinP / HKC;
  __shared__ EpiCoef<32> ecoef;                    // visible to the epilogue after the plane barriers
  ecoef.fill(a, m0, tid, 256);

  HS hs, hs2;
  hs.init(a, tid, r0, c0);
  hs2.init(a, tid, r0, c0);
  f32x16 acc[JW];
#pragma unroll
  for (int j = 0; j < JW; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

  // input planes the block's outputs read, clamped to the volume (zero planes contribute nothing)
  const int p_lo = max(d0 - PD, 0), p_hi = min(d0 + DB - 1 + PD, a.D - 1);
  const int jbase = d0 + JW * jh;  // output depth of this wave's acc[0]
  int sx = kNoExp, smin = kNoExp;
  bool ovf = false;
  for (int cc = 0; cc < nck; ++cc) {
    __syncthreads();               // the previous chunk's weights and plane are no longer read
    // weight slab of chunk cc: [kd][cout m0..m0+31][32 cin], rows past CoutP clamped (their
    // outputs are dropped by the epilogue)
#pragma unroll 2
    for (int e = tid; e < KD * 32 * 4; e += 256) {
      const int s = e & 3, m = (e >> 2) & 31, kd = e >> 7;
      const size_t off = (static_cast<size_t>(kd * nck + cc) * a.CoutP + min(m0 + m, a.CoutP - 1)) * HKC + 8 * s;
      const uint4 h = *reinterpret_cast<const uint4*>(a.whi + off);
      const uint4 l = *reinterpret_cast<const uint4*>(a.wlo + off);
      *reinterpret_cast<uint4*>(&Wh[kd][m][8 * wslot(m, s)]) = h;
      *reinterpret_cast<uint4*>(&Wl[kd][m][8 * wslot(m, s)]) = l;
    }
    // A fragments: a ring of the 8 taps this wave's outputs read at the current plane.  At plane p
    // output j reads tap kd = p - jbase + PD - j, so from one plane to the next every output moves
    // one tap on and exactly one new tap enters (output 0's): with slot = (plane index - j) mod 8
    // the ring is indexed statically inside each unrolled group of 8 planes and each plane reads
    // one tap (4 x ds_read_b128) instead of eight.
    half8 ra[8][2][2];             // [slot][k half][hi, lo]
    auto read_tap = [&](half8 (&r)[2][2], int kd) FSMI_HALO_INL {
      kd = min(max(kd, 0), KD - 1);                // outputs that skip this plane read a clamped tap
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int sl = wslot(rl, 2 * k + hsel);
        r[k][0] = *reinterpret_cast<const half8*>(&Wh[kd][rl][8 * sl]);
        r[k][1] = *reinterpret_cast<const half8*>(&Wl[kd][rl][8 * sl]);
      }
    };
    __syncthreads();               // the weight slab is visible
#pragma unroll
    for (int j = 1; j < 8; ++j) read_tap(ra[(8 - j) & 7], p_lo - jbase + PD - j);
    hs.load(a, b, cc, p_lo);
    if (p_lo + 1 <= p_hi) hs2.load(a, b, cc, p_lo + 1);
    // plane p = p_lo + 8 g + U, staged from register set st (loaded two planes ahead)
    auto plane = [&](auto u_c, HS& st, int p) FSMI_HALO_INL {
      constexpr int U = decltype(u_c)::value;
      const float m = wave_max(st.absmax());
      if (lane == 0) red[wave] = m;
      __syncthreads();             // every wave is done with the previous plane; maxima visible
      const float bm = red4_max(red);
      ovf |= !(bm <= 3.4e38f);
      // per-plane exponent, both directions: re-aim (4 bits of headroom) when the plane would
      // overflow the current one or sits more than 8 bits below it, rescaling the accumulators by
      // the exact power of two -- every plane keeps ~22 bits relative to its OWN maximum (a block
      // spans 31 planes of a cost volume, whose magnitudes differ by decades along the disparity
      // axis); the exponent never climbs more than 60 above the block's smallest, so accumulators
      // of earlier large planes stay far inside fp32 (< 2^100)
      const int fit = __builtin_amdgcn_readfirstlane(chunk_exp(bm));
      if (fit != kNoExp && (fit < sx || (sx != kNoExp && fit > sx + 8))) {
        int se = __builtin_amdgcn_readfirstlane(chunk_exp<kHeadroom1>(bm));
        if (sx != kNoExp) {
          se = min(se, smin + 60);
          const float f = exp2i(se - sx);
#pragma unroll
          for (int j = 0; j < JW; ++j) acc[j] *= f;
        }
        sx = se;
        smin = min(smin, se);
      }
      st.template store<1>(Xh, Xl, tid, exp2i(sx == kNoExp ? 0 : sx), ovf);
      if (p + 2 <= p_hi) st.load(a, b, cc, p + 2);   // in flight during the next two planes
      __syncthreads();
      read_tap(ra[U], p - jbase + PD);             // output 0's new tap (its slot's last reader was
                                                   // output 7 at the previous plane)
      half8 bh[2], bl[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        bh[k] = *reinterpret_cast<const half8*>(&Xh[row * 32 + rl][16 * k + 8 * hsel]);
        bl[k] = *reinterpret_cast<const half8*>(&Xl[row * 32 + rl][16 * k + 8 * hsel]);
      }
      // outputs 7..0 (output 0 last: its tap was just read)
#pragma unroll
      for (int jj = 0; jj < JW; ++jj) {
        const int j = JW - 1 - jj;
        const int kd = p - jbase + PD - j;
        if (kd < 0 || kd >= KD) continue;          // wave-uniform
        const int slot = (U - j) & 7;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          if constexpr (FSMI_NPROD == 3) {
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[slot][k][1], bh[k], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[slot][k][0], bl[k], acc[j], 0, 0, 0);
          }
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[slot][k][0], bh[k], acc[j], 0, 0, 0);
        }
      }
    };
    for (int p = p_lo; p <= p_hi; p += 8) {
      plane(std::integral_constant<int, 0>(), hs, p);
      if (p + 1 > p_hi) break;
      plane(std::integral_constant<int, 1>(), hs2, p + 1);
      if (p + 2 > p_hi) break;
      plane(std::integral_constant<int, 2>(), hs, p + 2);
      if (p + 3 > p_hi) break;
      plane(std::integral_constant<int, 3>(), hs2, p + 3);
      if (p + 4 > p_hi) break;
      plane(std::integral_constant<int, 4>(), hs, p + 4);
      if (p + 5 > p_hi) break;
      plane(std::integral_constant<int, 5>(), hs2, p + 5);
      if (p + 6 > p_hi) break;
      plane(std::integral_constant<int, 6>(), hs, p + 6);
      if (p + 7 > p_hi) break;
      plane(std::integral_constant<int, 7>(), hs2, p + 7);
    }
  }
  flag_overflow(a, ovf);
  const float xinv = exp2i(sx == kNoExp ? 0 : -sx);
  const int hh = r0 + row, ww = c0 + rl;
  if (hh >= a.H || ww >= a.W) return;
  const long long P = static_cast<long long>(a.H) * a.W;
  const int hw2 = hh * a.W + ww;
  const int cb = m0 + 4 * hsel;
  auto epi = [&](auto act_c) FSMI_HALO_INL {
    constexpr int ACT = decltype(act_c)::value;
#pragma unroll
    for (int j = 0; j < JW; ++j) {
      const int d = jbase + j;
      if (d >= a.D) break;
      const long long hw = static_cast<long long>(d) * P + hw2;
      FragCoef cf;                 // per-cout coefficients from LDS (conv_halo.h EpiCoef)
      frag_coef_lds<ACT>(xinv, 4 * hsel, ecoef.sb, ecoef.g, cf);
      store_frag_c<ACT, true>(a, acc[j], cf, cb, b, hw, hw2, a.out, a.res, a.gh, a.gz, a.gatt, a.grh);
    }
  };
  switch (a.act) {
    case 1: epi(std::integral_constant<int, 1>()); break;
    case 6: epi(std::integral_constant<int, 6>()); break;
    default: epi(std::integral_constant<int, 0>()); break;
  }
}


// ---------------------------------------------------------------- (3, 3, 3): cfg 31
// The same plane walk for the 3^3 convs of corr_stem / the ResNet blocks / the classifier
// (core/foundation_stereo.py:164-176, core/submodule.py:51-86,159-195).  On the generic volume tile
// each (output depth, kd) pair stages its own 32-channel chunk, so every input plane is staged three
// times and feeds 54 MFMAs per wave each time (~15 % of the MFMA rate at cfg2's 28-channel stem).
// Here a block owns DB = 8 output depths of a 4 x 32 pixel tile (wave w: row w, all 8 depths):
// staged plane U feeds output j = U - kd, kd in [0, 3), over all 9 spatial taps -- up to 3 outputs
// x 9 taps x 2 k-steps x 3 products = 162 MFMAs per wave per staging, (DB + 2) / DB stagings per
// output; the plane walk is unrolled so every accumulator index is a constant.  The (27 taps x 32 x
// 32) hi / lo weight slab of a chunk sits in LDS for the whole walk (108 KB, swizzled as above),
// the plane's halo (6 x 34 pixels) beside it: 141 KB, one block per CU.  Measured (cfg2 stem, 28 ->
// 28 at 48 x 120 x 160): 471 us vs 373 on the generic tile -- the compiler issues each A / B read
// right before its MFMAs with a full lgkmcnt wait (only 16 VGPRs left for operands at the 256-VGPR
// limit), so the tile stays opt-in (explicit cfg 31).
constexpr int kD3DB = 8;           // output depths per block
constexpr int kD3TR = 4;           // pixel rows per block (x 32 columns): wave w owns row w

__global__ __launch_bounds__(256) void conv_depth3_kernel(HaloArgs a) {
  constexpr int KD = 3, KS = 3, NTAP = KS * KS, DB = kD3DB, TR = kD3TR, NP = DB + KD - 1;
  using HS = HaloStage<KS, TR>;
  __shared__ __attribute__((aligned(16))) _Float16 Wh[KD * NTAP][32][32];
  __shared__ __attribute__((aligned(16))) _Float16 Wl[KD * NTAP][32][32];
  __shared__ __attribute__((aligned(16))) _Float16 Xh[HS::NHP][HROW];
  __shared__ __attribute__((aligned(16))) _Float16 Xl[HS::NHP][HROW];
  __shared__ __attribute__((aligned(16))) float red[4];

  const int tid = threadIdx.x, lane = tid & 63, row = tid >> 6;
  const int hsel = lane >> 5, rl = lane & 31;

  // block -> (cout tile, b, row tile, col tile, depth tile), depth fastest
  const unsigned item = xcd_remap(blockIdx.x, gridDim.x);
  const int ndt = (a.D + DB - 1) / DB;
  int rest = static_cast<int>(item);
  const int dt = rest % ndt; rest /= ndt;
  const int ct = rest % a.nct; rest /= a.nct;
  const int rt = rest % a.nrt; rest /= a.nrt;
  const int b = rest % a.B;
  const int m0 = (rest / a.B) * 32;
  const int d0 = dt * DB, r0 = rt * TR, c0 = ct * 32;
  const int nck = a.CinP / HKC;
  __shared__ EpiCoef<32> ecoef;                    // visible to the epilogue after the plane barriers
  ecoef.fill(a, m0, tid, 256);

  HS hs;                           // one register set, loaded one plane ahead (two sets took the
  hs.init(a, tid, r0, c0);         // VGPRs the MFMA operands need to be read ahead)
  f32x16 acc[DB];
#pragma unroll
  for (int j = 0; j < DB; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

  int sx = kNoExp, smin = kNoExp;
  bool ovf = false;
  for (int cc = 0; cc < nck; ++cc) {
    __syncthreads();               // the previous chunk's weights and plane are no longer read
    // weight slab of chunk cc: [(kd, kh, kw)][cout m0..m0+31][32 cin] (the packing's tap order)
    for (int e = tid; e < KD * NTAP * 32 * 4; e += 256) {
      const int s4 = e & 3, m = (e >> 2) & 31, kt = e >> 7;
      const size_t off = (static_cast<size_t>(kt * nck + cc) * a.CoutP + min(m0 + m, a.CoutP - 1)) * HKC + 8 * s4;
      const uint4 h = *reinterpret_cast<const uint4*>(a.whi + off);
      const uint4 l = *reinterpret_cast<const uint4*>(a.wlo + off);
      *reinterpret_cast<uint4*>(&Wh[kt][m][8 * wslot(m, s4)]) = h;
      *reinterpret_cast<uint4*>(&Wl[kt][m][8 * wslot(m, s4)]) = l;
    }
    // planes d0 - 1 .. d0 + DB, walked in order (zeros outside [0, D): HaloStage::load)
    hs.load(a, b, cc, d0 - 1);
    static_for<0, NP>([&](auto u_c) FSMI_HALO_INL {
      constexpr int U = decltype(u_c)::value;
      HS& st = hs;
      const float m = wave_max(st.absmax());
      if (lane == 0) red[row] = m;
      __syncthreads();             // every wave is done with the previous plane; maxima visible
      const float bm = red4_max(red);
      ovf |= !(bm <= 3.4e38f);
      // per-plane exponent, both directions, as conv_depth_kernel
      const int fit = __builtin_amdgcn_readfirstlane(chunk_exp(bm));
      if (fit != kNoExp && (fit < sx || (sx != kNoExp && fit > sx + 8))) {
        int se = __builtin_amdgcn_readfirstlane(chunk_exp<kHeadroom1>(bm));
        if (sx != kNoExp) {
          se = min(se, smin + 60);
          const float f = exp2i(se - sx);
#pragma unroll
          for (int j = 0; j < DB; ++j) acc[j] *= f;
        }
        sx = se;
        smin = min(smin, se);
      }
      st.template store<1>(Xh, Xl, tid, exp2i(sx == kNoExp ? 0 : sx), ovf);
      if constexpr (U + 1 < NP) st.load(a, b, cc, d0 - 1 + U + 1);   // in flight during this plane's MFMAs
      __syncthreads();
      // plane U feeds outputs j = U - kd in [0, DB): compile-time indices throughout
#pragma unroll
      for (int tap = 0; tap < NTAP; ++tap) {
        const int hp = (row + tap / KS) * HS::HC + rl + tap % KS;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const half8 bh = *reinterpret_cast<const half8*>(&Xh[hp][16 * k + 8 * hsel]);
          const half8 bl = *reinterpret_cast<const half8*>(&Xl[hp][16 * k + 8 * hsel]);
          const int sl = wslot(rl, 2 * k + hsel);
          static_for<0, KD>([&](auto kd_c) FSMI_HALO_INL {
            constexpr int KDI = decltype(kd_c)::value, J = U - KDI;
            if constexpr (J >= 0 && J < DB) {
              const half8 ah = *reinterpret_cast<const half8*>(&Wh[KDI * NTAP + tap][rl][8 * sl]);
              const half8 al = *reinterpret_cast<const half8*>(&Wl[KDI * NTAP + tap][rl][8 * sl]);
              if constexpr (FSMI_NPROD == 3) {
                acc[J] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[J], 0, 0, 0);
                acc[J] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[J], 0, 0, 0);
              }
              acc[J] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[J], 0, 0, 0);
            }
          });
        }
      }
    });
  }
  flag_overflow(a, ovf);
  const float xinv = exp2i(sx == kNoExp ? 0 : -sx);
  const int hh = r0 + row, ww = c0 + rl;
  if (hh >= a.H || ww >= a.W) return;
  const long long P = static_cast<long long>(a.H) * a.W;
  const int hw2 = hh * a.W + ww;
  const int cb = m0 + 4 * hsel;
  auto epi = [&](auto act_c) FSMI_HALO_INL {
    constexpr int ACT = decltype(act_c)::value;
#pragma unroll
    for (int j = 0; j < DB; ++j) {
      const int d = d0 + j;
      if (d >= a.D) break;
      const long long hw = static_cast<long long>(d) * P + hw2;
      FragCoef cf;
      frag_coef_lds<ACT>(xinv, 4 * hsel, ecoef.sb, ecoef.g, cf);
      store_frag_c<ACT, true>(a, acc[j], cf, cb, b, hw, hw2, a.out, a.res, a.gh, a.gz, a.gatt, a.grh);
    }
  };
  switch (a.act) {
    case 1: epi(std::integral_constant<int, 1>()); break;
    case 6: epi(std::integral_constant<int, 6>()); break;
    default: epi(std::integral_constant<int, 0>()); break;
  }
}

// The single-chunk (Cin <= 32) 3^3 walk as a rolled loop (cfg 31 when CinP == 32).  The tile above
// unrolls its ten planes into 88 KB of straight-line code, more than the instruction cache holds.
// Here one plane body is the loop: a wave keeps three accumulators (outputs U, U - 1, U - 2 of plane
// U); after each plane the finished output U - 2 is stored and the ring moves down one (48 register
// moves), so a block walks DB = 12 depths (14 stagings per 12 outputs) with 48 accumulator registers;
// the edge planes (U < 2, U >= nd) run only the taps whose outputs exist.  The staging keeps its raw
// loads in flight through the MFMAs (HaloStage DEFER).  Measured on cfg2's stem (28 -> 28, 48 x 120
// x 160): DB 8 / 12 / 16 / 24 = 385 / 364 / 404 / 498 us vs 467 for the unrolled tile and 373-377 for
// the table's generic volume tile (profiles/r05_depth3r_bench.txt).  SQ counters
// (profiles/r05_depth3r_pmc.txt): MFMA pipe 16 % busy at 0.76 waves per SIMD, 6.7 VALU per MFMA --
// the staging (~750 instructions between the plane's two barriers: absmax, the exponent, hi / lo split,
// the ragged chunk's per-lane 64-bit addresses) runs with no MFMA beside it, and a second X buffer to
// overlap it does not fit beside the 108-KB weight slab.  Opt-in (FSMI_DEPTH3_TILE=1).
#ifndef FSMI_D3_DB
#define FSMI_D3_DB 12
#endif
constexpr int kD3RDB = FSMI_D3_DB;

__global__ __launch_bounds__(256) void conv_depth3r_kernel(HaloArgs a) {
  constexpr int KD = 3, KS = 3, NTAP = KS * KS, DB = kD3RDB, TR = kD3TR;
  using HS = HaloStage<KS, TR, 1, true>;
  __shared__ __attribute__((aligned(16))) _Float16 Wh[KD * NTAP][32][32];
  __shared__ __attribute__((aligned(16))) _Float16 Wl[KD * NTAP][32][32];
  __shared__ __attribute__((aligned(16))) _Float16 Xh[HS::NHP][HROW];
  __shared__ __attribute__((aligned(16))) _Float16 Xl[HS::NHP][HROW];
  __shared__ __attribute__((aligned(16))) float red[4];

  const int tid = threadIdx.x, lane = tid & 63, row = tid >> 6;
  const int hsel = lane >> 5, rl = lane & 31;

  const unsigned item = xcd_remap(blockIdx.x, gridDim.x);
  const int ndt = (a.D + DB - 1) / DB;
  int rest = static_cast<int>(item);
  const int dt = rest % ndt; rest /= ndt;
  const int ct = rest % a.nct; rest /= a.nct;
  const int rt = rest % a.nrt; rest /= a.nrt;
  const int b = rest % a.B;
  const int m0 = (rest / a.B) * 32;
  const int d0 = dt * DB, r0 = rt * TR, c0 = ct * 32;
  const int nd = min(DB, a.D - d0);                // outputs of this block
  __shared__ EpiCoef<32> ecoef;
  ecoef.fill(a, m0, tid, 256);

  // the one chunk's weight slab, [(kd, kh, kw)][cout m0..m0+31][32 cin]
  for (int e = tid; e < KD * NTAP * 32 * 4; e += 256) {
    const int s4 = e & 3, m = (e >> 2) & 31, kt = e >> 7;
    const size_t off = (static_cast<size_t>(kt) * a.CoutP + min(m0 + m, a.CoutP - 1)) * HKC + 8 * s4;
    const uint4 h = *reinterpret_cast<const uint4*>(a.whi + off);
    const uint4 l = *reinterpret_cast<const uint4*>(a.wlo + off);
    *reinterpret_cast<uint4*>(&Wh[kt][m][8 * wslot(m, s4)]) = h;
    *reinterpret_cast<uint4*>(&Wl[kt][m][8 * wslot(m, s4)]) = l;
  }
  HS hs;
  hs.init(a, tid, r0, c0);
  hs.load(a, b, 0, d0 - 1);

  const int hh = r0 + row, ww = c0 + rl;
  const bool valid = hh < a.H && ww < a.W;
  const long long P = static_cast<long long>(a.H) * a.W;
  const int hw2 = hh * a.W + ww;
  const int cb = m0 + 4 * hsel;

  f32x16 acc0, acc1, acc2;                         // outputs U, U - 1, U - 2 of plane U
#pragma unroll
  for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = acc2[r] = 0.f;
  int sx = kNoExp, smin = kNoExp;
  bool ovf = false;
  for (int U = 0; U < nd + KD - 1; ++U) {
    const float mx = wave_max(hs.absmax());
    if (lane == 0) red[row] = mx;
    __syncthreads();               // every wave is done with the previous plane; maxima visible
    const float bm = red4_max(red);
    ovf |= !(bm <= 3.4e38f);
    const int fit = __builtin_amdgcn_readfirstlane(chunk_exp(bm));
    if (fit != kNoExp && (fit < sx || (sx != kNoExp && fit > sx + 8))) {
      int se = __builtin_amdgcn_readfirstlane(chunk_exp<kHeadroom1>(bm));
      if (sx != kNoExp) {
        se = min(se, smin + 60);
        const float f = exp2i(se - sx);
        acc0 *= f;
        acc1 *= f;
        acc2 *= f;
      }
      sx = se;
      smin = min(smin, se);
    }
    hs.template store<1>(Xh, Xl, tid, exp2i(sx == kNoExp ? 0 : sx), ovf);
    if (U + 1 < nd + KD - 1) hs.load(a, b, 0, d0 + U);   // plane U + 1, in flight during the MFMAs
    __syncthreads();
    // interior planes feed three outputs; an edge plane (U < 2 or U >= nd) only those in [0, nd)
    auto mfma_plane = [&](auto full_c) FSMI_HALO_INL {
      constexpr bool FULL = decltype(full_c)::value;
      const bool k0 = FULL || U < nd, k1 = FULL || (U >= 1 && U <= nd), k2 = FULL || U >= 2;
#pragma unroll
      for (int tap = 0; tap < NTAP; ++tap) {
        const int hp = (row + tap / KS) * HS::HC + rl + tap % KS;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const half8 bh = *reinterpret_cast<const half8*>(&Xh[hp][16 * k + 8 * hsel]);
          const half8 bl = *reinterpret_cast<const half8*>(&Xl[hp][16 * k + 8 * hsel]);
          const int sl = wslot(rl, 2 * k + hsel);
          auto prod = [&](f32x16& c, int kt) FSMI_HALO_INL {
            const half8 ah = *reinterpret_cast<const half8*>(&Wh[kt][rl][8 * sl]);
            const half8 al = *reinterpret_cast<const half8*>(&Wl[kt][rl][8 * sl]);
            if constexpr (FSMI_NPROD == 3) {
              c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, c, 0, 0, 0);
            }
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
          };
          if (k0) prod(acc0, tap);
          if (k1) prod(acc1, NTAP + tap);
          if (k2) prod(acc2, 2 * NTAP + tap);
        }
      }
    };
    if (U >= KD - 1 && U < nd) mfma_plane(std::true_type());
    else mfma_plane(std::false_type());
    if (U >= KD - 1 && valid) {    // output U - 2 has all 27 taps: store it in the current scale
      const long long hw = static_cast<long long>(d0 + U - (KD - 1)) * P + hw2;
      const float xinv = exp2i(sx == kNoExp ? 0 : -sx);
      auto epi = [&](auto act_c) FSMI_HALO_INL {
        constexpr int ACT = decltype(act_c)::value;
        FragCoef cf;
        frag_coef_lds<ACT>(xinv, 4 * hsel, ecoef.sb, ecoef.g, cf);
        store_frag_c<ACT, true>(a, acc2, cf, cb, b, hw, hw2, a.out, a.res, a.gh, a.gz, a.gatt, a.grh);
      };
      switch (a.act) {
        case 1: epi(std::integral_constant<int, 1>()); break;
        case 6: epi(std::integral_constant<int, 6>()); break;
        default: epi(std::integral_constant<int, 0>()); break;
      }
    }
    acc2 = acc1;
    acc1 = acc0;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc0[r] = 0.f;
  }
  flag_overflow(a, ovf);
}

}  // namespace

namespace halo {

bool depth_conv_ok(const HaloArgs& a) { return a.KD == 17 && a.str == 1 && !a.up; }

// (KD, 1, 1) stride-1 volume conv on the depth-blocked tile; a.Cin / CinP / CoutP / D / H / W / B /
// seg_ptr[0] / seg_bstride[0] / cstride / out / sb / epilogue fields as run_halo fills them
int launch_depth(HaloArgs& a, hipStream_t s) {
  if (!depth_conv_ok(a)) {
    set_error("fsmi_conv3d_halo: the depth tile takes (17, 1, 1) stride-1 convs");
    return FSMI_ERR_ARG;
  }
  a.nrt = (a.H + kDepthTR - 1) / kDepthTR;
  a.nct = (a.W + 31) / 32;
  const long long ndt = (a.D + kDepthDB - 1) / kDepthDB;
  const long long grid = static_cast<long long>(a.CoutP / 32) * a.B * a.nrt * a.nct * ndt;
  // no in-kernel clock: the tile sits at 498 of 512 VGPRs, and the stamps' registers spilled it to
  // scratch (56-64 B) -- it runs in the 3D filter only, outside the refinement loop's timeline
  a.clk = nullptr;
  hipLaunchKernelGGL((conv_depth_kernel<17>), dim3(static_cast<unsigned>(grid)), dim3(256), 0, s, a);
  return FSMI_OK;
}

bool depth3_conv_ok(const HaloArgs& a) { return a.KD == 3 && a.str == 1 && !a.up && a.D > 1; }

// (3, 3, 3) stride-1 volume conv on the depth-blocked 3^3 tile (cfg 31), fields as launch_depth
int launch_depth3(HaloArgs& a, hipStream_t s) {
  if (!depth3_conv_ok(a)) {
    set_error("fsmi_conv3d_halo: tile 31 takes (3, 3, 3) stride-1 volume convs");
    return FSMI_ERR_ARG;
  }
  a.nrt = (a.H + kD3TR - 1) / kD3TR;
  a.nct = (a.W + 31) / 32;
  // one chunk, one input segment, byte offsets of a batch item in 32 bits: the rolled ring walk
  const bool rolled = a.CinP == HKC && a.nseg == 1 && static_cast<long long>(a.Cin) * a.cstride * 4 < (1LL << 32);
  const int db = rolled ? kD3RDB : kD3DB;
  const long long ndt = (a.D + db - 1) / db;
  const long long grid = static_cast<long long>(a.CoutP / 32) * a.B * a.nrt * a.nct * ndt;
  a.clk = nullptr;
  if (rolled)
    hipLaunchKernelGGL(conv_depth3r_kernel, dim3(static_cast<unsigned>(grid)), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(conv_depth3_kernel, dim3(static_cast<unsigned>(grid)), dim3(256), 0, s, a);
  return FSMI_OK;
}

}  // namespace halo
}  // namespace fsmi
