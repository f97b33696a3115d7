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

}  // namespace halo
}  // namespace fsmi
