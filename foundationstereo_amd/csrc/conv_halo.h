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
// accumulation.  Epilogue: bias, ReLU/GELU, alpha, gamma, residual, channel-offset store.
//
// Layout of the sources: this header holds the device code; each (kernel size, 2D / volume)
// pair compiles in its own translation unit (conv_halo_k{1,3}_{2d,3d}.hip, built in parallel),
// and conv_halo_x3.hip holds the host side (tile / split-K policy, C ABI) and the reduce pass.
#pragma once
#include <cstdlib>
#include <type_traits>

#include "fsmi_common.h"

// activation range of the split.  Default (FSMI_HALO_RANGE 1):
//   * 2D maps (mode 2): a block exponent fixed by the block's first 32-channel chunk with 8 bits
//     of headroom, so every later chunk up to 2^9 x larger still fits fp16; a value beyond that
//     sets the range flag (fsmi_range_status -> RangeError), never a silent inf.  Callers put the
//     largest-magnitude input segment first where they know it (update.py: the motion encoder's
//     disparity features ahead of its correlation features).
//   * NCDHW volumes (mode 1): the exact block max of every chunk with accumulator rescaling --
//     a block's first chunk there is one depth plane, and planes differ by far more than 2^9
//     (the bias-only w < d region of the cost volume).
// Measured end to end (cfg2): mode 2 costs ~3 % against no scaling, mode 1 on every conv ~7 %;
// volumes are ~10 % of the conv time.  FSMI_HALO_RANGE=0 builds an A/B variant without either
// (fp16 range: |x| < 65504, 22 bits only for |x| >~ 0.1); 2 / 3 force mode 2 / 3 everywhere.
#ifndef FSMI_HALO_RANGE
#define FSMI_HALO_RANGE 1
#endif
template <bool D3>
constexpr int range_mode() { return FSMI_HALO_RANGE == 1 ? (D3 ? 1 : 2) : FSMI_HALO_RANGE; }
// the wreg kernel's lambdas are forced inline: left to the inliner's cost model, clang outlines
// the 128 x 8 x 32 volume tile's `segment` into a real call (captures passed through the stack,
// 464 B of scratch) -- the build that faulted in round 1.  Measured neutral elsewhere.
#ifndef FSMI_HALO_FORCE_INLINE
#define FSMI_HALO_FORCE_INLINE 1
#endif
#if FSMI_HALO_FORCE_INLINE
#define FSMI_HALO_INL __attribute__((always_inline))
#else
#define FSMI_HALO_INL
#endif
#ifndef FSMI_WREG_BPREF
#define FSMI_WREG_BPREF 1                            // 0: A/B build, B fragments read just before their MFMAs
#endif
// MFMA products per MAC: 3 (default) = hi*hi + hi*lo + lo*hi, the ~22-bit split that keeps the
// fp32 parity (|dd| < 1e-3 px); 1 = hi*hi only -- one fp16 product with fp32 accumulation, the
// precision of the reference's own GPU path (fp16 autocast, scripts/run_demo.py:161).  The 1-product
// build is a separate library (libfsmi_fast.so, FSMI_PRECISION=fast): lo halves are neither
// computed nor stored, lo weight fragments never loaded.
#ifndef FSMI_NPROD
#define FSMI_NPROD 3
#endif
static_assert(FSMI_NPROD == 1 || FSMI_NPROD == 3, "FSMI_NPROD: 1 or 3 MFMA products per MAC");
#ifndef FSMI_HALO_PERCOUT
#define FSMI_HALO_PERCOUT 1                          // 0: A/B build reading one weight scale (row 0's)
#endif

namespace fsmi {
namespace halo {

constexpr int kHMaxSeg = 4;        // input segments (zero-copy cat)

struct HaloArgs {
  const float* seg_ptr[kHMaxSeg];
  long long seg_bstride[kHMaxSeg];
  int seg_end[kHMaxSeg];
  int nseg, Cin, CinP;
  const _Float16* whi;             // [taps][CinP/32][CoutP][32]
  const _Float16* wlo;
  const float2* sb;                // per output channel (2^-wexp[co], bias[co]); weights packed x 2^wexp[co]
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
  int* ovf;                        // range flag (host-mapped; set to 1 when a scaled value overflows fp16)
  int pipe;                        // 2D register-weight tiles: the pipelined-staging variant (cfg 32 + c)
  // transposed-conv phase launches (fsmi_conv3d_up2_halo_x3 / fsmi_conv2d_up2_halo_x3; all 0
  // otherwise): the input window shifted by (sd, sh, sw) in {0, 1}, and output voxel (d, h, w)
  // written at (2d + od, 2h + oh, 2w + ow) of the (2D, 2H, 2W) output (2D maps: od = 0, D = 1),
  // whose channel stride is ocstride
  int up, sd, sh, sw, od, oh, ow;
  long long ocstride;
  // up == 2: all eight phases of a volume in one launch (blocks phase-major); up == 4: the four
  // phases of a 2D map.  Phase p's weights / scale-bias
  const _Float16* whi8[8];
  const _Float16* wlo8[8];
  const float2* sb8[8];
  // stride-2 volume launches (fsmi_conv3d_s2_halo_x3; str = 1 otherwise): D, H, W, cstride above are
  // the OUTPUT's, the input is (iD, iH, iW) with channel stride icstride; output voxel (d, h, w)
  // reads input (2d + kd - 1, 2h + kh - 1, 2w + kw - 1)
  int str, iD, iH, iW;
  long long icstride;
  // FeatureAtt gate (core/submodule.py:438-454) fused into a volume conv's epilogue: the final
  // value of output channel co at (d, h, w) is multiplied by sigmoid(fatt[b, co, h, w]),
  // fatt (B, Cout, H, W) contiguous; nullptr: no gate
  const float* fatt;
  unsigned long long* clk;         // in-kernel launch clock (timer mode 2 / eager timing; nullptr: off)
};

// Launch conv tile configuration `cfg` (0..9) for kernel size KS, 2D maps or NCDHW volumes
// (D3); defined in conv_halo_k<KS>_<2d|3d>.hip.  Returns FSMI_OK or an error code.
template <int KS, bool D3>
int launch_cfg(int cfg, int kg, const HaloArgs& a, hipStream_t s);

// Pointwise tiles (cfg 24-26, conv_pw.hip): 1x1 2D layers with an LDS-DMA input ring.
// pw_tile sets the tile geometry (a.nct = pixel tiles per image, npix, nco) before split-K.
int launch_pw(int cfg, const HaloArgs& a, hipStream_t s);
// stride-2 tiles, KS x KS (KS in {1, 3}) planes of the volume kernel (conv_halo_s2_3d.hip)
int launch_s2(int ks, int cfg, const HaloArgs& a, hipStream_t s);
// split-K reduce pass over a.ws (conv_halo_x3.hip)
void split_reduce(const HaloArgs& a, hipStream_t s);
void pw_tile(int cfg, HaloArgs& a);
// depth-blocked (17, 1, 1) volume tile (cfg 30, conv_depth.hip)
bool depth_conv_ok(const HaloArgs& a);
int launch_depth(HaloArgs& a, hipStream_t s);

// tiles with an in-block K-group (kg = 2) instantiation: the register-weight tiles that fit two
// waves per SIMD (<= 256 VGPRs) with 512-thread blocks
inline bool kg2_tile(int cfg) { return cfg == 3 || cfg == 4 || cfg == 5 || cfg == 7; }

}  // namespace halo

namespace {
using halo::HaloArgs;
using halo::kHMaxSeg;


typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x8 __attribute__((ext_vector_type(8)));

constexpr int HKC = 32;            // channels per chunk
constexpr int HROW = HKC + 8;      // padded LDS row (halves): conflict-free ds_read_b128 at 80-B stride


// erf without branches (tools/fit_erf.py: <= 2.4 ulp, mean 0.26 ulp over [-6, 6] in fp32 emulation):
// |z| < 1: z P(z^2); |z| >= 1: 1 - exp(-z^2) R(min(|z|, 4)) with R ~ erfcx on [1, 4] (erf is 1 in
// fp32 beyond 3.92).  Both halves are evaluated and one selected: the library erff branches on |z|,
// and a GELU's inputs straddle |z| = 1 within every wave, so each wave ran both paths plus the
// branch bookkeeping (~34 VALU per element vs ~25 here).
#ifndef FSMI_GELU_FAST
#define FSMI_GELU_FAST 1
#endif
__device__ __forceinline__ float erf_nb(float z) {
  const float t = z * z;
  float p = 7.847259258e-05f;
  p = fmaf(p, t, -8.008189034e-04f);
  p = fmaf(p, t, 5.188099109e-03f);
  p = fmaf(p, t, -2.685369179e-02f);
  p = fmaf(p, t, 1.128358245e-01f);
  p = fmaf(p, t, -3.761262596e-01f);
  p = fmaf(p, t, 1.128379107e+00f);
  const float small = z * p;
  const float az = fminf(fabsf(z), 4.f);
  float r = 1.498133884e-06f;
  r = fmaf(r, az, -4.378752783e-05f);
  r = fmaf(r, az, 5.791864241e-04f);
  r = fmaf(r, az, -4.594380967e-03f);
  r = fmaf(r, az, 2.443690039e-02f);
  r = fmaf(r, az, -9.241911769e-02f);
  r = fmaf(r, az, 2.575692832e-01f);
  r = fmaf(r, az, -5.418152213e-01f);
  r = fmaf(r, az, 8.737412691e-01f);
  r = fmaf(r, az, -1.082139969e+00f);
  r = fmaf(r, az, 9.922678471e-01f);
  const float e = __builtin_amdgcn_exp2f(-t * 1.4426950408889634f);   // exp(-z^2); underflows to 0 past |z| ~ 9.4
  const float big = copysignf(fmaf(-e, r, 1.f), z);
  return fabsf(z) < 1.f ? small : big;
}
__device__ __forceinline__ float gelu_erf_h(float x) {
#if FSMI_GELU_FAST
  return 0.5f * x * (1.f + erf_nb(x * 0.70710678118654752f));
#else
  return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
#endif
}
__device__ __forceinline__ float sigm_h(float x) { return 1.f / (1.f + expf(-x)); }

// Final value of output channel co at (b, sp) -- sp = d*H*W + h*W + w -- from the conv sum v in
// packed weight units (x 2^wexp[co]; the split-K partials): v * sb[co].x + sb[co].y, then:
//  act 0/1/2/6: out[b, co0+co] = res + gamma * alpha * act(v + bias)   (none / ReLU / GELU-erf /
//               LeakyReLU 0.01); with res_pre: gamma * alpha * act(v + bias + res)
//  act 7:       out[b, co0+co] = ReLU(v + bias + res) -- 2D maps: the rest of a conv whose other input
//               channels' contribution (+ bias) was computed once into res (a loop-invariant segment)
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
                                         float* __restrict__ out, const float2* __restrict__ sb,
                                         const float* __restrict__ gamma, const float* __restrict__ res,
                                         const float* __restrict__ gh, float* __restrict__ gz,
                                         const float* __restrict__ gatt, float* __restrict__ grh) {
  const long long HW = a.cstride;
  {
    const float2 q = sb[co];       // v: conv sum in packed units (split-K partials)
    v = v * q.x + q.y;
  }
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
  // FeatureAtt gate of volume convs: sigmoid(fatt[b, co, h, w]) (1 without one)
  float g = 1.f;
  if (RESPRE && a.fatt) {
    const long long P = static_cast<long long>(a.H) * a.W;
    g = sigm_h(a.fatt[(static_cast<long long>(b) * a.Cout + co) * P + hw % P]);
  }
  if ((RESPRE && a.res_pre) || a.act == 7) {   // ResNet tail / act 7: act(v + bias + res)
    v += res[b * a.res_bstride + static_cast<long long>(co) * HW + hw];
    *o = g * ((a.act == 1 || a.act == 7) ? fmaxf(v, 0.f) : (a.act == 6 ? (v >= 0.f ? v : 0.01f * v) : v));
    return;
  }
  if (a.act == 1) v = fmaxf(v, 0.f);
  else if (a.act == 2) v = gelu_erf_h(v);
  else if (a.act == 6) v = v >= 0.f ? v : 0.01f * v;
  v *= a.alpha;
  if (gamma) v *= gamma[co];
  if (res) v += res[b * a.res_bstride + static_cast<long long>(co) * HW + hw];
  *o = g * v;
}

template <bool RESPRE = true>
__device__ __forceinline__ void store_out(const HaloArgs& a, float v, int co, int b, long long hw) {
  store_el<RESPRE>(a, v, co, b, hw, a.out, a.sb, a.gamma, a.res, a.gh, a.gz, a.gatt, a.grh);
}

// Per-cout epilogue coefficients of one 16-row fragment (couts cb + (r&3) + 8(r>>2)): the
// (2^-wexp * xinv, bias) pair and gamma.  Loaded once per cout block of a tile: fetched per
// fragment they were a dependent L2/HBM round trip before each fragment's 16 stores -- 21-24 us of
// a 170-200 us block on the nsplit = 1 loop layers (tools/conv_phases.py, round 3).
struct FragCoef {
  float2 q[16];
  float g[16];
};

template <int ACT>
__device__ __forceinline__ void frag_coef(const HaloArgs& a, float xinv, int cb, const float2* __restrict__ sb,
                                          const float* __restrict__ gamma, FragCoef& c) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    c.q[r] = sb[min(cb + (r & 3) + 8 * (r >> 2), a.Cout - 1)];
    c.q[r].x *= xinv;
  }
  if constexpr (!(ACT >= 3 && ACT <= 5)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) c.g[r] = gamma ? gamma[min(cb + (r & 3) + 8 * (r >> 2), a.Cout - 1)] : 1.f;
  }
}

// One 16-element accumulator fragment (couts cb + (r&3) + 8(r>>2)) at one pixel, activation ACT
// fixed at compile time and one restrict scope: the fragment's residual / gate loads are issued
// together, then 16 branch-free finishes and stores.  (The generic store_el per element compiled to
// ~400 instructions per fragment with a wait per element: 20-56 % of a block's lifetime went to the
// epilogue on the nsplit = 1 layers, tools/conv_phases.py.)
template <int ACT, bool RESPRE>
__device__ __forceinline__ void store_frag_c(const HaloArgs& a, const f32x16& v, const FragCoef& c, int cb, int b,
                                             long long hw, int hw2, float* __restrict__ out,
                                             const float* __restrict__ res, const float* __restrict__ gh,
                                             float* __restrict__ gz, const float* __restrict__ gatt,
                                             float* __restrict__ grh) {
  // Every load of the fragment is issued before its first store: vmcnt counts loads and stores in
  // issue order, so a load placed after a store waits for that store's completion too -- with the
  // loads interleaved per element (and the residual load inside a per-element branch) the compiler
  // emitted s_waitcnt vmcnt(0) after every store, ~128 serialised store round trips per wave
  // (20 us of a 185 us block, round 3).  Rows past Cout only exist in the last cout tile.
  const long long HW = a.cstride;
  const long long OHW = a.up ? a.ocstride : HW;   // output channel stride (transposed conv)
  const bool full = (cb - (cb & 4)) + 32 <= a.Cout;          // all 32 rows of the fragment exist
  if constexpr (ACT >= 3 && ACT <= 5) {
    float ghv[16], gzv[16], ov[16];
    const float at = ACT == 3 ? 0.f : gatt[static_cast<size_t>(b) * HW + hw];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = min(cb + (r & 3) + 8 * (r >> 2), a.Cout - 1);
      const size_t g = (static_cast<size_t>(b) * a.gHd + (co % a.gHd)) * HW + hw;
      ghv[r] = (ACT != 3 || co >= a.gHd) ? gh[g] : 0.f;
      gzv[r] = ACT != 3 ? gz[g] : 0.f;
      ov[r] = ACT == 5 ? out[b * a.out_bstride + static_cast<long long>(a.co0 + co) * HW + hw] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = cb + (r & 3) + 8 * (r >> 2);
      if (!full && co >= a.Cout) continue;
      const float x = v[r] * c.q[r].x + c.q[r].y;
      const size_t g = (static_cast<size_t>(b) * a.gHd + (co % a.gHd)) * HW + hw;
      if constexpr (ACT == 3) {
        const float sg = sigm_h(x);
        if (co < a.gHd) gz[g] = sg;
        else grh[g] = sg * ghv[r];
      } else {
        const float z = gzv[r];
        const float hn = (1.f - z) * ghv[r] + z * tanhf(x);
        float* o = out + b * a.out_bstride + static_cast<long long>(a.co0 + co) * HW + hw;
        if constexpr (ACT == 4) *o = hn * at;
        else *o = ov[r] + hn * (1.f - at);
      }
    }
    return;
  } else {
    const bool pre = (RESPRE && a.res_pre) || ACT == 7;
    // FeatureAtt gate (volumes only): sigmoid(fatt[b, co, hw2]), hw2 = h * W + w of the output plane
    const float* __restrict__ fatt = RESPRE ? a.fatt : nullptr;
    const long long P = static_cast<long long>(a.H) * a.W;
    float rv[16], fv[16];
    if (res || fatt) {             // block-uniform; the common case has no loads at all
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = min(cb + (r & 3) + 8 * (r >> 2), a.Cout - 1);
        rv[r] = res ? res[b * a.res_bstride + static_cast<long long>(co) * HW + hw] : 0.f;
        fv[r] = fatt ? fatt[(static_cast<long long>(b) * a.Cout + co) * P + hw2] : 0.f;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) rv[r] = fv[r] = 0.f;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = cb + (r & 3) + 8 * (r >> 2);
      if (!full && co >= a.Cout) continue;
      float x = v[r] * c.q[r].x + c.q[r].y;
      if (pre) x += rv[r];         // ResNet tail / act 7: act(conv + bias + res)
      if constexpr (ACT == 1 || ACT == 7) x = fmaxf(x, 0.f);
      else if constexpr (ACT == 2) x = gelu_erf_h(x);
      else if constexpr (ACT == 6) x = x >= 0.f ? x : 0.01f * x;
      if (!pre) x = x * a.alpha * c.g[r] + rv[r];
      if (fatt) x *= sigm_h(fv[r]);
      out[b * a.out_bstride + static_cast<long long>(a.co0 + co) * OHW + hw] = x;
    }
  }
}

template <int ACT, bool RESPRE>
__device__ __forceinline__ void store_frag(const HaloArgs& a, const f32x16& v, float xinv, int cb, int b,
                                           long long hw, int hw2, float* __restrict__ out, const float2* __restrict__ sb,
                                           const float* __restrict__ gamma, const float* __restrict__ res,
                                           const float* __restrict__ gh, float* __restrict__ gz,
                                           const float* __restrict__ gatt, float* __restrict__ grh) {
  FragCoef c;
  frag_coef<ACT>(a, xinv, cb, sb, gamma, c);
  store_frag_c<ACT, RESPRE>(a, v, c, cb, b, hw, hw2, out, res, gh, gz, gatt, grh);
}

// 4 consecutive pixels of one channel, one restrict scope
__device__ __forceinline__ void store4(const HaloArgs& a, const float (&v)[4], int co, int b, long long hw,
                                       float* __restrict__ out, const float2* __restrict__ sb,
                                       const float* __restrict__ gamma, const float* __restrict__ res,
                                       const float* __restrict__ gh, float* __restrict__ gz,
                                       const float* __restrict__ gatt, float* __restrict__ grh) {
  // the split-K reduce's epilogue for 4 consecutive pixels: every operand load (gates, residual,
  // FeatureAtt gate) is issued before the first store -- interleaved, each load waited for the
  // stores issued ahead of it (vmcnt counts both in order)
  const long long HW = a.cstride;
  const float2 q = sb[co];
  if (a.act >= 3 && a.act <= 5) {
    const size_t g = (static_cast<size_t>(b) * a.gHd + (co % a.gHd)) * HW + hw;
    float hv[4], zv[4], ov[4], at[4];
    float* o = out + b * a.out_bstride + static_cast<long long>(a.co0 + co) * HW + hw;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      hv[k] = (a.act != 3 || co >= a.gHd) ? gh[g + k] : 0.f;
      zv[k] = a.act != 3 ? gz[g + k] : 0.f;
      ov[k] = a.act == 5 ? o[k] : 0.f;
      at[k] = a.act != 3 ? gatt[static_cast<size_t>(b) * HW + hw + k] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float x = v[k] * q.x + q.y;
      if (a.act == 3) {
        const float sg = sigm_h(x);
        if (co < a.gHd) gz[g + k] = sg;
        else grh[g + k] = sg * hv[k];
      } else {
        const float hn = (1.f - zv[k]) * hv[k] + zv[k] * tanhf(x);
        o[k] = a.act == 4 ? hn * at[k] : ov[k] + hn * (1.f - at[k]);
      }
    }
    return;
  }
  float rv[4], fv[4];
  const long long P = static_cast<long long>(a.H) * a.W;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    rv[k] = res ? res[b * a.res_bstride + static_cast<long long>(co) * HW + hw + k] : 0.f;
    fv[k] = a.fatt ? a.fatt[(static_cast<long long>(b) * a.Cout + co) * P + (hw + k) % P] : 0.f;
  }
  const float gm = gamma ? gamma[co] : 1.f;
  float* o = out + b * a.out_bstride + static_cast<long long>(a.co0 + co) * HW + hw;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float x = v[k] * q.x + q.y;
    if (a.res_pre || a.act == 7) {   // ResNet tail / act 7: act(v + bias + res)
      x += rv[k];
      x = (a.act == 1 || a.act == 7) ? fmaxf(x, 0.f) : (a.act == 6 ? (x >= 0.f ? x : 0.01f * x) : x);
    } else {
      if (a.act == 1) x = fmaxf(x, 0.f);
      else if (a.act == 2) x = gelu_erf_h(x);
      else if (a.act == 6) x = x >= 0.f ? x : 0.01f * x;
      x = x * a.alpha * gm + rv[k];
    }
    if (a.fatt) x *= sigm_h(fv[k]);
    o[k] = x;
  }
}

// ---------------------------------------------------------------- shared pieces

// The input segments (zero-copy cat) of batch b as uniform base pointers: channel ci (of the
// concatenated input) at element offset `off` of its plane is p[q] + ci * HW + off, q the segment
// holding ci -- p[q] is segment q's pointer for batch b moved back by its first channel's HW
// multiple.  Computed once per staging call from kernel arguments (scalar registers); per lane
// only the segment select and one multiply-add remain (the per-lane select of pointer, batch
// stride and first channel plus two 64-bit products was ~60 VALU per 8-channel task).
// chan() returns a GLOBAL (address space 1) pointer: a pointer rebuilt from an integer is generic,
// and loads through it were flat_load_dword -- which count in lgkmcnt as well as vmcnt, so every
// LDS operand wait after a chunk's halo loads also waited for those HBM loads (round 5).
#ifndef FSMI_HALO_FLAT
#define FSMI_HALO_FLAT 0                             // 1: the round-4 generic pointers (A/B build only)
#endif
#if FSMI_HALO_FLAT
typedef const float* gcfptr;
#else
typedef const __attribute__((address_space(1))) float* gcfptr;
#endif

struct SegBases {
  uintptr_t p[kHMaxSeg];
  __device__ __forceinline__ void init(const HaloArgs& a, int b, long long HW) {
    int start = 0;
#pragma unroll
    for (int q = 0; q < kHMaxSeg; ++q) {
      p[q] = reinterpret_cast<uintptr_t>(a.seg_ptr[q]) +
             static_cast<uintptr_t>(b * a.seg_bstride[q] - static_cast<long long>(start) * HW) * sizeof(float);
      start = a.seg_end[q];
    }
  }
  __device__ __forceinline__ gcfptr chan(const HaloArgs& a, int ci, long long HW) const {
    uintptr_t sp = p[0];
#pragma unroll
    for (int q = 1; q < kHMaxSeg; ++q) sp = (q < a.nseg && ci >= a.seg_end[q - 1]) ? p[q] : sp;
    return reinterpret_cast<gcfptr>(sp) + static_cast<long long>(ci) * HW;
  }
};

// Input-halo staging for a TR x 32 pixel tile: task = (halo pixel, 8-channel
// group); per task a packed descriptor (clamped pixel offset << 3 | in-image << 2
// | group) computed once per block; a chunk is loaded into registers one chunk
// ahead and split into fp16 hi/lo when stored to LDS.
// DEFER: keep the raw loads and mask them where they are read (absmax / store), so the loads stay in
// flight until then; otherwise they are masked on arrival -- which the compiler schedules right after
// the loads, waiting on them there (the default, kept for the tuned tiles' register budgets).
template <int KS, int TR, int STR = 1, bool DEFER = false>
struct HaloStage {
  // STR = 2: a stride-2 conv's window, (2 TR + 1) x 65 input pixels for TR x 32 outputs
  static constexpr int PD = KS / 2, HR = STR * (TR - 1) + KS, HC = STR * 31 + KS, NHP = HR * HC;
  static constexpr int X_TASKS = NHP * (HKC / 8), X_PER_T = (X_TASKS + 255) / 256;
  int desc[X_PER_T];
  int lim[DEFER ? X_PER_T : 1];    // DEFER: channels of task u's group that hold data (0 outside)
  f32x8 xv[X_PER_T];

  __device__ __forceinline__ void init(const HaloArgs& a, int tid, int r0, int c0) {
#pragma unroll
    for (int u = 0; u < X_PER_T; ++u) {
      const int task = min(tid + 256 * u, X_TASKS - 1);
      const int hp = task % NHP, g = task / NHP;
      const int hr = hp / HC, hc = hp - hr * HC;
      const int IH = STR == 1 ? a.H : a.iH, IW = STR == 1 ? a.W : a.iW;   // input plane
      const int hh = STR * r0 + hr - PD + a.sh, ww = STR * c0 + hc - PD + a.sw;
      const bool in = hh >= 0 && hh < IH && ww >= 0 && ww < IW && tid + 256 * u < X_TASKS;
      const int pix = min(max(hh, 0), IH - 1) * IW + min(max(ww, 0), IW - 1);
      desc[u] = (pix << 3) | (in ? 4 : 0) | g;
    }
  }

  // chunk cc of input depth plane d (zeros outside [0, D))
  __device__ __forceinline__ void load(const HaloArgs& a, int b, int cc, int d = 0) {
    const long long HW = STR == 1 ? a.cstride : a.icstride;
    const int ID = STR == 1 ? a.D : a.iD;
    const bool full = (cc + 1) * HKC <= a.Cin;     // block-uniform: only the last chunk is ragged
    const bool plane_ok = d >= 0 && d < ID;
    const long long poff = static_cast<long long>(min(max(d, 0), ID - 1)) *
                           (STR == 1 ? a.H * a.W : a.iH * a.iW);
    SegBases seg;
    seg.init(a, b, HW);
#pragma unroll
    for (int u = 0; u < X_PER_T; ++u) {
      const int g = desc[u] & 3, pix = desc[u] >> 3;
      const int ci0 = cc * HKC + g * 8;
      const int cic = min(ci0, a.Cin - 1);
      // segment of this 8-channel group (segments hold multiples of 8 channels): a select chain
      // over constant indices, so the kernarg arrays are never indexed per lane
      const gcfptr src = seg.chan(a, cic, HW) + poff + pix;
      const bool ok = (desc[u] & 4) && plane_ok;
      if constexpr (DEFER) {
        // one input segment of < 4 GB per batch item (the launcher checks): byte offsets from the
        // block-uniform base, channel j of the group at ob0 + j * HW * 4, clamped to the group's last
        // channel with one min (offsets grow with j) -- two VALU per load instead of a 64-bit product
        const int nv = a.Cin - ci0;                // may be <= 0 in the padded tail
        const int last = max(0, min(nv, 8) - 1);
        const unsigned hwb = static_cast<unsigned>(HW) * 4u;
        const unsigned ob0 = (static_cast<unsigned>(cic) * static_cast<unsigned>(HW) +
                              static_cast<unsigned>(poff) + static_cast<unsigned>(pix)) * 4u;
        const unsigned oblast = ob0 + static_cast<unsigned>(last) * hwb;
        using gccptr = const __attribute__((address_space(1))) char*;
        const gccptr base = reinterpret_cast<gccptr>(seg.p[0]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const unsigned ob = full ? ob0 + j * hwb : min(ob0 + j * hwb, oblast);
          xv[u][j] = *reinterpret_cast<gcfptr>(base + ob);
        }
        lim[u] = ok ? (full ? 8 : max(0, min(nv, 8))) : 0;
        (void)src;
      } else {
        f32x8 v;
        if (full) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = src[static_cast<size_t>(j) * HW];
        } else {
          const int nv = a.Cin - ci0;              // may be <= 0 in the padded tail
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
  }

  // largest |x| of the chunk this thread holds (zero padding included; NaN ignored here, it still
  // propagates through the products)
  __device__ __forceinline__ float absmax() const {
    float m = 0.f;
#pragma unroll
    for (int u = 0; u < X_PER_T; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, !DEFER || j < lim[DEFER ? u : 0] ? fabsf(xv[u][j]) : 0.f);
    return m;
  }

  // split x * 2^s (scale = 2^s, the block exponent) into fp16 hi + lo; ovf |= an x whose scaled
  // value leaves fp16's range
  template <int RMODE>
  __device__ __forceinline__ void store(_Float16 (*Xh)[HROW], _Float16 (*Xl)[HROW], int tid, float scale,
                                        bool& ovf) const {
#pragma unroll
    for (int u = 0; u < X_PER_T; ++u) {
      const int task = tid + 256 * u;
      if (X_TASKS % 256 == 0 || task < X_TASKS) {
        const int hp = task % NHP, g = task / NHP;
        f32x8 x;
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = !DEFER || j < lim[DEFER ? u : 0] ? xv[u][j] * scale : 0.f;
        if constexpr (RMODE == 2) {               // largest scaled |x| of the task, one compare after
          float m = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(x[j]));
          ovf |= m >= 65504.f;                    // (an inf input flags too; NaN is ignored by fmax)
        }
        const half8 hi = __builtin_convertvector(x, half8);
        *reinterpret_cast<half8*>(&Xh[hp][g * 8]) = hi;
        if constexpr (FSMI_NPROD == 3) {
          const half8 lo = __builtin_convertvector(x - __builtin_convertvector(hi, f32x8), half8);
          *reinterpret_cast<half8*>(&Xl[hp][g * 8]) = lo;
        }
      }
    }
  }
};

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>());
    static_for<B + 1, E>(f);
  }
}

struct TileCoord {
  int m0, b, d0, r0, c0, split;
};

// ---- range-safe split: a block exponent per 32-channel chunk
// fp16 hi / lo halves hold x to ~22 bits only while |x| < 65504 and x's low half stays normal
// (|x| >~ 0.1).  Before a chunk is split, the block takes the largest |x| of the chunk (wave
// reduce + one LDS slot per wave, read after the staging barrier the kernel has anyway) and
// scales the chunk by 2^s so that max|x| * 2^s lies in [2^14, 2^15): the hi halves never overflow
// and every value within 2^-17 of the chunk maximum keeps its full 22 bits.  s only decreases
// over a block's chunks; when it does, the fp32 accumulators are rescaled by the exact power of
// two, and the epilogue multiplies by 2^-s.  Values far below the chunk maximum lose low bits
// only at ~2^-40 of that maximum -- below the fp32 rounding of the sum they are added to.
constexpr int kNoExp = 127;                          // no chunk seen yet / all-zero chunks

// max over the wave of v >= 0: DPP row shifts within each 16-lane row, then the row_bcast:15 /
// row_bcast:31 steps of the GFX9 scan idiom (all VALU, no LDS round trip); lane 63 ends with the
// wave max, read into an SGPR.  Lanes without a DPP source read 0, harmless for a max of v >= 0.
__device__ __forceinline__ float wave_max(float v) {
  int x = __float_as_int(v);
  x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false))));
  x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false))));
  x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false))));
  x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false))));
  x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false))));
  x = __float_as_int(fmaxf(__int_as_float(x), __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false))));
  return __int_as_float(__builtin_amdgcn_readlane(x, 63));
}

__device__ __forceinline__ float exp2i(int e) {     // 2^e for e in [-126, 127], exact
  return __uint_as_float(static_cast<unsigned>(e + 127) << 23);
}

// target exponent for a chunk whose largest |x| is m (kNoExp when m == 0): max * 2^s in
// [2^(14-headroom), 2^(15-headroom))
template <int HEADROOM = 0>
__device__ __forceinline__ int chunk_exp(float m) {
  if (!(m > 0.f)) return kNoExp;
  const int e = static_cast<int>((__float_as_uint(m) >> 23) & 0xff) - 127;   // floor(log2 m); m < 2^-126 -> -127
  return min(max(14 - HEADROOM - e, -126), 126);
}

// range mode 2: the block's first chunk fixes its exponent with 8 bits of headroom, so later
// chunks up to 2^9 x larger still fit fp16; a value beyond that raises the range flag instead
// (fsmi_range_status) -- no per-chunk reduction and no accumulator rescale in the main loop.
// The one-product build (FSMI_NPROD = 1) keeps no lo half, so its hi half holds fp16's 11 bits for
// any value in fp16's normal range whatever the scale: there the first chunk's maximum is aimed at
// [2, 4) (13 bits of headroom), so later chunks up to 2^14 x larger still fit.
constexpr int kRangeHeadroom = FSMI_NPROD == 1 ? 13 : 8;

__device__ __forceinline__ void flag_overflow(const HaloArgs& a, bool ovf) {
  if (ovf && a.ovf) *a.ovf = 1;    // vector store from the lanes that saw one (same value, benign race)
}

constexpr int kHeadroom3 = 4;
constexpr int kHeadroom1 = 4;       // mode 1: exponent re-aimed 4 bits below a chunk's fit

// mode 3: does any lane's chunk value overflow fp16 at scale 2^sx?  One flag word per wave.
__device__ __forceinline__ void range3_check(int* rflag, float local_max, int sx, int lane, int wave) {
  const bool need = local_max * exp2i(sx == kNoExp ? 0 : sx) >= 32768.f;
  const unsigned long long any = __builtin_amdgcn_ballot_w64(need);
  if (lane == 0) rflag[wave] = any != 0ull;
}

__device__ __forceinline__ bool range3_any(const int* rflag) {
  const int4 f = *reinterpret_cast<const int4*>(rflag);
  return (f.x | f.y | f.z | f.w) != 0;
}

__device__ __forceinline__ float red4_max(const float* red) {
  const float4 r = *reinterpret_cast<const float4*>(red);       // one ds_read_b128
  return fmaxf(fmaxf(r.x, r.y), fmaxf(r.z, r.w));
}

template <int TM, int TN>
__device__ __forceinline__ void rescale_acc(f32x16 (&acc)[TM][TN], float f) {
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] *= f;
}

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
__device__ __forceinline__ TileCoord decode_tile(const HaloArgs& a, unsigned bid, unsigned nblocks) {
  const unsigned item = xcd_remap(bid, nblocks);
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
      if constexpr (FSMI_NPROD == 3) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
      }
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
    }
}

// The block's per-cout epilogue coefficients, staged into LDS at the start of the kernel (their
// global loads hidden under the main loop): lsb[c] = (2^-wexp, bias) and lg[c] = gamma of cout
// m0 + c (clamped to Cout - 1).  Fetched from global memory per fragment in the epilogue they were a
// dependent L2/HBM round trip before each fragment's 16 stores -- 21-24 us of a 170-200 us block on
// the nsplit = 1 loop layers (tools/conv_phases.py, round 3); from LDS each is ~100 cycles, and one
// fragment's coefficients at a time keep the register peak of the per-fragment loads.
template <int BM>
struct EpiCoef {
  float2 sb[BM];
  float g[BM];
  __device__ __forceinline__ void fill(const HaloArgs& a, int m0, int tid, int nthreads) {
    for (int e = tid; e < BM; e += nthreads) {
      const int co = min(m0 + e, a.Cout - 1);
      sb[e] = a.sb[co];
      g[e] = a.gamma ? a.gamma[co] : 1.f;
    }
  }
};

template <int ACT>
__device__ __forceinline__ void frag_coef_lds(float xinv, int cl, const float2* lsb, const float* lg, FragCoef& c) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    c.q[r] = lsb[cl + (r & 3) + 8 * (r >> 2)];
    c.q[r].x *= xinv;
  }
  if constexpr (!(ACT >= 3 && ACT <= 5)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) c.g[r] = lg[cl + (r & 3) + 8 * (r >> 2)];
  }
}

// Non-split epilogue of the block's tile with the activation fixed at compile time.  UP: the
// instantiation may run transposed-conv phases (volumes, and the 2x2 kernel on 2D maps)
template <int ACT, int TM, int TN, bool D3, bool UP = D3>
__device__ __forceinline__ void epi_tile(const HaloArgs& a, const f32x16 (&acc)[TM][TN], float xinv, const TileCoord& t,
                                         int wm, int wn, int lane, unsigned fown, const float2* lsb, const float* lg) {
  const int hsel = lane >> 5, rl = lane & 31;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int hh = t.r0 + wn * TN + j, ww = t.c0 + rl;
    if (hh >= a.H || ww >= a.W) continue;
    // transposed-conv phases (KS == 2 on 2D maps, or any volume launch with up set): the output
    // pixel of input (d0, hh, ww) in phase (od, oh, ow); 2D maps have d0 = od = 0
    const long long hw = UP && a.up
                             ? (static_cast<long long>(2 * t.d0 + a.od) * 2 * a.H + 2 * hh + a.oh) * 2 * a.W + 2 * ww + a.ow
                             : static_cast<long long>(t.d0) * a.H * a.W + hh * a.W + ww;
#pragma unroll
    for (int i = 0; i < TM; ++i)
      if ((fown >> (i * TN + j)) & 1u) {
        const int cl = (wm * TM + i) * 32 + 4 * hsel;
        FragCoef c;
        frag_coef_lds<ACT>(xinv, cl, lsb, lg, c);
        store_frag_c<ACT, D3>(a, acc[i][j], c, t.m0 + cl, t.b, hw, hh * a.W + ww, a.out, a.res, a.gh, a.gz, a.gatt,
                              a.grh);
      }
  }
}

// n = lane&31 is the pixel column, tile row wn*TN + j; D row map of the 32x32 MFMA
template <int TM, int TN, bool D3, bool UP = D3>
__device__ __forceinline__ void conv_epilogue(const HaloArgs& a, const f32x16 (&acc)[TM][TN], float xinv,
                                              const TileCoord& t, int wm, int wn, int lane, bool partial,
                                              const float2* lsb, const float* lg, unsigned fown = ~0u) {
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
      for (int i = 0; i < TM; ++i) {
        if (!((fown >> (i * TN + j)) & 1u)) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = t.m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hsel;
          if (co < a.Cout) wp[static_cast<size_t>(co) * HW] = acc[i][j][r] * xinv;   // packed units
        }
      }
    }
    return;
  }
  switch (a.act) {                 // uniform: one specialised tile epilogue per activation
    case 1: epi_tile<1, TM, TN, D3, UP>(a, acc, xinv, t, wm, wn, lane, fown, lsb, lg); break;
    case 2: epi_tile<2, TM, TN, D3, UP>(a, acc, xinv, t, wm, wn, lane, fown, lsb, lg); break;
    case 3: epi_tile<3, TM, TN, D3, UP>(a, acc, xinv, t, wm, wn, lane, fown, lsb, lg); break;
    case 4: epi_tile<4, TM, TN, D3, UP>(a, acc, xinv, t, wm, wn, lane, fown, lsb, lg); break;
    case 5: epi_tile<5, TM, TN, D3, UP>(a, acc, xinv, t, wm, wn, lane, fown, lsb, lg); break;
    case 6: epi_tile<6, TM, TN, D3, UP>(a, acc, xinv, t, wm, wn, lane, fown, lsb, lg); break;
    case 7: epi_tile<7, TM, TN, D3, UP>(a, acc, xinv, t, wm, wn, lane, fown, lsb, lg); break;
    default: epi_tile<0, TM, TN, D3, UP>(a, acc, xinv, t, wm, wn, lane, fown, lsb, lg); break;
  }
}

// ---------------------------------------------------------------- cfg 0/1: weights through LDS

template <int KS, int BM, int TR, int WM, bool D3>
__global__ __launch_bounds__(256) void conv_halo_x3_kernel(HaloArgs a) {
  FSMI_TIMELINE_CLOCK(a.clk);
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM / 32, TN = TR / WN;
  constexpr int NTAP = KS * KS;
  constexpr int W_PIECES = BM * HKC / 8;           // 16-B pieces per hi (or lo) weight slice
  constexpr int W_PER_T = W_PIECES / 256;
  static_assert(W_PIECES % 256 == 0, "weight pieces must tile the block");
  using HS = HaloStage<KS, TR>;
  constexpr int RM = range_mode<D3>();
  __shared__ __attribute__((aligned(16))) _Float16 Xh[HS::NHP][HROW];
  __shared__ __attribute__((aligned(16))) _Float16 Xl[HS::NHP][HROW];
  __shared__ __attribute__((aligned(16))) _Float16 Wh[2][BM][HROW];
  __shared__ __attribute__((aligned(16))) _Float16 Wl[2][BM][HROW];
  __shared__ __attribute__((aligned(16))) float red[4];   // per-wave chunk max |x| (block exponent)
  __shared__ __attribute__((aligned(16))) int rflag[4];   // per-wave 'chunk overflows the exponent' (mode 3)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int hsel = lane >> 5, rl = lane & 31;
  const TileCoord tc = decode_tile<BM, TR, D3>(a, blockIdx.x, gridDim.x);
  const int m0 = tc.m0;
  const int nck = a.CinP / HKC;
  const int nq = D3 ? a.KD * nck : nck;            // chunks = (kd, 32-channel chunk) pairs, kd major
  __shared__ EpiCoef<BM> ecoef;                    // visible to the epilogue after the main loop's barriers
  if (a.nsplit == 1) ecoef.fill(a, m0, tid, 256);

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
  if constexpr (D3) hs.load(a, tc.b, cc_begin % nck, tc.d0 + cc_begin / nck - a.PDD + a.sd);
  else hs.load(a, tc.b, cc_begin);
  int sx = kNoExp;                 // block exponent of the split (see chunk_exp)
  bool ovf = false;
  constexpr bool m1 = RM == 1;     // per-chunk exponent (mode 1)
  for (int cc = cc_begin; cc < cc_end; ++cc) {
    if constexpr (RM == 3) {
      const float lm = hs.absmax();
      if (cc == cc_begin) {
        const float m = wave_max(lm);
        if (lane == 0) red[wave] = m;
      } else {
        range3_check(rflag, lm, sx, lane, wave);
      }
    } else if (m1 || (RM == 2 && sx == kNoExp)) {
      const float m = wave_max(hs.absmax());
      if (lane == 0) red[wave] = m;           // m is wave-uniform (SGPR)
    }
    __syncthreads();               // every wave is done with the previous chunk's halo; maxima visible
    if constexpr (RM == 3) {
      if (cc == cc_begin) {
        const float bm = red4_max(red);
        ovf |= !(bm <= 3.4e38f);
        sx = bm > 0.f ? __builtin_amdgcn_readfirstlane(chunk_exp<kHeadroom3>(bm)) : 0;
      } else if (__builtin_amdgcn_readfirstlane(range3_any(rflag))) {   // rare: beyond the headroom
        const float m = wave_max(hs.absmax());
        if (lane == 0) red[wave] = m;
        __syncthreads();
        const float bm = red4_max(red);
        ovf |= !(bm <= 3.4e38f);
        const int se = __builtin_amdgcn_readfirstlane(chunk_exp<kHeadroom3>(bm));
        if (se < sx) {
          rescale_acc<TM, TN>(acc, exp2i(se - sx));
          sx = se;
        }
      }
    } else if (m1) {
      const float bm = red4_max(red);
      ovf |= !(bm <= 3.4e38f);                  // an inf input (NaN is ignored by the max)
      // rescale only when the chunk does not fit the current exponent; then re-aim with headroom
      // so that the chunks after it rarely trigger another rescale
      if (__builtin_amdgcn_readfirstlane(chunk_exp(bm)) < sx) {
        const int se = __builtin_amdgcn_readfirstlane(chunk_exp<kHeadroom1>(bm));     // block-uniform
        if (sx != kNoExp) rescale_acc<TM, TN>(acc, exp2i(se - sx));
        sx = se;
      }
    } else if (RM == 2 && sx == kNoExp) {       // first chunk with a nonzero value
      sx = __builtin_amdgcn_readfirstlane(chunk_exp<kRangeHeadroom>(red4_max(red)));
    }
    hs.template store<RM>(Xh, Xl, tid, exp2i(sx == kNoExp ? 0 : sx), ovf);
    if (cc + 1 < cc_end) {
      if constexpr (D3) hs.load(a, tc.b, (cc + 1) % nck, tc.d0 + (cc + 1) / nck - a.PDD + a.sd);
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
  flag_overflow(a, ovf);
  conv_epilogue<TM, TN, D3, D3 || KS == 2>(a, acc, exp2i(sx == kNoExp ? 0 : -sx), tc, wm, wn, lane, a.nsplit > 1,
                                           ecoef.sb, ecoef.g);
}

// ---------------------------------------------------------------- cfg 2/3: weights in registers

// KG = 2 ("K groups"): the block runs two groups of four waves on one tile, each accumulating
// every other (kd, channel) chunk with its own halo buffers, and sums the two halves through LDS
// before the epilogue -- split-K inside one workgroup, with no partial sums through memory and
// no reduce pass; each group then runs the epilogue of half of the fragments.
// STR = 2: stride-2 volume conv (fsmi_conv3d_s2_halo_x3): the staged window covers the strided
// input footprint of the TR x 32 output tile and tap (dh, dw) of output (r, c) reads window pixel
// (2r + dh, 2c + dw).
template <int KS, int BM, int TR, int WM, bool D3, int KG = 1, int STR = 1>
__global__ __launch_bounds__(256 * KG) void conv_halo_wreg_kernel(HaloArgs a) {
  FSMI_TIMELINE_CLOCK(a.clk);
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM / 32, TN = TR / WN;
  constexpr int NTAP = KS * KS;
  static_assert(KG == 1 || KG == 2, "K groups: 1 or 2");
  static_assert(STR == 1 || (STR == 2 && D3 && (KS == 3 || KS == 1)), "stride 2: 3x3 / 1x1 tiles of the volume kernel");
  using HS = HaloStage<KS, TR, STR>;
  constexpr int RM = range_mode<D3>();
  __shared__ __attribute__((aligned(16))) _Float16 Xh[KG][HS::NHP][HROW];
  __shared__ __attribute__((aligned(16))) _Float16 Xl[KG][HS::NHP][HROW];
  __shared__ __attribute__((aligned(16))) float red[KG][4];   // per-wave chunk max |x| (block exponent)
  // K-group exchange (2 x 16 KB): the halo buffers when they are large enough, else its own
  constexpr bool XCH_IN_HALO = sizeof(_Float16) * KG * HS::NHP * HROW >= 16 * 256 * sizeof(float);
  __shared__ __attribute__((aligned(16))) float xch_own[(KG == 2 && !XCH_IN_HALO) ? 2 * 16 * 256 : 1];
  __shared__ EpiCoef<BM> ecoef;

  const int grp = KG == 1 ? 0 : static_cast<int>(threadIdx.x >> 8);
  const int tid = threadIdx.x & 255, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int hsel = lane >> 5, rl = lane & 31;
  const int nck = a.CinP / HKC;
  const int nq = D3 ? a.KD * nck : nck;            // chunks = (kd, 32-channel chunk) pairs, kd major
  unsigned long long* tsb = a.ts ? a.ts + static_cast<size_t>(blockIdx.x) * 40 : nullptr;
  if (tsb && threadIdx.x == 0) tsb[0] = wall_clock64();

  // one segment: chunks [cc_begin, cc_end) of tile tc (group g: cc_begin + g, + g + KG, ...);
  // partial: raw sums into ws slot tc.split
  auto segment = [&](const TileCoord& tc, int cc_begin, int cc_end, bool partial) FSMI_HALO_INL {
    // this lane's A-fragment rows (rows past Cout only feed outputs the epilogue drops:
    // clamped so every address is mapped, no zeroing needed)
    int wrow[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) wrow[i] = min(tc.m0 + (wm * TM + i) * 32 + rl, a.CoutP - 1) * HKC + 8 * hsel;
    half8 wf[2][TM][2][2];         // [buffer][i][k half][hi, lo]
    auto load_wf = [&](auto buf_c, int cc, int tap) FSMI_HALO_INL {
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
    _Float16 (*gXh)[HROW] = Xh[grp];
    _Float16 (*gXl)[HROW] = Xl[grp];
    float* gred = red[grp];

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int c_first = cc_begin + grp;              // this group's chunks: c_first, c_first + KG, ...
    const int n_g = c_first < cc_end ? (cc_end - c_first + KG - 1) / KG : 0;
    const int c_last = c_first + KG * max(n_g - 1, 0);

    // tap t of a chunk uses register buffer (t + P) & 1, P = chunk parity; each tap prefetches the
    // next.  The B fragments (LDS) of each (tap, k half) step are read one step ahead (as the
    // pipelined tiles), so a step's MFMAs never wait on their own reads' LDS latency.
    auto chunk = [&](auto par_c, int cc) FSMI_HALO_INL {
      // an even tap count (KS = 2) starts every chunk on buffer 0; an odd one alternates
      constexpr int P = (NTAP & 1) ? decltype(par_c)::value : 0;
      half8 bh[2][TN], bl[2][TN];  // [step parity][j]
      auto read_b = [&](auto s_c) FSMI_HALO_INL {  // B fragments of step S = 2 tap + k
        constexpr int S = decltype(s_c)::value;
        constexpr int tp = S / 2, k = S % 2, dh = tp / KS, dw = tp % KS;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int hp = ((wn * TN + j) * STR + dh) * HS::HC + STR * rl + dw;
          bh[S & 1][j] = *reinterpret_cast<const half8*>(&gXh[hp][16 * k + 8 * hsel]);
          bl[S & 1][j] = *reinterpret_cast<const half8*>(&gXl[hp][16 * k + 8 * hsel]);
        }
      };
      if constexpr (FSMI_WREG_BPREF) read_b(std::integral_constant<int, 0>());
      static_for<0, NTAP>([&](auto tap_c) FSMI_HALO_INL {
        constexpr int tap = decltype(tap_c)::value;
        constexpr bool last = tap + 1 == NTAP;
        if constexpr (((tap + P) & 1) == 0) {
          load_wf(std::integral_constant<int, 1>(), last ? min(cc + KG, c_last) : cc, last ? 0 : tap + 1);
        } else {
          load_wf(std::integral_constant<int, 0>(), last ? min(cc + KG, c_last) : cc, last ? 0 : tap + 1);
        }
        // issue the next tap's loads before this tap's MFMAs: unfenced, the scheduler sinks them
        // below the last MFMA and reuses the current buffer's registers -- a single buffer whose
        // L2 round trip every tap then waits on
        __builtin_amdgcn_sched_barrier(0);
        static_for<0, 2>([&](auto k_c) FSMI_HALO_INL {
          constexpr int k = decltype(k_c)::value, S = 2 * tap + k;
          if constexpr (FSMI_WREG_BPREF) {
            if constexpr (S + 1 < 2 * NTAP) read_b(std::integral_constant<int, S + 1>());   // next step's B
          } else {
            read_b(std::integral_constant<int, S>());   // A/B: this step's B, read just before its MFMAs
          }
          half8 ah[TM], al[TM];
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            ah[i] = wf[(tap + P) & 1][i][k][0];
            al[i] = wf[(tap + P) & 1][i][k][1];
          }
          mma3<TM, TN>(acc, ah, al, bh[S & 1], bl[S & 1]);
        });
        // keep the one-tap-ahead structure: without this fence the scheduler hoists every
        // tap's loads of the unrolled chunk to its top (500 registers, 1 wave per SIMD)
        __builtin_amdgcn_sched_barrier(0);
      });
    };
    int sx = kNoExp;               // block (group) exponent of the segment (see chunk_exp)
    bool ovf = false;
    constexpr bool m1 = RM == 1;     // per-chunk exponent (mode 1)
    // q-th chunk of this group (cc = c_first + KG q); both groups run the same number of stages
    // (barriers), a group past its last chunk idles through them
    auto stage = [&](int q) FSMI_HALO_INL {
      const int cc = c_first + KG * q;
      const bool valid = q < n_g;
      // mode 2 fixes the exponent at the first chunk holding a nonzero value (an all-zero first
      // chunk would otherwise leave scale 1 and drop small later values to fp16 subnormals)
      if (valid && (m1 || (RM == 2 && sx == kNoExp))) {
        const float m = wave_max(hs.absmax());
        if (lane == 0) gred[wave] = m;          // m is wave-uniform (SGPR)
      }
      __syncthreads();             // every wave is done with the previous chunk's halo; maxima visible
      if (tsb && threadIdx.x == 0 && q < 36) tsb[1 + q] = wall_clock64();
      if (valid) {
        if (m1) {
          const float bm = red4_max(gred);
          ovf |= !(bm <= 3.4e38f);              // an inf input (NaN is ignored by the max)
          // rescale only when the chunk does not fit the current exponent; then re-aim with headroom
          if (__builtin_amdgcn_readfirstlane(chunk_exp(bm)) < sx) {
            const int se = __builtin_amdgcn_readfirstlane(chunk_exp<kHeadroom1>(bm));   // group-uniform
            if (sx != kNoExp) rescale_acc<TM, TN>(acc, exp2i(se - sx));
            sx = se;
          }
        } else if (RM == 2 && sx == kNoExp) {
          sx = __builtin_amdgcn_readfirstlane(chunk_exp<kRangeHeadroom>(red4_max(gred)));
        }
        hs.template store<RM>(gXh, gXl, tid, exp2i(sx == kNoExp ? 0 : sx), ovf);
        if (cc + KG < cc_end && !(a.dbg & 2)) {
          if constexpr (D3) hs.load(a, tc.b, (cc + KG) % nck, STR * tc.d0 + (cc + KG) / nck - a.PDD + a.sd);
          else hs.load(a, tc.b, cc + KG);
        }   // in flight during this chunk's taps
      }
      __syncthreads();
    };
    if (n_g > 0) {
      load_wf(std::integral_constant<int, 0>(), c_first, 0);
      if constexpr (D3) hs.load(a, tc.b, c_first % nck, STR * tc.d0 + c_first / nck - a.PDD + a.sd);
      else hs.load(a, tc.b, c_first);
    }
    // chunks in pairs so every register-buffer index is static (parity 0, then 1)
    const int n_all = (cc_end - cc_begin + KG - 1) / KG;   // stages every group runs
    int q = 0;
    for (; q + 1 < n_all; q += 2) {
      stage(q);
      if (q < n_g) chunk(std::integral_constant<int, 0>(), c_first + KG * q);
      stage(q + 1);
      if (q + 1 < n_g) chunk(std::integral_constant<int, 1>(), c_first + KG * (q + 1));
    }
    if (q < n_all) {
      stage(q);
      if (q < n_g) chunk(std::integral_constant<int, 0>(), c_first + KG * q);
    }
    if (tsb && threadIdx.x == 0) tsb[37] = wall_clock64();
    flag_overflow(a, ovf);
    float xinv = exp2i(sx == kNoExp ? 0 : -sx);
    unsigned fown = ~0u;
    if constexpr (KG == 2) {
      // the other group's half of every fragment this group finishes, through LDS (the halo
      // buffers, free once both groups are past their last chunk): fragment f = i*TN + j is
      // finished by group f & 1 (group 0 when there is only one), in rounds of two fragments
      // (one per direction, 16 KB each)
      constexpr int F = TM * TN;
      float* xb = XCH_IN_HALO ? reinterpret_cast<float*>(&Xh[0][0][0]) : xch_own;
      float* xbB = XCH_IN_HALO ? reinterpret_cast<float*>(&Xl[0][0][0]) : xch_own + 16 * 256;
      fown = 0u;
#pragma unroll
      for (int pr = 0; pr < (F + 1) / 2; ++pr) {
        const int f0 = 2 * pr, f1 = 2 * pr + 1;      // f0 finished by group 0, f1 by group 1
        __syncthreads();
        if (grp == 1) {
#pragma unroll
          for (int r = 0; r < 16; ++r) xb[r * 256 + tid] = acc[f0 / TN][f0 % TN][r] * xinv;
        } else if (f1 < F) {
#pragma unroll
          for (int r = 0; r < 16; ++r) xbB[r * 256 + tid] = acc[f1 / TN][f1 % TN][r] * xinv;
        }
        __syncthreads();
        if (grp == 0) {
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[f0 / TN][f0 % TN][r] = acc[f0 / TN][f0 % TN][r] * xinv + xb[r * 256 + tid];
          fown |= 1u << f0;
        } else if (f1 < F) {
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[f1 / TN][f1 % TN][r] = acc[f1 / TN][f1 % TN][r] * xinv + xbB[r * 256 + tid];
          fown |= 1u << f1;
        }
      }
      xinv = 1.f;
    }
    conv_epilogue<TM, TN, D3, D3 || KS == 2>(a, acc, xinv, tc, wm, wn, lane, partial, ecoef.sb, ecoef.g, fown);
    if (tsb && threadIdx.x == 0) {
      tsb[38] = wall_clock64();
      tsb[39] = (static_cast<unsigned long long>(cc_end - cc_begin) << 32) | blockIdx.x;
    }
  };

  unsigned bid = blockIdx.x, nb = gridDim.x;
  if constexpr (KS == 2) {
    if (a.up == 2 || a.up == 4) {                  // transposed-conv phases, phase-major blocks
      nb = a.up == 2 ? nb / 8 : nb / 4;
      const int ph = static_cast<int>(bid / nb);
      bid -= static_cast<unsigned>(ph) * nb;
      // constant indices only (a dynamic index into the by-value args puts them in scratch)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (ph == q) {
          a.whi = a.whi8[q];
          a.wlo = a.wlo8[q];
          a.sb = a.sb8[q];
        }
      }
      if (a.up == 2) {
        a.sd = a.od = ph >> 2;
        a.sh = a.oh = (ph >> 1) & 1;
      } else {                                     // 2D map: phase = (oh, ow)
        a.sd = a.od = 0;
        a.sh = a.oh = ph >> 1;
      }
      a.sw = a.ow = ph & 1;
    }
  }
  const TileCoord tc = decode_tile<BM, TR, D3>(a, bid, nb);
  const int c0 = tc.split * a.kpc;
  if (a.nsplit == 1) ecoef.fill(a, tc.m0, threadIdx.x, 256 * KG);   // read after the main loop's barriers
  segment(tc, c0, min(nq, c0 + a.kpc), a.nsplit > 1);
}

// ---------------------------------------------------------------- cfg 32 + c: pipelined staging

// Tile c of the register-weight kernel for 2D maps (KG = 1, stride 1) with the next chunk's
// staging moved into the MFMA stream.  conv_halo_wreg_kernel stages a chunk between two barriers
// while the MFMA pipes idle: load (one chunk ahead) -> barrier -> split fp32 into fp16 hi / lo and
// store to LDS -> barrier -> 9 taps of MFMAs.  Here the halo is double-buffered in LDS: while the
// waves run chunk q's taps on buffer q & 1, the split + store of chunk q + 1 (its registers loaded
// during chunk q - 1) into buffer (q + 1) & 1 is issued after tap 0 (the VALU work co-issues
// between MFMAs, MI355X_MICROARCH.md: ~5 single-issue instructions hide per 32x32x16 MFMA gap), the
// loads of chunk q + 2 follow it, and ONE barrier closes the chunk.  Range mode 2 as the wreg
// kernel: the exponent comes from the first chunk with a nonzero value (a chunk that is still all
// zero takes one extra block-wide max + barrier, block-uniform and rare).  LDS: twice the halo
// (65 KB for TR = 4, 109 KB for TR = 8).
template <int KS, int BM, int TR, int WM>
__global__ __launch_bounds__(256) void conv_halo_pipe_kernel(HaloArgs a) {
  FSMI_TIMELINE_CLOCK(a.clk);
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM / 32, TN = TR / WN;
  constexpr int NTAP = KS * KS;
  constexpr int STAGE_TAP = NTAP > 1 ? 1 : 0;      // the tap whose MFMAs cover the next chunk's store
  using HS = HaloStage<KS, TR>;
  constexpr int RM = range_mode<false>();
  static_assert(RM == 2 || RM == 0, "pipelined tiles: range mode 2 (or none)");
  __shared__ __attribute__((aligned(16))) _Float16 Xh[2][HS::NHP][HROW];
  __shared__ __attribute__((aligned(16))) _Float16 Xl[2][HS::NHP][HROW];
  __shared__ __attribute__((aligned(16))) float red[4];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int hsel = lane >> 5, rl = lane & 31;
  const int nck = a.CinP / HKC;
  const TileCoord tc = decode_tile<BM, TR, false>(a, blockIdx.x, gridDim.x);
  __shared__ EpiCoef<BM> ecoef;                    // visible to the epilogue after the main loop's barriers
  if (a.nsplit == 1) ecoef.fill(a, tc.m0, tid, 256);
  const int c_first = tc.split * a.kpc;
  const int c_end = min(nck, c_first + a.kpc);
  const int n = c_end - c_first;                   // >= 1: no empty splits (run_halo)

  int wrow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) wrow[i] = min(tc.m0 + (wm * TM + i) * 32 + rl, a.CoutP - 1) * HKC + 8 * hsel;
  half8 wf[2][TM][2][2];           // [buffer][i][k half][hi, lo]
  auto load_wf = [&](auto buf_c, int cc, int tap) FSMI_HALO_INL {
    constexpr int buf = decltype(buf_c)::value;
    const size_t base = (static_cast<size_t>(tap) * nck + cc) * a.CoutP * HKC;
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

  int sx = kNoExp;
  bool ovf = false;
  auto scale = [&]() FSMI_HALO_INL { return RM == 2 ? exp2i(sx == kNoExp ? 0 : sx) : 1.f; };
  auto fix_exponent = [&]() FSMI_HALO_INL {        // block-wide max of the registers' chunk -> sx
    const float m = wave_max(hs.absmax());
    if (lane == 0) red[wave] = m;
    __syncthreads();
    sx = __builtin_amdgcn_readfirstlane(chunk_exp<kRangeHeadroom>(red4_max(red)));
  };
  // prologue: chunk 0 -> buffer 0 (its max fixes the exponent), chunk 1 into registers
  load_wf(std::integral_constant<int, 0>(), c_first, 0);
  hs.load(a, tc.b, c_first);
  if (RM == 2) fix_exponent();
  hs.template store<RM>(Xh[0], Xl[0], tid, scale(), ovf);
  if (n > 1) hs.load(a, tc.b, c_first + 1);
  __syncthreads();

  // chunk q on buffer P = q & 1; tap t uses weight buffer (t + PP) & 1 and prefetches tap t + 1.
  // The B fragments (LDS) of each (tap, k half) step are read one step ahead into the other half of
  // a double buffer, so a step's MFMAs never wait on the LDS latency of their own reads (only the
  // chunk's first step does: the next chunk's buffer is complete only after the closing barrier)
  auto chunk = [&](auto par_c, int q) FSMI_HALO_INL {
    constexpr int P = decltype(par_c)::value;
    constexpr int PP = (NTAP & 1) ? P : 0;
    const int cc = c_first + q;
    half8 bh[2][TN], bl[2][TN];    // [step parity][j]
    auto read_b = [&](auto s_c) FSMI_HALO_INL {    // B fragments of step S = 2 tap + k
      constexpr int S = decltype(s_c)::value;
      constexpr int tp = S / 2, k = S % 2, dh = tp / KS, dw = tp % KS;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int hp = ((wn * TN + j) + dh) * HS::HC + rl + dw;
        bh[S & 1][j] = *reinterpret_cast<const half8*>(&Xh[P][hp][16 * k + 8 * hsel]);
        bl[S & 1][j] = *reinterpret_cast<const half8*>(&Xl[P][hp][16 * k + 8 * hsel]);
      }
    };
    read_b(std::integral_constant<int, 0>());
    static_for<0, NTAP>([&](auto tap_c) FSMI_HALO_INL {
      constexpr int tap = decltype(tap_c)::value;
      constexpr bool last = tap + 1 == NTAP;
      if constexpr (((tap + PP) & 1) == 0) {
        load_wf(std::integral_constant<int, 1>(), last ? min(cc + 1, c_end - 1) : cc, last ? 0 : tap + 1);
      } else {
        load_wf(std::integral_constant<int, 0>(), last ? min(cc + 1, c_end - 1) : cc, last ? 0 : tap + 1);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (tap == STAGE_TAP && q + 1 < n) {
        // next chunk: registers (loaded one chunk ago) -> fp16 hi / lo -> the other buffer, then the
        // chunk after it into the registers
        if (RM == 2 && sx == kNoExp) fix_exponent();   // every chunk so far all zero (uniform)
        hs.template store<RM>(Xh[P ^ 1], Xl[P ^ 1], tid, scale(), ovf);
        if (q + 2 < n) hs.load(a, tc.b, cc + 2);
        __builtin_amdgcn_sched_barrier(0);
      }
      static_for<0, 2>([&](auto k_c) FSMI_HALO_INL {
        constexpr int k = decltype(k_c)::value, S = 2 * tap + k;
        if constexpr (S + 1 < 2 * NTAP) read_b(std::integral_constant<int, S + 1>());   // next step's B
        half8 ah[TM], al[TM];
        constexpr int wb = (tap + PP) & 1;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          ah[i] = wf[wb][i][k][0];
          al[i] = wf[wb][i][k][1];
        }
        mma3<TM, TN>(acc, ah, al, bh[S & 1], bl[S & 1]);
      });
      __builtin_amdgcn_sched_barrier(0);
    });
    __syncthreads();               // buffer P free; buffer P ^ 1 complete and visible
  };
  int q = 0;
  for (; q + 1 < n; q += 2) {
    chunk(std::integral_constant<int, 0>(), q);
    chunk(std::integral_constant<int, 1>(), q + 1);
  }
  if (q < n) chunk(std::integral_constant<int, 0>(), q);
  flag_overflow(a, ovf);
  conv_epilogue<TM, TN, false>(a, acc, exp2i(sx == kNoExp || RM != 2 ? 0 : -sx), tc, wm, wn, lane, a.nsplit > 1,
                                ecoef.sb, ecoef.g);
}

template <int KS, int BM, int TR, int WM, bool WREG, bool D3, int KG = 1, int STR = 1>
void launch_tile(const HaloArgs& a, hipStream_t s) {
  const unsigned grid = static_cast<unsigned>(a.npix) * a.nco * a.nsplit * (a.up == 2 ? 8 : a.up == 4 ? 4 : 1);
  if constexpr (WREG && !D3 && KG == 1 && STR == 1 && KS != 2) {
    if (a.pipe) {                                  // cfg 32 + c: the pipelined-staging variant
      hipLaunchKernelGGL((conv_halo_pipe_kernel<KS, BM, TR, WM>), dim3(grid), dim3(256), 0, s, a);
      return;
    }
  }
  if constexpr (WREG)
    hipLaunchKernelGGL((conv_halo_wreg_kernel<KS, BM, TR, WM, D3, KG, STR>), dim3(grid), dim3(256 * KG), 0, s, a);
  else hipLaunchKernelGGL((conv_halo_x3_kernel<KS, BM, TR, WM, D3>), dim3(grid), dim3(256), 0, s, a);
}

}  // namespace
}  // namespace fsmi

// tiles = couts x (rows x 32 px), as listed in conv_halo_x3.hip's tile_counts switch
#define FSMI_HALO_LAUNCH_CFG(KS, D3)                                                       \
  namespace fsmi {                                                                          \
  namespace halo {                                                                          \
  template <>                                                                               \
  int launch_cfg<KS, D3>(int cfg, int kg, const HaloArgs& a, hipStream_t s) {               \
    if (kg == 2) {                                                                          \
      switch (cfg) {                                                                        \
        case 3: launch_tile<KS, 128, 4, 2, true, D3, 2>(a, s); break;                       \
        case 4: launch_tile<KS, 128, 2, 2, true, D3, 2>(a, s); break;                       \
        case 5: launch_tile<KS, 64, 4, 1, true, D3, 2>(a, s); break;                        \
        case 7: launch_tile<KS, 32, 4, 1, true, D3, 2>(a, s); break;                        \
        default: set_error("fsmi_conv_halo: tile %d has no K-group variant", cfg); return FSMI_ERR_ARG; \
      }                                                                                     \
      return finish_launch("fsmi_conv_halo");                                               \
    }                                                                                       \
    switch (cfg) {                                                                          \
      case 0: launch_tile<KS, 64, 8, 1, false, D3>(a, s); break;                            \
      case 1: launch_tile<KS, 128, 4, 2, false, D3>(a, s); break;                           \
      case 2: launch_tile<KS, 64, 8, 1, true, D3>(a, s); break;                             \
      case 3: launch_tile<KS, 128, 4, 2, true, D3>(a, s); break;                            \
      case 4: launch_tile<KS, 128, 2, 2, true, D3>(a, s); break;                            \
      case 5: launch_tile<KS, 64, 4, 1, true, D3>(a, s); break;                             \
      case 6: launch_tile<KS, 32, 8, 1, true, D3>(a, s); break;                             \
      case 8: launch_tile<KS, 128, 8, 2, true, D3>(a, s); break;                            \
      case 9: launch_tile<KS, 256, 4, 4, true, D3>(a, s); break;                            \
      case 11:                                                                              \
        if constexpr (!D3 && KS != 2) launch_tile<KS, 256, 5, 4, true, D3>(a, s);           \
        else { set_error("fsmi_conv_halo: tile 11 is 2D only"); return FSMI_ERR_ARG; }      \
        break;                                                                              \
      default: launch_tile<KS, 32, 4, 1, true, D3>(a, s); break;                            \
    }                                                                                       \
    return finish_launch("fsmi_conv_halo");                                                 \
  }                                                                                         \
  }                                                                                         \
  }
