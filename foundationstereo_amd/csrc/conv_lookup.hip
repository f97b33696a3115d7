// The motion encoder's first conv with the geometry lookup fused into its input staging.
//
// convc1 (core/update.py:56,62: Conv2d(cor_planes, 256, 1) + ReLU) reads nothing but the lookup
// output of the same iteration (core/geometry.py:43-65): L levels x (Cv + 1) groups x (2r+1) taps,
// 80 MB per iteration at cfg2 written by geo_lookup_kernel and read straight back.  Here the 1x1
// conv's stager computes those values itself: a 32-channel chunk holds 3 whole (level, channel)
// groups of 9 taps (27 channels + 5 zero rows; the packed weights follow that order,
// ops.pack_lookup_conv), so each staging task is one (group, pixel): the 2r+1 interpolations of
// TapPairs (lookup_taps.h: the coordinate math of geo_lookup_kernel's Taps, so the same fp32
// values).  The window loads of chunk q+1 are issued before chunk q's MFMAs and
// interpolated after them into the other of two fp32 LDS slots.
//
// Block: all Cout <= 256 output channels (4 waves x 2 fragments: the lookup is computed once per
// pixel, not once per cout tile) x 64 consecutive pixels; split-K over chunks through the usual
// partials + reduce.  Range mode 1 (conv_halo.h): the exact block max of every staged chunk, the
// accumulators rescaled by powers of two when it grows.
#include "conv_halo.h"
#include "lookup_taps.h"

namespace fsmi {
namespace {

struct LookupConvArgs {
  const float* vol[FSMI_MAX_LEVELS];
  const float* cor[FSMI_MAX_LEVELS];
  const float* disp;               // (B, 1, H, W)
  int L, Cv, D, W2;
};

template <int R>
__global__ __launch_bounds__(256) void conv_lookup_kernel(HaloArgs a, LookupConvArgs f) {
  constexpr int K = 2 * R + 1, PX = 64, TM = 2, TN = 2, GPC = HKC / K;
  static_assert(GPC * K <= HKC && GPC * PX <= 256, "lookup chunk");
  __shared__ __attribute__((aligned(16))) float xs[2][HKC][PX];
  __shared__ __attribute__((aligned(16))) float red[2][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave, hsel = lane >> 5, rl = lane & 31;
  const int HW = a.H * a.W;
  const int G = f.L * (f.Cv + 1);
  const int nck = (G + GPC - 1) / GPC;

  const unsigned item = xcd_remap(blockIdx.x, gridDim.x);
  const int split = item / a.npix, ptile = item - split * a.npix;
  const int b = ptile / a.nct;
  const int px0 = (ptile - b * a.nct) * PX;
  const int c_begin = split * a.kpc, c_end = min(nck, c_begin + a.kpc), n = c_end - c_begin;

  for (int e = tid; e < 2 * (HKC - GPC * K) * PX; e += 256) {       // the zero rows, both slots
    const int sl = e / ((HKC - GPC * K) * PX), r = e % ((HKC - GPC * K) * PX);
    xs[sl][GPC * K + r / PX][r % PX] = 0.f;
  }

  // staging task of this thread: group sg of each chunk at pixel spx
  const bool stager = tid < GPC * PX;
  const int sg = __builtin_amdgcn_readfirstlane(tid / PX), spx = tid % PX;   // PX = 64: one group per wave
  const int hw = px0 + spx;
  const bool pin = stager && hw < HW;
  const float dsp = pin ? f.disp[static_cast<size_t>(b) * HW + hw] : 0.f;
  const int w = hw % a.W;
  TapPairs<R> tp;
  bool gval = false;
  auto fetch = [&](int c) FSMI_HALO_INL {          // the task's tap samples of chunk c (in flight)
    const int g = c * GPC + sg;
    gval = pin && g < G;
    const int gi = gval ? g : 0;
    const int i = gi / (f.Cv + 1), ch = gi - i * (f.Cv + 1);
    const float* vp = i == 0 ? f.vol[0] : (i == 1 ? f.vol[1] : (i == 2 ? f.vol[2] : f.vol[3]));
    const float* cp = i == 0 ? f.cor[0] : (i == 1 ? f.cor[1] : (i == 2 ? f.cor[2] : f.cor[3]));
    const float s = static_cast<float>(1 << i);
    const float ds = dsp / s;
    const bool geo = ch < f.Cv;
    const int Di = f.D >> i, W2i = f.W2 >> i;
    const float* src = geo ? vp + (static_cast<size_t>(b) * f.Cv + ch) * Di * HW + hw
                           : cp + (static_cast<size_t>(b) * HW + hw) * W2i;
    const int nn = geo ? Di : W2i;
    // an invalid task aims far left of the row: every load is predicated off (zeros)
    const float xc = !gval ? -1.0e5f : (geo ? ds : static_cast<float>(w) / s - ds);
    tp.load(src, geo ? static_cast<size_t>(HW) : size_t(1), nn, xc);
  };
  auto stage = [&](int slot) FSMI_HALO_INL {       // interpolate into slot; per-wave max |x|
    float m = 0.f;
    if (stager) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float x = gval ? tp.value(k) : 0.f;
        xs[slot][sg * K + k][spx] = x;
        m = fmaxf(m, fabsf(x));
      }
    }
    m = wave_max(m);
    if (lane == 0) red[slot][wave] = m;
  };

  int wrow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) wrow[i] = min((wm * TM + i) * 32 + rl, a.CoutP - 1) * HKC + 8 * hsel;
  half8 wf[2][TM][2][2];
  auto load_wf = [&](auto buf_c, int c) FSMI_HALO_INL {
    constexpr int buf = decltype(buf_c)::value;
    const size_t base = static_cast<size_t>(c) * a.CoutP * HKC;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        wf[buf][i][k][0] = *reinterpret_cast<const half8*>(a.whi + base + wrow[i] + 16 * k);
        wf[buf][i][k][1] = *reinterpret_cast<const half8*>(a.wlo + base + wrow[i] + 16 * k);
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
  for (int j = 0; j < TN; ++j) pix_ok[j] = px0 + j * 32 + rl < HW;

  int sx = kNoExp;
  float scale = 1.f;
  bool ovf = false;
  auto set_exp = [&](int slot) FSMI_HALO_INL {     // range mode 1 for the chunk just staged
    const float bm = red4_max(red[slot]);
    ovf |= !(bm <= 3.4e38f);
    if (__builtin_amdgcn_readfirstlane(chunk_exp(bm)) < sx) {
      const int se = __builtin_amdgcn_readfirstlane(chunk_exp<kHeadroom1>(bm));
      if (sx != kNoExp) rescale_acc<TM, TN>(acc, exp2i(se - sx));
      sx = se;
      scale = exp2i(sx);
    }
  };

  if (n > 0) {
    load_wf(std::integral_constant<int, 0>(), c_begin);
    fetch(c_begin);
    stage(0);
    __syncthreads();
    set_exp(0);
  }
  auto step = [&](auto par_c, int q) FSMI_HALO_INL {
    constexpr int P = decltype(par_c)::value;
    const int c = c_begin + q;
    const bool more = q + 1 < n;
    if (more) fetch(c + 1);                        // in flight during this chunk's MFMAs
    load_wf(std::integral_constant<int, P ^ 1>(), min(c + 1, c_end - 1));
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      half8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        ah[i] = wf[P][i][k][0];
        al[i] = wf[P][i][k][1];
      }
      const int ci0 = 16 * k + 8 * hsel;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x8 x;
        float mx = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          x[t] = pix_ok[j] ? xs[q & 1][ci0 + t][j * 32 + rl] * scale : 0.f;
          mx = fmaxf(mx, fabsf(x[t]));
        }
        ovf |= mx >= 65504.f;
        bh[j] = __builtin_convertvector(x, half8);
        if constexpr (FSMI_NPROD == 3) bl[j] = __builtin_convertvector(x - __builtin_convertvector(bh[j], f32x8), half8);
      }
      mma3<TM, TN>(acc, ah, al, bh, bl);
    }
    if (more) stage((q + 1) & 1);
    __syncthreads();
    if (more) set_exp((q + 1) & 1);
  };
  int q = 0;
  for (; q + 1 < n; q += 2) {
    step(std::integral_constant<int, 0>(), q);
    step(std::integral_constant<int, 1>(), q + 1);
  }
  if (q < n) step(std::integral_constant<int, 0>(), q);
  flag_overflow(a, ovf);

  const float xinv = exp2i(sx == kNoExp ? 0 : -sx);
  if (a.nsplit > 1) {                              // raw partials (packed units) into ws slot `split`
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (!pix_ok[j]) continue;
      const long long p = px0 + j * 32 + rl;
      float* wp = a.ws + (static_cast<size_t>(split) * a.B + b) * a.Cout * HW + p;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hsel;
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
      const long long p = px0 + j * 32 + rl;
#pragma unroll
      for (int i = 0; i < TM; ++i)
        store_frag<ACT, false>(a, acc[i][j], xinv, (wm * TM + i) * 32 + 4 * hsel, b, p, 0, a.out, a.sb, a.gamma, a.res,
                               a.gh, a.gz, a.gatt, a.grh);
    }
  };
  if (a.act == 1) epi(std::integral_constant<int, 1>());
  else epi(std::integral_constant<int, 0>());
}

}  // namespace
}  // namespace fsmi

using namespace fsmi;

extern "C" int fsmi_conv1x1_lookup(const float* const* vol_levels, const float* const* corr_levels, const float* disp,
                                   int num_levels, int radius, int B, int Cv, int D, int H, int W, int W2,
                                   const void* whi, const void* wlo, const float* scale_bias, float* out, int out_ctot,
                                   int co0, int Cout, int act, int nsplit, float* ws, long long ws_floats,
                                   void* stream) {
  FSMI_CHECK_ARG(vol_levels && corr_levels && disp && whi && wlo && scale_bias && out,
                 "fsmi_conv1x1_lookup: null pointer");
  FSMI_CHECK_ARG(num_levels >= 1 && num_levels <= FSMI_MAX_LEVELS, "fsmi_conv1x1_lookup: num_levels %d", num_levels);
  FSMI_CHECK_ARG(radius == 4, "fsmi_conv1x1_lookup: radius %d unsupported (4)", radius);
  FSMI_CHECK_ARG(B > 0 && Cv > 0 && H > 0 && W > 0 && Cout > 0 && Cout <= 256, "fsmi_conv1x1_lookup: bad shape");
  FSMI_CHECK_ARG((D >> (num_levels - 1)) >= 2 && (W2 >> (num_levels - 1)) >= 2,
                 "fsmi_conv1x1_lookup: level %d too short (D=%d, W2=%d)", num_levels - 1, D, W2);
  FSMI_CHECK_ARG(act == 0 || act == 1, "fsmi_conv1x1_lookup: act %d (0, 1)", act);
  FSMI_CHECK_ARG(co0 >= 0 && co0 + Cout <= out_ctot, "fsmi_conv1x1_lookup: output slice outside the tensor");
  FSMI_CHECK_ARG(reinterpret_cast<uintptr_t>(scale_bias) % 8 == 0, "fsmi_conv1x1_lookup: scale_bias alignment");
  LookupConvArgs f{};
  for (int i = 0; i < FSMI_MAX_LEVELS; ++i) {
    f.vol[i] = vol_levels[min(i, num_levels - 1)];
    f.cor[i] = corr_levels[min(i, num_levels - 1)];
    FSMI_CHECK_ARG(f.vol[i] && f.cor[i], "fsmi_conv1x1_lookup: null level %d", i);
  }
  f.disp = disp;
  f.L = num_levels;
  f.Cv = Cv;
  f.D = D;
  f.W2 = W2;
  const int K = 2 * radius + 1, GPC = 32 / K;
  const int nck = (num_levels * (Cv + 1) + GPC - 1) / GPC;
  const long long HW = static_cast<long long>(H) * W;
  HaloArgs a{};
  a.Cin = a.CinP = nck * 32;
  a.whi = static_cast<const _Float16*>(whi);
  a.wlo = static_cast<const _Float16*>(wlo);
  a.sb = reinterpret_cast<const float2*>(scale_bias);
  a.out = out;
  a.out_bstride = static_cast<long long>(out_ctot) * HW;
  a.co0 = co0;
  a.Cout = Cout;
  a.CoutP = (Cout + 31) / 32 * 32;
  a.B = B;
  a.H = H;
  a.W = W;
  a.D = 1;
  a.KD = 1;
  a.act = act;
  a.alpha = 1.f;
  a.cstride = HW;
  a.nrt = 1;
  a.nct = static_cast<int>((HW + 63) / 64);
  a.npix = B * a.nct;
  a.nco = 1;
  nsplit = max(1, min(nsplit, nck));
  a.kpc = (nck + nsplit - 1) / nsplit;
  a.nsplit = (nck + a.kpc - 1) / a.kpc;
  const long long per_split = static_cast<long long>(B) * Cout * HW;
  FSMI_CHECK_ARG(a.nsplit == 1 || (ws && per_split * a.nsplit <= ws_floats),
                 "fsmi_conv1x1_lookup: split-K %d needs %lld workspace floats", a.nsplit, per_split * a.nsplit);
  a.ws = ws;
  a.ovf = range_flag_device();
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_CONV2D, s);
  hipLaunchKernelGGL(conv_lookup_kernel<4>, dim3(static_cast<unsigned>(a.npix) * a.nsplit), dim3(256), 0, s, a, f);
  if (a.nsplit > 1) halo::split_reduce(a, s);
  return finish_launch("fsmi_conv1x1_lookup");
}
