// Halo-tiled split-precision convolution: host side (tile / split-K policy, C ABI entry points)
// and the split-K reduce pass.  Device code and its description: conv_halo.h.
#include <atomic>

#include "conv_halo.h"

namespace fsmi {
namespace {

// Sums the split-K partials in split order (deterministic) and applies the epilogue.
__global__ __launch_bounds__(256) void conv_split_reduce_kernel(HaloArgs a) {
  FSMI_TIMELINE_CLOCK(a.clk);
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
  FSMI_TIMELINE_CLOCK(a.clk);
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
  if ((a.act <= 2 || a.act == 6) && !a.res && !a.fatt) {      // plain epilogue: vector store
    const float2 q = a.sb[co];
    const float gg = a.gamma ? a.gamma[co] : 1.f;
    float r[4] = {v.x * q.x + q.y, v.y * q.x + q.y, v.z * q.x + q.y, v.w * q.x + q.y};
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
  store4(a, sv, co, b, hw, a.out, a.sb, a.gamma, a.res, a.gh, a.gz, a.gatt, a.grh);
}

template <int KS, int BM, int TR, int WM>
void tile_counts(HaloArgs& a) {
  a.nrt = (a.H + TR - 1) / TR;
  a.nct = (a.W + 31) / 32;
  a.npix = a.B * a.D * a.nrt * a.nct;
  a.nco = (a.Cout + BM - 1) / BM;
}

}  // namespace
}  // namespace fsmi

namespace fsmi {
namespace halo {

// the split-K reduce pass of a launch whose partials are in a.ws (also used by conv_lookup.hip)
void split_reduce(const HaloArgs& a_in, hipStream_t s) {
  HaloArgs a = a_in;
  const long long SP = a.cstride;
  const bool vec = SP % 4 == 0 && a.nsplit <= 8 && reinterpret_cast<uintptr_t>(a.out) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(a.ws) % 16 == 0 &&
                   (!a.res || reinterpret_cast<uintptr_t>(a.res) % 16 == 0);
  if (vec) {
    const dim3 grid(static_cast<unsigned>((SP / 4 + 255) / 256), a.B * a.Cout);
    a.clk = clock_slot(FSMI_K_CONV2D, s, 4ll * grid.x * grid.y, "split_reduce", true);
    hipLaunchKernelGGL(conv_split_reduce4_kernel, grid, dim3(256), 0, s, a);
  } else {
    const long long n = static_cast<long long>(a.B) * a.Cout * SP;
    a.clk = clock_slot(FSMI_K_CONV2D, s, 4ll * ((n + 255) / 256), "split_reduce", true);
    hipLaunchKernelGGL(conv_split_reduce_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, a);
  }
}

}  // namespace halo
}  // namespace fsmi

using namespace fsmi;

// debug phase stamps (fsmi_debug_conv_timestamps): halo convs here, the EdgeNeXt MLP kernel too
unsigned long long* g_conv_ts = nullptr;

namespace {

// launches per tile config as launched (0..9 and 11 register / LDS tiles, 10 stride-2, 16 + c K groups,
// 24..29 pointwise, 30 depth-blocked, 32 + c pipelined): fsmi_conv_launch_counts
std::atomic<long long> g_cfg_launches[64];

// in-kernel clock slot of a conv launch, tagged with its shape and tile (fsmi_timer_dump_captured)
unsigned long long* conv_clock(const HaloArgs& a, hipStream_t s, int cfg, int KS, int KD, long long nwaves) {
  char tag[112];
  snprintf(tag, sizeof(tag), "conv k%dx%d%s cfg%d ci%d co%d d%d h%d w%d ns%d%s", KD, KS, a.str == 2 ? " s2" : "", cfg,
           a.Cin, a.Cout, a.D, a.H, a.W, a.nsplit, a.up ? " up" : "");
  return clock_slot(FSMI_K_CONV2D, s, nwaves, tag, true);
}

// Shared host side of both entry points: validates, fills HaloArgs (gate fields preset by the
// caller), picks tiles and split-K, launches.
int run_halo(HaloArgs& a, const char* what, const float* const* seg_ptr, const int* seg_ch, const int* seg_ctot,
             int nseg, const void* whi, const void* wlo, const float* scale_bias, float* out, int out_ctot,
             int co0, int B, int Cout, int KS, int H, int W, int cfg, int nsplit, float* ws, long long ws_floats,
             void* stream, int D = 1, int KD = 1) {
  FSMI_CHECK_ARG(seg_ptr && seg_ch && seg_ctot && whi && wlo && scale_bias, "%s: null pointer", what);
  FSMI_CHECK_ARG(reinterpret_cast<uintptr_t>(scale_bias) % 8 == 0, "%s: scale_bias must be 8-B aligned", what);
  FSMI_CHECK_ARG(nseg >= 1 && nseg <= kHMaxSeg, "%s: 1..%d segments, got %d", what, kHMaxSeg, nseg);
  FSMI_CHECK_ARG(B > 0 && Cout > 0 && H > 0 && W > 0, "%s: bad shape", what);
  FSMI_CHECK_ARG(KS == 1 || KS == 3 || (KS == 2 && ((a.up == 2 && KD == 2) || (a.up == 4 && KD == 1 && D == 1))),
                 "%s: kernel %d unsupported (1, 3; 2 only for transposed-conv phases)", what, KS);
  if (a.str == 0) a.str = 1;
  FSMI_CHECK_ARG(a.str == 1 || (a.str == 2 && (KS == 3 || KS == 1) && (KD == 3 || KD == 1) && !a.up),
                 "%s: stride 2 needs a KD x KS x KS kernel with KS, KD in {1, 3}", what);
  FSMI_CHECK_ARG(D >= 1 && KD >= 1 && (KD % 2 == 1 || a.up), "%s: depth %d / depth kernel %d (odd)", what, D, KD);
  FSMI_CHECK_ARG(a.act == 3 || (out && co0 >= 0 && co0 + Cout <= out_ctot), "%s: output slice outside the tensor",
                 what);
  int cin = 0;
  const long long HW = static_cast<long long>(D) * H * W;     // channel stride
  const long long IHW = a.str == 2 ? a.icstride : HW;          // the input's (stride 2: D, H, W are the output's)
  a.D = D;
  a.KD = KD;
  a.PDD = KD / 2;
  a.cstride = HW;
  for (int i = 0; i < nseg; ++i) {
    FSMI_CHECK_ARG(seg_ptr[i] && seg_ch[i] > 0 && seg_ctot[i] >= seg_ch[i], "%s: bad segment %d", what, i);
    FSMI_CHECK_ARG(i == nseg - 1 || seg_ch[i] % 8 == 0,
                   "%s: inner segments must be multiples of 8 channels (segment %d: %d)", what, i, seg_ch[i]);
    a.seg_ptr[i] = seg_ptr[i];
    a.seg_bstride[i] = static_cast<long long>(seg_ctot[i]) * IHW;
    cin += seg_ch[i];
    a.seg_end[i] = cin;
  }
  a.nseg = nseg;
  a.Cin = cin;
  a.CinP = (cin + HKC - 1) / HKC * HKC;
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
  bool d3 = D > 1 || KD > 1;
  if (!d3 && range_safe()) {
    // safe range mode: the volume instantiation (range mode 1: per-chunk block exponent with exact
    // accumulator rescaling) with D = KD = 1 is the same 2D conv; the pointwise tiles (mode 2 only)
    // take the 128 x 2 x 32 register-weight tile
    d3 = true;
    if (cfg == 11 || cfg == 43) cfg = 9;           // the 5-row tile is 2D only
    else if (cfg >= 24 && cfg <= 29) cfg = 4;      // (pipelined 32 + c: the plain tile c, below)
  }
  if (cfg == 30) {                                 // depth-blocked (17, 1, 1) tile (conv_depth.hip)
    FSMI_CHECK_ARG(d3 && KS == 1 && KD == 17 && a.str == 1 && !a.up, "%s: tile 30 takes (17, 1, 1) stride-1 "
                   "volume convs", what);
    a.nsplit = 1;
    a.kpc = KD * a.CinP / HKC;
    a.ws = nullptr;
    a.ts = nullptr;
    a.ovf = range_flag_device();
    g_cfg_launches[30].fetch_add(1, std::memory_order_relaxed);
    const int rc = halo::launch_depth(a, s);
    if (rc != FSMI_OK) return rc;
    return finish_launch(what);
  }
  // cfg 32 + c: register-weight tile c (2..9) of a 2D map with the pipelined staging (conv_halo.h,
  // conv_halo_pipe_kernel); the volume instantiation (safe range mode) keeps the plain tile
  if (cfg >= 32) {
    cfg -= 32;
    FSMI_CHECK_ARG(((cfg >= 2 && cfg <= 9) || cfg == 11) && a.str == 1 && !a.up,
                   "%s: pipelined tile 32 + %d (2..9, 11; stride 1)", what, cfg);
    a.pipe = d3 ? 0 : 1;
  }
  const bool pw = cfg >= 24;
  if (pw) {                                        // pointwise LDS-DMA tiles (conv_pw.hip)
    FSMI_CHECK_ARG(cfg <= 29 && KS == 1 && !d3 && HW % 4 == 0, "%s: pointwise tile %d needs a 2D 1x1 conv with "
                   "H*W %% 4 == 0", what, cfg);
    for (int i = 0; i < nseg; ++i)
      FSMI_CHECK_ARG(reinterpret_cast<uintptr_t>(seg_ptr[i]) % 16 == 0, "%s: pointwise tile needs 16-B aligned "
                     "segments", what);
  }
  int kg = 1;
  if (cfg >= 16 && !pw) {
    kg = 2;
    cfg -= 16;
    FSMI_CHECK_ARG(halo::kg2_tile(cfg), "%s: tile %d has no K-group variant (16 + 3/4/5/7)", what, cfg);
  }
  FSMI_CHECK_ARG((cfg >= 0 && cfg <= 9) || pw || (a.str == 2 && cfg == 10) || (cfg == 11 && !d3 && KS != 2),
                 "%s: cfg %d (0..9, 11 on 2D maps, 16 + 3/4/5/7, 24..29)", what, cfg);
  FSMI_CHECK_ARG(a.str == 1 || (kg == 1 && (cfg == 4 || cfg == 5 || cfg == 7 || cfg == 10)),
                 "%s: stride-2 tile %d (4, 5, 7, 10)", what, cfg);
  if (pw) halo::pw_tile(cfg, a);
  else switch (cfg) {                             // tile = couts x (rows x 32 px)
    case 0: case 2: tile_counts<3, 64, 8, 1>(a); break;
    case 1: case 3: tile_counts<3, 128, 4, 2>(a); break;
    case 4: tile_counts<3, 128, 2, 2>(a); break;
    case 5: tile_counts<3, 64, 4, 1>(a); break;
    case 6: tile_counts<3, 32, 8, 1>(a); break;
    case 8: tile_counts<3, 128, 8, 2>(a); break;
    case 9: tile_counts<3, 256, 4, 4>(a); break;
    case 11: tile_counts<3, 256, 5, 4>(a); break;  // 5 rows: 24 row tiles at 120 (one round at 2 cout tiles)
    case 10: tile_counts<3, 64, 2, 2>(a); break;
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
  // in-block K groups (conv_halo.h, KG = 2; cfg 16 + c = tile c with K groups): the block's two
  // wave groups split its chunks and sum through LDS -- no partials in memory, no reduce pass.
  // FSMI_HALO_KG=2 (A/B) turns every eligible split-K >= 2 into K groups + half the splits.
  static const int kg_env = [] {
    const char* e = std::getenv("FSMI_HALO_KG");
    return e ? std::atoi(e) : -1;
  }();
  if (kg == 1 && kg_env == 2 && halo::kg2_tile(cfg) && nsplit >= 2) {   // A/B: fold a split of 2 into K groups
    kg = 2;
    nsplit = (nsplit + 1) / 2;
  }
  a.kpc = (nck + nsplit - 1) / nsplit;
  a.nsplit = (nck + a.kpc - 1) / a.kpc;                    // no empty splits
  FSMI_CHECK_ARG(a.nsplit == 1 || (ws && per_split * a.nsplit <= ws_floats),
                 "%s: split-K %d needs %lld workspace floats", what, a.nsplit, per_split * a.nsplit);
  a.ws = ws;
  a.ts = g_conv_ts;
  a.ovf = range_flag_device();
  static const int conv_dbg = [] {
    const char* e = std::getenv("FSMI_CONV_DBG");
    return e ? std::atoi(e) : 0;
  }();
  a.dbg = conv_dbg;
  g_cfg_launches[(a.pipe ? 32 : 0) + (kg == 2 ? 16 : 0) + cfg].fetch_add(1, std::memory_order_relaxed);
  a.clk = conv_clock(a, s, (a.pipe ? 32 : 0) + (kg == 2 ? 16 : 0) + cfg, KS, KD,
                     4ll * kg * a.npix * a.nco * a.nsplit * (a.up == 2 ? 8 : a.up == 4 ? 4 : 1));
  const int rc = a.str == 2 ? halo::launch_s2(KS, cfg, a, s) : pw ? halo::launch_pw(cfg, a, s) : KS == 2 ? (d3 ? halo::launch_cfg<2, true>(cfg, kg, a, s) : halo::launch_cfg<2, false>(cfg, kg, a, s)) : KS == 3 ? (d3 ? halo::launch_cfg<3, true>(cfg, kg, a, s) : halo::launch_cfg<3, false>(cfg, kg, a, s))
                         : (d3 ? halo::launch_cfg<1, true>(cfg, kg, a, s) : halo::launch_cfg<1, false>(cfg, kg, a, s));
  if (rc != FSMI_OK) return rc;
  if (a.nsplit > 1) halo::split_reduce(a, s);
  return finish_launch(what);
}

}  // namespace

// Debug: while buf is non-NULL every halo conv launch records, per block, thread 0's wall clock
// (100 MHz) at start [0], at each chunk's staging barrier [1..36], before / after the epilogue
// [37] / [38] and (chunks << 32 | block) [39] into buf[block * 40 ..] (tools/conv_phases.py).
extern "C" int fsmi_conv_launch_counts(long long* counts, int n, int reset) {
  FSMI_CHECK_ARG(counts && n > 0 && n <= 64, "fsmi_conv_launch_counts: 1..64 counters");
  for (int i = 0; i < n; ++i) counts[i] = g_cfg_launches[i].load(std::memory_order_relaxed);
  if (reset)
    for (auto& c : g_cfg_launches) c.store(0, std::memory_order_relaxed);
  return FSMI_OK;
}

extern "C" int fsmi_debug_conv_timestamps(unsigned long long* buf) {
  g_conv_ts = buf;
  return FSMI_OK;
}

extern "C" int fsmi_conv2d_halo_x3(const float* const* seg_ptr, const int* seg_ch, const int* seg_ctot, int nseg,
                                   const void* whi, const void* wlo, const float* scale_bias, const float* gamma,
                                   const float* res, int res_ctot, float* out, int out_ctot, int co0, int B, int Cout,
                                   int KS, int H, int W, int act, float alpha, int cfg, int nsplit, float* ws,
                                   long long ws_floats, void* stream) {
  FSMI_CHECK_ARG(out, "fsmi_conv2d_halo_x3: null output");
  FSMI_CHECK_ARG((act >= 0 && act <= 2) || act == 6 || act == 7, "fsmi_conv2d_halo_x3: act %d (0, 1, 2, 6, 7)", act);
  FSMI_CHECK_ARG(act != 7 || (res && !gamma && alpha == 1.f), "fsmi_conv2d_halo_x3: act 7 (ReLU(conv + bias + res)) "
                 "needs res, no gamma, alpha 1");
  HaloArgs a{};
  a.act = act;
  a.alpha = alpha;
  a.gamma = gamma;
  a.res = res;
  a.res_bstride = static_cast<long long>(res_ctot) * H * W;
  return run_halo(a, "fsmi_conv2d_halo_x3", seg_ptr, seg_ch, seg_ctot, nseg, whi, wlo, scale_bias, out, out_ctot,
                  co0, B, Cout, KS, H, W, cfg, nsplit, ws, ws_floats, stream);
}

extern "C" int fsmi_conv2d_halo_x3_gate(const float* const* seg_ptr, const int* seg_ch, const int* seg_ctot,
                                        int nseg, const void* whi, const void* wlo, const float* scale_bias,
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
  return run_halo(a, "fsmi_conv2d_halo_x3_gate", seg_ptr, seg_ch, seg_ctot, nseg, whi, wlo, scale_bias, out,
                  out_ctot, co0, B, Cout, KS, H, W, cfg, nsplit, ws, ws_floats, stream);
}

extern "C" int fsmi_conv3d_halo_x3_ex(const float* x, int Cin, const void* whi, const void* wlo,
                                      const float* scale_bias, const float* res, const float* fatt, float* out, int B,
                                      int Cout, int D, int H, int W, int KD, int KS, int stride, int act, int res_pre,
                                      int cfg, int nsplit, float* ws, long long ws_floats, void* stream) {
  FSMI_CHECK_ARG(x && out && Cin > 0, "fsmi_conv3d_halo_x3: null pointer / channels");
  FSMI_CHECK_ARG(act == 0 || act == 1 || act == 6, "fsmi_conv3d_halo_x3: act %d (0 none, 1 ReLU, 6 LeakyReLU)", act);
  FSMI_CHECK_ARG(stride == 1 || stride == 2, "fsmi_conv3d_halo_x3: stride %d (1, 2)", stride);
  FSMI_CHECK_ARG(B > 0 && D > 0 && H > 0 && W > 0, "fsmi_conv3d_halo_x3: bad shape");
  HaloArgs a{};
  a.act = act;
  a.alpha = 1.f;
  a.fatt = fatt;
  a.str = stride;
  // the 2D instantiation (D = KD = 1 at stride 1) has no res_pre path
  FSMI_CHECK_ARG(!res_pre || D > 1 || KD > 1 || stride == 2, "fsmi_conv3d_halo_x3: res_pre needs a volume (D or KD > 1)"
                 " or stride 2");
  if (stride == 2) {                               // k3 p1 / k1 p0, stride 2: output (n - 1) / 2 + 1 per dimension
    FSMI_CHECK_ARG((KS == 3 || KS == 1) && (KD == 3 || KD == 1), "fsmi_conv3d_halo_x3: stride 2 needs KS, KD in {1, 3}");
    a.iD = D;
    a.iH = H;
    a.iW = W;
    a.icstride = static_cast<long long>(D) * H * W;
    D = (D - 1) / 2 + 1;
    H = (H - 1) / 2 + 1;
    W = (W - 1) / 2 + 1;
    if (cfg < 0) cfg = Cout <= 64 ? 10 : 4;          // TR = 2 tiles: 52 KB of LDS, three blocks per CU
  }
  a.res = res;
  a.res_pre = res_pre;
  a.res_bstride = static_cast<long long>(Cout) * D * H * W;
  // (17, 1, 1) disparity-axis convs (Conv3dNormActReduced.conv2) on the depth-blocked tile unless a
  // tile is forced; FSMI_DEPTH_TILE=0 keeps the generic volume tiles (A/B)
  static const bool depth_tile = [] {
    const char* e = std::getenv("FSMI_DEPTH_TILE");
    return !e || std::atoi(e) != 0;
  }();
  if (stride == 1 && KS == 1 && KD == 17 && cfg < 0 && depth_tile) cfg = 30;
  const float* seg[1] = {x};
  const int ch[1] = {Cin}, tot[1] = {Cin};
  return run_halo(a, "fsmi_conv3d_halo_x3", seg, ch, tot, 1, whi, wlo, scale_bias, out, Cout, 0, B, Cout, KS, H, W,
                  cfg, nsplit, ws, ws_floats, stream, D, KD);
}

extern "C" int fsmi_conv3d_halo_x3(const float* x, int Cin, const void* whi, const void* wlo, const float* scale_bias,
                                   const float* res, float* out, int B, int Cout, int D, int H,
                                   int W, int KD, int KS, int act, int res_pre, int cfg, int nsplit, float* ws,
                                   long long ws_floats, void* stream) {
  return fsmi_conv3d_halo_x3_ex(x, Cin, whi, wlo, scale_bias, res, nullptr, out, B, Cout, D, H, W, KD, KS, 1, act,
                                res_pre, cfg, nsplit, ws, ws_floats, stream);
}

extern "C" int fsmi_conv3d_up2_halo_x3(const float* x, int Cin, const void* const* whi, const void* const* wlo,
                                       const float* const* scale_bias, float* out, int B, int Cout, int D, int H,
                                       int W, int act, int cfg, void* stream) {
  FSMI_CHECK_ARG(x && out && whi && wlo && scale_bias && Cin > 0, "fsmi_conv3d_up2_halo_x3: null pointer / channels");
  FSMI_CHECK_ARG(act == 0 || act == 1 || act == 6, "fsmi_conv3d_up2_halo_x3: act %d (0, 1, 6)", act);
  // tools/up3d_bench.py at cfg2 (one launch, 8 phases): 32-cout x 4-row tiles for 28 and 112 couts,
  // 64 x 8 for 56 (conv1_up 296 us, conv2_up 139 us, conv3_up 64 us vs 711 / 249 / 97 us for
  // MIOpen / CK + BatchNorm + LeakyReLU)
  if (cfg < 0) cfg = (Cout > 32 && Cout <= 64) ? 2 : 7;
  FSMI_CHECK_ARG(cfg == 2 || cfg == 3 || cfg == 5 || cfg == 6 || cfg == 7,
                 "fsmi_conv3d_up2_halo_x3: tile %d (2, 3, 5, 6, 7)", cfg);
  const long long V = static_cast<long long>(D) * H * W;
  HaloArgs a{};
  for (int p = 0; p < 8; ++p) {
    FSMI_CHECK_ARG(whi[p] && wlo[p] && scale_bias[p], "fsmi_conv3d_up2_halo_x3: null phase %d", p);
    FSMI_CHECK_ARG(reinterpret_cast<uintptr_t>(scale_bias[p]) % 8 == 0, "fsmi_conv3d_up2_halo_x3: scale_bias align");
    a.whi8[p] = static_cast<const _Float16*>(whi[p]);
    a.wlo8[p] = static_cast<const _Float16*>(wlo[p]);
    a.sb8[p] = reinterpret_cast<const float2*>(scale_bias[p]);
  }
  a.act = act;
  a.alpha = 1.f;
  a.up = 2;                                       // all eight phases in one launch
  a.ocstride = 8 * V;
  const float* seg[1] = {x};
  const int ch[1] = {Cin}, tot[1] = {Cin};
  // out_ctot = 8 * Cout: run_halo's batch stride (out_ctot x the input volume) is then the
  // (Cout, 2D, 2H, 2W) output's
  const int rc = run_halo(a, "fsmi_conv3d_up2_halo_x3", seg, ch, tot, 1, whi[0], wlo[0], scale_bias[0], out,
                          8 * Cout, 0, B, Cout, 2, H, W, cfg, 1, nullptr, 0, stream, D, 2);
  if (rc != FSMI_OK) return rc;
  return FSMI_OK;
}

extern "C" int fsmi_conv2d_up2_halo_x3(const float* x, int Cin, const void* const* whi, const void* const* wlo,
                                       const float* const* scale_bias, float* out, int B, int Cout, int H, int W,
                                       int act, int cfg, void* stream) {
  FSMI_CHECK_ARG(x && out && whi && wlo && scale_bias && Cin > 0, "fsmi_conv2d_up2_halo_x3: null pointer / channels");
  FSMI_CHECK_ARG(act == 0 || act == 1 || act == 6, "fsmi_conv2d_up2_halo_x3: act %d (0, 1, 6)", act);
  // ConvTranspose2d(k=4, s=2, p=1) as four 2x2 stride-1 phase convs over the input (the 2D analogue of
  // fsmi_conv3d_up2_halo_x3); 32-cout x 4-row tiles unless told otherwise (the spx layers: 32 and 9 couts)
  if (cfg < 0) cfg = Cout > 64 ? 3 : (Cout > 32 ? 5 : 7);
  FSMI_CHECK_ARG(cfg == 2 || cfg == 3 || cfg == 5 || cfg == 6 || cfg == 7,
                 "fsmi_conv2d_up2_halo_x3: tile %d (2, 3, 5, 6, 7)", cfg);
  HaloArgs a{};
  for (int p = 0; p < 4; ++p) {
    FSMI_CHECK_ARG(whi[p] && wlo[p] && scale_bias[p], "fsmi_conv2d_up2_halo_x3: null phase %d", p);
    FSMI_CHECK_ARG(reinterpret_cast<uintptr_t>(scale_bias[p]) % 8 == 0, "fsmi_conv2d_up2_halo_x3: scale_bias align");
    a.whi8[p] = static_cast<const _Float16*>(whi[p]);
    a.wlo8[p] = static_cast<const _Float16*>(wlo[p]);
    a.sb8[p] = reinterpret_cast<const float2*>(scale_bias[p]);
  }
  for (int p = 4; p < 8; ++p) {       // never selected (four phases); keep the array defined
    a.whi8[p] = a.whi8[0];
    a.wlo8[p] = a.wlo8[0];
    a.sb8[p] = a.sb8[0];
  }
  a.act = act;
  a.alpha = 1.f;
  a.up = 4;                                       // the four phases of a 2D map in one launch
  a.ocstride = 4ll * H * W;
  const float* seg[1] = {x};
  const int ch[1] = {Cin}, tot[1] = {Cin};
  // out_ctot = 4 * Cout: run_halo's batch stride (out_ctot x the input plane) is the (Cout, 2H, 2W) output's
  return run_halo(a, "fsmi_conv2d_up2_halo_x3", seg, ch, tot, 1, whi[0], wlo[0], scale_bias[0], out, 4 * Cout, 0, B,
                  Cout, 2, H, W, cfg, 1, nullptr, 0, stream, 1, 1);
}
