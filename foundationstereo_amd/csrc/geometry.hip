// Geometry encoding volume and its per-iteration lookup (SURVEY §8a rows a5,
// a6): all-pairs correlation on fp32 MFMA with the W2 avg-pool pyramid fused
// in the epilogue, the D pyramid of the filtered volume read in its native
// NCDHW layout (no permute copy), and the fused multi-level 9-tap lookup.
#include "fsmi_common.h"
#include "lookup_taps.h"

namespace fsmi {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------
// a5: corr[b,h,w1,w2] = <fl/|fl|, fr/|fr|> over all C   (core/geometry.py:68-77)
// One block = 4 waves = one (b, h, 32-wide w1 tile); each wave walks 32-wide
// w2 tiles.  v_mfma_f32_32x32x2_f32 (exact fp32, an fmaf chain over k):
//   A[i][k] = nL[k][w1_0+i]  lane l holds i=l&31, k=l>>5
//   B[k][j] = nR[k][w2_0+j]  lane l holds j=l&31, k=l>>5
// so each operand load is two coalesced 128-B segments of a feature row.
// Epilogue: D[i][j] in acc[r], i=(r&3)+8(r>>2)+4(l>>5), j=l&31; the pooled
// levels average lane pairs (xor 1, 2, 4) -- the same (a+b)/2 as avg_pool2d.
// ---------------------------------------------------------------------------
// Block = (b, h, w1 tile) with one wave per w2 tile (blockDim = 64*T).  The
// blocks of one row sit on one XCD (xcd_remap) so the R row is fetched from
// HBM once and re-read from that L2.  Prologue: column norms of the w1 tile
// and of the whole R row into LDS.  K loop: stage KC channels of the
// normalised L tile and R row in LDS (x / max(|x|, eps), the F.normalize
// division, once per element per block), then KC/2 MFMAs per wave with
// conflict-free LDS operand reads.
constexpr int kCorrKC = 16;
constexpr int kCorrMaxT = 16;  // W <= 512

__device__ __forceinline__ void corr_epilogue(const f32x16& acc, float* __restrict__ lv0, float* __restrict__ lv1,
                                              float* __restrict__ lv2, float* __restrict__ lv3, int L, int H, int W,
                                              int b, int h, int t1, int t2, int lane);

__global__ __launch_bounds__(kCorrMaxT * kWave) void allpairs_corr_kernel(
    const float* __restrict__ fl, const float* __restrict__ fr, float* __restrict__ lv0, float* __restrict__ lv1,
    float* __restrict__ lv2, float* __restrict__ lv3, int L, int C, int H, int W, int T) {
  __shared__ __attribute__((aligned(16))) float As[kCorrKC][32];
  __shared__ __attribute__((aligned(16))) float Bs[kCorrKC][kCorrMaxT * 32];
  __shared__ float nA[32];
  __shared__ float nB[kCorrMaxT * 32];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nthr = blockDim.x;
  const unsigned item = xcd_remap(blockIdx.x, gridDim.x);
  const int row = item / T, t1 = item - row * T;
  const int b = row / H, h = row - b * H;
  const size_t plane = static_cast<size_t>(H) * W;
  const float* L0 = fl + static_cast<size_t>(b) * C * plane + static_cast<size_t>(h) * W;
  const float* R0 = fr + static_cast<size_t>(b) * C * plane + static_cast<size_t>(h) * W;
  const int WT = T * 32;

  // column norms: ||f[:, w]||_2 clamped at 1e-12 (F.normalize, core/geometry.py:75)
  for (int j = threadIdx.x; j < 32 + WT; j += nthr) {
    const bool isA = j < 32;
    const int w = isA ? t1 * 32 + j : j - 32;
    const float* f = isA ? L0 : R0;
    float s = 0.f;
    if (w < W)
      for (int c = 0; c < C; ++c) {
        const float v = f[c * plane + w];
        s += v * v;
      }
    const float n = fmaxf(sqrtf(s), 1e-12f);
    if (isA) nA[j] = n; else nB[w] = n;
  }

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int i_l = lane & 31, k_l = lane >> 5;
  const int t2 = wave;
  for (int k0 = 0; k0 < C; k0 += kCorrKC) {
    __syncthreads();  // previous chunk consumed (and norms visible on the first pass)
    for (int e = threadIdx.x; e < kCorrKC * 32; e += nthr) {
      const int k = e >> 5, i = e & 31, c = k0 + k, w = t1 * 32 + i;
      As[k][i] = (c < C && w < W) ? L0[c * plane + w] / nA[i] : 0.f;
    }
    for (int e = threadIdx.x; e < kCorrKC * WT; e += nthr) {
      const int k = e / WT, w = e - k * WT, c = k0 + k;
      Bs[k][w] = (c < C && w < W) ? R0[c * plane + w] / nB[w] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < kCorrKC; kk += 2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[kk + k_l][i_l], Bs[kk + k_l][t2 * 32 + i_l], acc, 0, 0, 0);
  }
  corr_epilogue(acc, lv0, lv1, lv2, lv3, L, H, W, b, h, t1, t2, lane);
}

// Epilogue shared by both all-pairs variants: D[i][j] in acc[r] with
// i=(r&3)+8(r>>2)+4(l>>5) (w1), j=l&31 (w2); pooled levels by lane-pair shuffles.
__device__ __forceinline__ void corr_epilogue(const f32x16& acc, float* __restrict__ lv0, float* __restrict__ lv1,
                                              float* __restrict__ lv2, float* __restrict__ lv3, int L, int H, int W,
                                              int b, int h, int t1, int t2, int lane) {
  const int j = lane & 31;
  const size_t rowbase = static_cast<size_t>(b) * H + h;
  const int W1 = W >> 1, W2 = W >> 2, W3 = W >> 3;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    const int gw1 = t1 * 32 + i;
    const bool okr = gw1 < W;
    float v = acc[r];
    const int gw2 = t2 * 32 + j;
    if (okr && gw2 < W) lv0[(rowbase * W + gw1) * W + gw2] = v;
    if (L > 1) {
      v = (v + __shfl_xor(v, 1)) / 2.f;
      const int c1 = t2 * 16 + (j >> 1);
      if (okr && (j & 1) == 0 && c1 < W1) lv1[(rowbase * W + gw1) * W1 + c1] = v;
      if (L > 2) {
        v = (v + __shfl_xor(v, 2)) / 2.f;
        const int c2 = t2 * 8 + (j >> 2);
        if (okr && (j & 3) == 0 && c2 < W2) lv2[(rowbase * W + gw1) * W2 + c2] = v;
        if (L > 3) {
          v = (v + __shfl_xor(v, 4)) / 2.f;
          const int c3 = t2 * 4 + (j >> 3);
          if (okr && (j & 7) == 0 && c3 < W3) lv3[(rowbase * W + gw1) * W3 + c3] = v;
        }
      }
    }
  }
}

// F.normalize over channels (core/geometry.py:75) into a workspace, one thread
// per pixel: out[b,c,p] = f[b,c,p] / max(||f[b,:,p]||_2, 1e-12).  grid.y picks fl / fr.
__global__ __launch_bounds__(256) void normalize_cols_kernel(const float* __restrict__ f0,
                                                             const float* __restrict__ f1, float* __restrict__ o0,
                                                             float* __restrict__ o1, int C, int HW, long long P) {
  const long long p = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x;
  if (p >= P) return;
  const float* f = blockIdx.y ? f1 : f0;
  float* o = blockIdx.y ? o1 : o0;
  const long long b = p / HW;
  const size_t base = static_cast<size_t>(b) * C * HW + static_cast<size_t>(p - b * HW);
  float s = 0.f;
  int c = 0;
  for (; c + 8 <= C; c += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = f[base + static_cast<size_t>(c + u) * HW];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u] * v[u];
  }
  for (; c < C; ++c) {
    const float v = f[base + static_cast<size_t>(c) * HW];
    s += v * v;
  }
  const float n = fmaxf(sqrtf(s), 1e-12f);
  for (c = 0; c + 8 <= C; c += 8) {  // second pass (L2-hot), again 8 loads in flight per lane
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = f[base + static_cast<size_t>(c + u) * HW];
#pragma unroll
    for (int u = 0; u < 8; ++u) o[base + static_cast<size_t>(c + u) * HW] = v[u] / n;
  }
  for (; c < C; ++c) o[base + static_cast<size_t>(c) * HW] = f[base + static_cast<size_t>(c) * HW] / n;
}

// all-pairs on pre-normalised operands: no LDS, no barriers.  Block = (b, h,
// w1 tile), one wave per w2 tile; each wave streams its two 32-column slabs
// from L2 (row-major blocks of a row share one XCD) 16 k-steps of loads ahead
// of the MFMAs that consume them.
__global__ __launch_bounds__(kCorrMaxT * kWave) void allpairs_corr_direct_kernel(
    const float* __restrict__ nl, const float* __restrict__ nr, float* __restrict__ lv0, float* __restrict__ lv1,
    float* __restrict__ lv2, float* __restrict__ lv3, int L, int C, int H, int W, int T) {
  const int lane = threadIdx.x & 63, t2 = threadIdx.x >> 6;
  const unsigned item = xcd_remap(blockIdx.x, gridDim.x);
  const int row = item / T, t1 = item - row * T;
  const int b = row / H, h = row - b * H;
  const size_t plane = static_cast<size_t>(H) * W;
  const int i_l = lane & 31, k_l = lane >> 5;
  const int w1 = t1 * 32 + i_l, w2 = t2 * 32 + i_l;
  const bool ok1 = w1 < W, ok2 = w2 < W;
  const float* A0 = nl + static_cast<size_t>(b) * C * plane + static_cast<size_t>(h) * W + (ok1 ? w1 : 0);
  const float* B0 = nr + static_cast<size_t>(b) * C * plane + static_cast<size_t>(h) * W + (ok2 ? w2 : 0);
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  int k0 = 0;
  for (; k0 + 32 <= C; k0 += 32) {
    float av[16], bv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const size_t off = static_cast<size_t>(k0 + 2 * u + k_l) * plane;
      av[u] = ok1 ? A0[off] : 0.f;
      bv[u] = ok2 ? B0[off] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
  }
  for (; k0 < C; k0 += 2) {
    const int c = k0 + k_l;
    const float a = (ok1 && c < C) ? A0[static_cast<size_t>(c) * plane] : 0.f;
    const float bb = (ok2 && c < C) ? B0[static_cast<size_t>(c) * plane] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bb, acc, 0, 0, 0);
  }
  corr_epilogue(acc, lv0, lv1, lv2, lv3, L, H, W, b, h, t1, t2, lane);
}

// ---------------------------------------------------------------------------
// a5: D pyramid of the filtered volume, native (B,Cv,D,H,W) layout.  One
// thread owns S = 2^(L-1) consecutive level-0 disparities of one (b,c,h,w)
// column and emits its whole sub-tree; lanes over w keep every load/store
// coalesced.  Iterated (a+b)/2 == avg_pool2d([1,2]) applied level by level.
// ---------------------------------------------------------------------------
template <int S>
__global__ __launch_bounds__(256) void volume_pyramid_kernel(const float* __restrict__ vol, float* __restrict__ o1,
                                                             float* __restrict__ o2, float* __restrict__ o3, int D,
                                                             int HW, int nq, long long total) {
  const long long idx = blockIdx.x * 256ll + threadIdx.x;
  if (idx >= total) return;
  const int p = static_cast<int>(idx % HW);
  long long r = idx / HW;
  const int q = static_cast<int>(r % nq);
  const long long bc = r / nq;
  const int D1 = D >> 1, D2 = D >> 2, D3 = D >> 3;
  float v[S];
  const float* src = vol + bc * D * HW + p;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int x = q * S + s;
    v[s] = x < D ? src[static_cast<size_t>(x) * HW] : 0.f;
  }
  int len = S;
  float* outs[3] = {o1, o2, o3};
  const int lens[3] = {D1, D2, D3};
#pragma unroll
  for (int lvl = 0; lvl < 3; ++lvl) {
    if ((S >> (lvl + 1)) == 0) break;
    len >>= 1;
#pragma unroll
    for (int s = 0; s < (S >> (lvl + 1)); ++s) {
      v[s] = (v[2 * s] + v[2 * s + 1]) / 2.f;
      const int x = q * (S >> (lvl + 1)) + s;
      if (x < lens[lvl]) outs[lvl][(bc * lens[lvl] + x) * HW + p] = v[s];
    }
  }
  (void)len;
}

// ---------------------------------------------------------------------------
// a6: fused lookup.  grid = (ceil(P/64), L, nchunk/4); one wave = 64
// consecutive pixels x one chunk of kCPC = 4 geo channels (or the corr channel)
// of one level.  (7 per wave: 36.5 vs 37.4 us alone at cfg2 but 44.2 vs 42.0 us
// average inside the concurrent loop under rocprof; 2 per wave 37.9 us.)  Coordinates follow bilinear_sampler: x -> 2x/(n-1)-1 -> (x'+1)
// * ((n-1)/2) (the CPU grid_sampler's align_corners unnormalise), then linear
// interpolation with zero padding.  The 2r+4 window around floor(x) is loaded
// once per channel into registers; each tap selects its pair with
// compile-time indices (no scratch), so a channel costs 2r+4 loads, not 4r+2.
// ---------------------------------------------------------------------------
#ifndef FSMI_LOOKUP_CPC
#define FSMI_LOOKUP_CPC 4
#endif
constexpr int kCPC = FSMI_LOOKUP_CPC;  // geo channels per wave

struct LookupArgs {
  const float* vol[FSMI_MAX_LEVELS];
  const float* cor[FSMI_MAX_LEVELS];
  const float* disp;
  float* out;
  int L, Cv, D, H, W, W2, B;
  unsigned long long* clk;   // in-kernel launch clock (nullptr: off)
};

template <int R>
__global__ __launch_bounds__(256) void geo_lookup_kernel(LookupArgs a) {
  constexpr int K = 2 * R + 1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = blockIdx.y;  // level
  clock_begin(a.clk);
  const int chunk = blockIdx.z * 4 + wave;
  const int nchunk_geo = (a.Cv + kCPC - 1) / kCPC;
  if (chunk > nchunk_geo) return;
  const int HW = a.H * a.W;
  const long long p = static_cast<long long>(blockIdx.x) * 64 + lane;
  if (p >= static_cast<long long>(a.B) * HW) return;
  const int b = static_cast<int>(p / HW);
  const int hw = static_cast<int>(p - static_cast<long long>(b) * HW);
  const int w = hw % a.W;
  const float s = static_cast<float>(1 << i);
  const float ds = a.disp[p] / s;
  const int CH = a.L * K * (a.Cv + 1);
  const int base = i * K * (a.Cv + 1);
  float* outp = a.out + static_cast<size_t>(b) * CH * HW + hw;
  Taps<R> tp;
  if (chunk < nchunk_geo) {
    const int Di = a.D >> i;
    tp.init(ds, Di);
    const float* vol = a.vol[i] + static_cast<size_t>(b) * a.Cv * Di * HW + hw;
    const int c0 = chunk * kCPC;
    if (c0 + kCPC <= a.Cv) {
#pragma unroll
      for (int u = 0; u < kCPC; ++u)
        tp.sample(vol + static_cast<size_t>(c0 + u) * Di * HW, HW, Di,
                  outp + static_cast<size_t>(base + (c0 + u) * K) * HW, HW);
    } else {
      for (int c = c0; c < a.Cv; ++c)
        tp.sample(vol + static_cast<size_t>(c) * Di * HW, HW, Di, outp + static_cast<size_t>(base + c * K) * HW, HW);
    }
  } else {
    const int W2i = a.W2 >> i;
    const float* row = a.cor[i] + static_cast<size_t>(p) * W2i;
    tp.init(static_cast<float>(w) / s - ds, W2i);
    tp.sample(row, 1, W2i, outp + static_cast<size_t>(base + a.Cv * K) * HW, HW);
  }
  clock_end(a.clk);
}

// bilinear_sampler 1-D: img (P,C,1,Lx), x (P,K) -> out (P,C,1,K)
__global__ __launch_bounds__(256) void sampler_kernel(const float* __restrict__ img, const float* __restrict__ xs,
                                                      float* __restrict__ out, int C, int Lx, int K,
                                                      long long total) {
#pragma clang fp contract(off)
  const long long idx = blockIdx.x * 256ll + threadIdx.x;
  if (idx >= total) return;
  const int k = static_cast<int>(idx % K);
  const long long pc = idx / K;
  const long long pp = pc / C;
  const float ix = unnorm(xs[pp * K + k], Lx);
  const float fl = floorf(fminf(fmaxf(ix, -1.0e6f), 1.0e6f));
  const float f = ix - fl;
  const int i0 = static_cast<int>(fl);
  const float* row = img + pc * Lx;
  const float v0 = (i0 >= 0 && i0 < Lx) ? row[i0] : 0.f;
  const float v1 = (i0 + 1 >= 0 && i0 + 1 < Lx) ? row[i0 + 1] : 0.f;
  out[idx] = v0 * (1.f - f) + v1 * f;
}

}  // namespace
}  // namespace fsmi

using namespace fsmi;

extern "C" {

int fsmi_allpairs_corr(const float* fl, const float* fr, float* const* levels, int num_levels, int B, int C, int H,
                       int W, float* ws, void* stream) {
  FSMI_CHECK_ARG(fl && fr && levels, "fsmi_allpairs_corr: null pointer");
  FSMI_CHECK_ARG(num_levels >= 1 && num_levels <= FSMI_MAX_LEVELS, "fsmi_allpairs_corr: num_levels %d", num_levels);
  FSMI_CHECK_ARG(B > 0 && C > 0 && H > 0 && W > 0, "fsmi_allpairs_corr: bad shape");
  for (int i = 0; i < num_levels; ++i) FSMI_CHECK_ARG(levels[i], "fsmi_allpairs_corr: null level %d", i);
  const int T = (W + 31) / 32;
  FSMI_CHECK_ARG(T <= kCorrMaxT, "fsmi_allpairs_corr: W=%d exceeds %d", W, kCorrMaxT * 32);
  float* lv[4] = {levels[0], nullptr, nullptr, nullptr};
  for (int i = 1; i < num_levels; ++i) lv[i] = levels[i];
  for (int i = num_levels; i < 4; ++i) lv[i] = lv[0];
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_CORR, s);
  if (ws) {  // normalise once into the workspace, then the barrier-free MFMA pass
    const long long P = static_cast<long long>(B) * H * W;
    float* nl = ws;
    float* nr = ws + static_cast<size_t>(B) * C * H * W;
    hipLaunchKernelGGL(normalize_cols_kernel, dim3(ceil_div(P, 64), 2), dim3(64), 0, s, fl, fr, nl, nr, C, H * W, P);
    hipLaunchKernelGGL(allpairs_corr_direct_kernel, dim3(static_cast<unsigned>(B) * H * T), dim3(T * kWave), 0, s,
                       nl, nr, lv[0], lv[1], lv[2], lv[3], num_levels, C, H, W, T);
  } else {
    hipLaunchKernelGGL(allpairs_corr_kernel, dim3(static_cast<unsigned>(B) * H * T), dim3(T * kWave), 0, s,
                       fl, fr, lv[0], lv[1], lv[2], lv[3], num_levels, C, H, W, T);
  }
  return finish_launch("fsmi_allpairs_corr");
}

int fsmi_volume_pyramid(const float* vol, float* const* levels, int num_levels, int B, int Cv, int D, int H, int W,
                        void* stream) {
  FSMI_CHECK_ARG(vol && (num_levels <= 1 || levels), "fsmi_volume_pyramid: null pointer");
  FSMI_CHECK_ARG(num_levels >= 1 && num_levels <= FSMI_MAX_LEVELS, "fsmi_volume_pyramid: num_levels %d",
                 num_levels);
  FSMI_CHECK_ARG(B > 0 && Cv > 0 && D > 0 && H > 0 && W > 0, "fsmi_volume_pyramid: bad shape");
  if (num_levels == 1) return FSMI_OK;
  float* o[3] = {levels[0], num_levels > 2 ? levels[1] : levels[0], num_levels > 3 ? levels[2] : levels[0]};
  const int HW = H * W;
  const int S = 1 << (num_levels - 1);
  const int nq = (D + S - 1) / S;
  const long long total = static_cast<long long>(B) * Cv * nq * HW;
  const unsigned grid = ceil_div(total, 256);
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_VOLPYR, s);
  switch (S) {
    case 2: hipLaunchKernelGGL(volume_pyramid_kernel<2>, dim3(grid), dim3(256), 0, s, vol, o[0], o[1], o[2], D, HW, nq, total); break;
    case 4: hipLaunchKernelGGL(volume_pyramid_kernel<4>, dim3(grid), dim3(256), 0, s, vol, o[0], o[1], o[2], D, HW, nq, total); break;
    default: hipLaunchKernelGGL(volume_pyramid_kernel<8>, dim3(grid), dim3(256), 0, s, vol, o[0], o[1], o[2], D, HW, nq, total); break;
  }
  return finish_launch("fsmi_volume_pyramid");
}

int fsmi_geo_lookup(const float* const* vol_levels, const float* const* corr_levels, const float* disp, float* out,
                    int num_levels, int radius, int B, int Cv, int D, int H, int W, int W2, void* stream) {
  FSMI_CHECK_ARG(vol_levels && corr_levels && disp && out, "fsmi_geo_lookup: null pointer");
  FSMI_CHECK_ARG(num_levels >= 1 && num_levels <= FSMI_MAX_LEVELS, "fsmi_geo_lookup: num_levels %d", num_levels);
  FSMI_CHECK_ARG(radius == 4 || radius == 2 || radius == 3, "fsmi_geo_lookup: radius %d unsupported", radius);
  FSMI_CHECK_ARG(B > 0 && Cv > 0 && H > 0 && W > 0, "fsmi_geo_lookup: bad shape");
  FSMI_CHECK_ARG((D >> (num_levels - 1)) >= 2 && (W2 >> (num_levels - 1)) >= 2,
                 "fsmi_geo_lookup: level %d too short (D=%d, W2=%d): needs >= 2 samples", num_levels - 1, D, W2);
  LookupArgs a;
  for (int i = 0; i < FSMI_MAX_LEVELS; ++i) {
    a.vol[i] = i < num_levels ? vol_levels[i] : nullptr;
    a.cor[i] = i < num_levels ? corr_levels[i] : nullptr;
    if (i < num_levels) FSMI_CHECK_ARG(a.vol[i] && a.cor[i], "fsmi_geo_lookup: null level %d", i);
  }
  a.disp = disp;
  a.out = out;
  a.L = num_levels;
  a.Cv = Cv;
  a.D = D;
  a.H = H;
  a.W = W;
  a.W2 = W2;
  a.B = B;
  const long long P = static_cast<long long>(B) * H * W;
  const int nchunk = (Cv + kCPC - 1) / kCPC + 1;
  dim3 grid(ceil_div(P, 64), num_levels, (nchunk + 3) / 4);
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_LOOKUP, s);
  auto launch = [grid, radius, s](const LookupArgs& la) {
    switch (radius) {
      case 2: hipLaunchKernelGGL(geo_lookup_kernel<2>, grid, dim3(256), 0, s, la); break;
      case 3: hipLaunchKernelGGL(geo_lookup_kernel<3>, grid, dim3(256), 0, s, la); break;
      default: hipLaunchKernelGGL(geo_lookup_kernel<4>, grid, dim3(256), 0, s, la); break;
    }
  };
  a.clk = nullptr;
  set_replay(FSMI_K_LOOKUP, s, [launch, a] { launch(a); });
  a.clk = clock_slot(FSMI_K_LOOKUP, s, static_cast<long long>(grid.x) * grid.y * grid.z * 4);
  launch(a);
  return finish_launch("fsmi_geo_lookup");
}

int fsmi_bilinear_sampler_1d(const float* img, const float* x, float* out, int P, int C, int Lx, int K,
                             void* stream) {
  FSMI_CHECK_ARG(img && x && out, "fsmi_bilinear_sampler_1d: null pointer");
  FSMI_CHECK_ARG(P > 0 && C > 0 && K > 0 && Lx >= 2, "fsmi_bilinear_sampler_1d: bad shape (Lx must be >= 2)");
  const long long total = static_cast<long long>(P) * C * K;
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_SAMPLER, s);
  hipLaunchKernelGGL(sampler_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, s, img, x, out, C, Lx, K, total);
  return finish_launch("fsmi_bilinear_sampler_1d");
}

}  // extern "C"
