// Cost-volume construction: group-wise correlation,
// concat volume, and the fused comb-volume + corr_stem[0] build.
//
// Layout: features (B,C,H,W) fp32; volumes (B,Ch,D,H,W) fp32 -- the native
// NCDHW layout MIOpen's conv3d consumes, so nothing downstream re-packs.
//
// Roofline: HBM-bound (arithmetic intensity ~1 flop/B).  One block owns one
// (b,h) row and a chunk of DC disparities; the row's feature group is staged
// in LDS once and normalised there, every output lane writes consecutive w so
// stores are coalesced 256 B per wave-instruction.  Blocks of the same row
// are placed on one XCD (xcd_remap) so re-staging a row hits that XCD's L2.
#include "fsmi_common.h"

namespace fsmi {
namespace {

constexpr int kThreads = 256;

// Stage rows [g*Cg, (g+1)*Cg) of feature map `f` at (b,h) into lds[Cg][W],
// then L2-normalise every column over the Cg channels (F.normalize, eps 1e-12,
// core/submodule.py:395).
__device__ __forceinline__ void stage_group(const float* __restrict__ f, float* lds, int b, int h,
                                            int g, int Cg, int C, int H, int W) {
  const size_t plane = static_cast<size_t>(H) * W;
  const float* src = f + (static_cast<size_t>(b) * C + static_cast<size_t>(g) * Cg) * plane +
                     static_cast<size_t>(h) * W;
  if ((W & 3) == 0) {
    const int W4 = W >> 2;
    for (int i = threadIdx.x; i < Cg * W4; i += kThreads) {
      const int c = i / W4, q = i - c * W4;
      const float4 v = *reinterpret_cast<const float4*>(src + c * plane + 4 * q);
      *reinterpret_cast<float4*>(lds + c * W + 4 * q) = v;
    }
  } else {
    for (int i = threadIdx.x; i < Cg * W; i += kThreads) {
      const int c = i / W, w = i - c * W;
      lds[c * W + w] = src[c * plane + w];
    }
  }
  __syncthreads();
  for (int w = threadIdx.x; w < W; w += kThreads) {
    float s = 0.f;
    for (int c = 0; c < Cg; ++c) {
      const float v = lds[c * W + w];
      s += v * v;
    }
    const float n = fmaxf(sqrtf(s), 1e-12f);
    for (int c = 0; c < Cg; ++c) lds[c * W + w] = lds[c * W + w] / n;
  }
  __syncthreads();
}

template <int VEC>
__device__ __forceinline__ void load_vec(const float* p, float (&v)[VEC]) {
  if constexpr (VEC == 4) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else {
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[j] = p[j];
  }
}

template <int VEC>
__device__ __forceinline__ void store_vec(float* p, const float (&v)[VEC]) {
  if constexpr (VEC == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
#pragma unroll
    for (int j = 0; j < VEC; ++j) p[j] = v[j];
  }
}

__device__ __forceinline__ float group_dot(const float* L, const float* R, int Cg, int W, int w, int d) {
  float v = 0.f;
  for (int c = 0; c < Cg; ++c) v += L[c * W + w] * R[c * W + (w - d)];
  return v;
}

// a1: out (B,G,D,H,W)
template <int NOUT>
__global__ __launch_bounds__(kThreads) void gwc_kernel(const float* __restrict__ fl, const float* __restrict__ fr,
                                                       float* __restrict__ out, int C, int G, int D, int H,
                                                       int W, int DC, int nDC) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Cg = C / G;
  float* L = smem;
  float* R = smem + Cg * W;
  const unsigned item = xcd_remap(blockIdx.x, gridDim.x);
  const int row = item / nDC, dc = item - row * nDC;
  const int b = row / H, h = row - b * H;
  const int d0 = dc * DC, dn = min(DC, D - d0);
  const size_t plane = static_cast<size_t>(H) * W;
  for (int g = 0; g < G; ++g) {
    stage_group(fl, L, b, h, g, Cg, C, H, W);
    stage_group(fr, R, b, h, g, Cg, C, H, W);
#pragma unroll
    for (int k = 0; k < NOUT; ++k) {
      const int j = threadIdx.x + k * kThreads;
      if (j < dn * W) {
        const int dl = j / W, w = j - dl * W, d = d0 + dl;
        const float v = (w >= d) ? group_dot(L, R, Cg, W, w, d) : 0.f;
        out[((static_cast<size_t>(b) * G + g) * D + d) * plane + static_cast<size_t>(h) * W + w] = v;
      }
    }
    __syncthreads();
  }
}

// a1, vector path (D % 4 == 0, W % 4 == 0): block = one (b, h, g), the group's
// two rows staged + normalised ONCE, every thread owns a 4(d) x 4(w) output
// block: per channel one ds_read_b128 of L and a 7-wide window of R feed 16
// FMAs (vs 2 LDS reads per FMA), and the block writes 4 x 16-B per item.
__global__ __launch_bounds__(kThreads) void gwc_tile_kernel(const float* __restrict__ fl,
                                                            const float* __restrict__ fr, float* __restrict__ out,
                                                            int C, int G, int D, int H, int W) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Cg = C / G;
  float* L = smem;
  float* R = smem + Cg * W;
  const unsigned item = xcd_remap(blockIdx.x, gridDim.x);
  const int g = item % G;
  const int row = item / G;
  const int b = row / H, h = row - b * H;
  const size_t plane = static_cast<size_t>(H) * W;
  stage_group(fl, L, b, h, g, Cg, C, H, W);
  stage_group(fr, R, b, h, g, Cg, C, H, W);
  const int nwq = W >> 2, items = (D >> 2) * nwq;
  for (int it = threadIdx.x; it < items; it += kThreads) {
    const int dq = it / nwq, wq = it - dq * nwq;
    const int d0 = dq * 4, w0 = wq * 4;
    float acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
    // window index t = j - i + 3 in [0,7): R[w0 + j - d0 - i] = R[w0 - d0 - 3 + t]
    int ridx[7];
#pragma unroll
    for (int t = 0; t < 7; ++t) ridx[t] = max(w0 - d0 - 3 + t, 0);
    for (int c = 0; c < Cg; ++c) {
      const float4 l4 = *reinterpret_cast<const float4*>(L + c * W + w0);
      const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
      const float* Rc = R + c * W;
      float rv[7];
#pragma unroll
      for (int t = 0; t < 7; ++t) rv[t] = Rc[ridx[t]];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += lv[j] * rv[j - i + 3];
    }
    float* dst = out + ((static_cast<size_t>(b) * G + g) * D + d0) * plane + static_cast<size_t>(h) * W + w0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int d = d0 + i;
      float4 v;
      v.x = (w0 + 0 >= d) ? acc[i][0] : 0.f;
      v.y = (w0 + 1 >= d) ? acc[i][1] : 0.f;
      v.z = (w0 + 2 >= d) ? acc[i][2] : 0.f;
      v.w = (w0 + 3 >= d) ? acc[i][3] : 0.f;
      *reinterpret_cast<float4*>(dst + static_cast<size_t>(i) * plane) = v;
    }
  }
}

// corr_stem[0] applied to [gwc | concat] as a pure stream (the fused build's
// second half): thread = (b, d, h, VEC consecutive w); reads the G gwc values
// (coalesced), the L2-resident A/Bm rows, writes Cs channels as 16-B stores.
// out[b,o,d,h,w] = A[b,o,h,w] + [w>=d] Bm[b,o,h,w-d] + sum_g Wg[o,g] gwc[b,g,d,h,w]
template <int G, int VEC>
__global__ __launch_bounds__(kThreads) void stem_stream_kernel(const float* __restrict__ gwc,
                                                               const float* __restrict__ A,
                                                               const float* __restrict__ Bm,
                                                               const float* __restrict__ Wg, float* __restrict__ out,
                                                               int Cs, int D, int H, int W, long long total) {
  const long long t = blockIdx.x * static_cast<long long>(kThreads) + threadIdx.x;
  if (t >= total) return;
  const int nq = W / VEC;
  const int q = static_cast<int>(t % nq);
  long long r = t / nq;
  const int h = static_cast<int>(r % H);
  r /= H;
  const int d = static_cast<int>(r % D);
  const int b = static_cast<int>(r / D);
  const int w0 = q * VEC;
  const size_t plane = static_cast<size_t>(H) * W;
  const size_t hw = static_cast<size_t>(h) * W + w0;
  float gv[G][VEC];
#pragma unroll
  for (int g = 0; g < G; ++g) load_vec<VEC>(gwc + ((static_cast<size_t>(b) * G + g) * D + d) * plane + hw, gv[g]);
  bool ok[VEC];
  int bi[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    ok[j] = w0 + j >= d;
    bi[j] = max(w0 + j - d, 0);
  }
  const float* Ab = A + static_cast<size_t>(b) * Cs * plane + hw;
  const float* Bb = Bm + static_cast<size_t>(b) * Cs * plane + static_cast<size_t>(h) * W;
  float* dst = out + (static_cast<size_t>(b) * Cs * D + d) * plane + hw;
  for (int o = 0; o < Cs; ++o) {
    float v[VEC];
    load_vec<VEC>(Ab + o * plane, v);
    const float* Bo = Bb + o * plane;
    const float* wo = Wg + o * G;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float s = 0.f;
#pragma unroll
      for (int g = 0; g < G; ++g) s += wo[g] * gv[g][j];
      v[j] = v[j] + (ok[j] ? Bo[bi[j]] : 0.f) + s;
    }
    store_vec<VEC>(dst + static_cast<size_t>(o) * D * plane, v);
  }
}

// a1 + a2 + corr_stem[0] (1x1x1 conv 32 -> Cs):
// out[b,o,d,h,w] = A[o,w] + [w>=d] Bm[o,w-d] + sum_g Wg[o,g] gwc_g(d,w)
//
// Block = one (b,h) row x DC disparities.  Phase 1 walks the G groups: stage
// the normalised group rows of fl/fr in LDS, each thread computes the group
// correlation of VEC consecutive w for one d (one ds_read_b128 of L per
// channel) into an LDS gwc tile [G][DC][W].  Phase 2 re-uses the staging
// space for the A/Bm rows and emits all Cs output channels of VEC consecutive
// w per item as 16-B stores (one 1-KiB coalesced store per wave-instruction).
template <int G, int VEC>
__global__ __launch_bounds__(kThreads) void comb_stem_kernel(const float* __restrict__ fl,
                                                             const float* __restrict__ fr,
                                                             const float* __restrict__ A,
                                                             const float* __restrict__ Bm,
                                                             const float* __restrict__ Wg,
                                                             float* __restrict__ out, int C, int Cs, int D,
                                                             int H, int W, int DC, int nDC) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Cg = C / G;
  const unsigned item = xcd_remap(blockIdx.x, gridDim.x);
  const int row = item / nDC, dc = item - row * nDC;
  const int b = row / H, h = row - b * H;
  const int d0 = dc * DC, dn = min(DC, D - d0);
  const size_t plane = static_cast<size_t>(H) * W;
  const int region0 = max(2 * Cg * W, 2 * Cs * W);
  float* L = smem;
  float* R = smem + Cg * W;
  float* gw = smem + region0;            // [G][DC][W]
  float* Ws = gw + G * DC * W;           // [Cs][G]
  const int nq = W / VEC;
  const int items = dn * nq;

  // ---- phase 1: group correlations into LDS
  for (int g = 0; g < G; ++g) {
    stage_group(fl, L, b, h, g, Cg, C, H, W);
    stage_group(fr, R, b, h, g, Cg, C, H, W);
    for (int it = threadIdx.x; it < items; it += kThreads) {
      const int dl = it / nq, q = it - dl * nq;
      const int d = d0 + dl, w0 = q * VEC;
      float acc[VEC];
      int ri[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        acc[j] = 0.f;
        ri[j] = max(w0 + j - d, 0);  // clamped in-bounds; invalid lanes zeroed below
      }
      for (int c = 0; c < Cg; ++c) {
        float lv[VEC];
        load_vec<VEC>(L + c * W + w0, lv);
        const float* Rc = R + c * W;
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[j] += lv[j] * Rc[ri[j]];
      }
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] = (w0 + j >= d) ? acc[j] : 0.f;
      store_vec<VEC>(gw + (g * DC + dl) * W + w0, acc);
    }
    __syncthreads();
  }

  // ---- phase 2: stage A/Bm rows and the gwc columns of the stem weight, emit Cs channels
  float* As = smem;
  float* Bs = smem + Cs * W;
  const float* Ab = A + static_cast<size_t>(b) * Cs * plane + static_cast<size_t>(h) * W;
  const float* Bb = Bm + static_cast<size_t>(b) * Cs * plane + static_cast<size_t>(h) * W;
  for (int i = threadIdx.x; i < Cs * nq; i += kThreads) {
    const int o = i / nq, q = i - o * nq;
    float va[VEC], vb[VEC];
    load_vec<VEC>(Ab + o * plane + q * VEC, va);
    load_vec<VEC>(Bb + o * plane + q * VEC, vb);
    store_vec<VEC>(As + o * W + q * VEC, va);
    store_vec<VEC>(Bs + o * W + q * VEC, vb);
  }
  for (int i = threadIdx.x; i < Cs * G; i += kThreads) Ws[i] = Wg[i];
  __syncthreads();

  for (int it = threadIdx.x; it < items; it += kThreads) {
    const int dl = it / nq, q = it - dl * nq;
    const int d = d0 + dl, w0 = q * VEC;
    float gv[G][VEC];
#pragma unroll
    for (int g = 0; g < G; ++g) load_vec<VEC>(gw + (g * DC + dl) * W + w0, gv[g]);
    int bi[VEC];
    bool ok[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      ok[j] = w0 + j >= d;
      bi[j] = max(w0 + j - d, 0);
    }
    float* dst = out + (static_cast<size_t>(b) * Cs * D + d) * plane + static_cast<size_t>(h) * W + w0;
    for (int o = 0; o < Cs; ++o) {
      float v[VEC];
      load_vec<VEC>(As + o * W + w0, v);
      const float* Bo = Bs + o * W;
      const float* wo = Ws + o * G;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        float s = 0.f;
#pragma unroll
        for (int g = 0; g < G; ++g) s += wo[g] * gv[g][j];
        v[j] = v[j] + (ok[j] ? Bo[bi[j]] : 0.f) + s;
      }
      store_vec<VEC>(dst + static_cast<size_t>(o) * D * plane, v);
    }
  }
}

// a2: out (B,2C,D,H,W); one thread per output element, w fastest.
__global__ __launch_bounds__(kThreads) void concat_kernel(const float* __restrict__ pl, const float* __restrict__ pr,
                                                          float* __restrict__ out, int C, int D, int H, int W,
                                                          long long total) {
  const size_t plane = static_cast<size_t>(H) * W;
  for (long long i = blockIdx.x * static_cast<long long>(kThreads) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * kThreads) {
    const int w = static_cast<int>(i % W);
    long long r = i / W;
    const int h = static_cast<int>(r % H);
    r /= H;
    const int d = static_cast<int>(r % D);
    r /= D;
    const int c2 = static_cast<int>(r % (2 * C));
    const int b = static_cast<int>(r / (2 * C));
    float v;
    if (c2 < C) {
      v = pl[(static_cast<size_t>(b) * C + c2) * plane + static_cast<size_t>(h) * W + w];
    } else {
      v = (w >= d) ? pr[(static_cast<size_t>(b) * C + (c2 - C)) * plane + static_cast<size_t>(h) * W + (w - d)] : 0.f;
    }
    out[i] = v;
  }
}

// out[b,o,p] = bias[o] + sum_c Wt[o,c] x[b,c,p]; 8 outputs per thread.
constexpr int kProjO = 8;
__global__ __launch_bounds__(kThreads) void proj_kernel(const float* __restrict__ x, const float* __restrict__ Wt,
                                                        const float* __restrict__ bias, float* __restrict__ out,
                                                        int C, int O, int P) {
  extern __shared__ __attribute__((aligned(16))) float wsm[];  // [kProjO][C]
  const int o0 = blockIdx.y * kProjO;
  const int on = min(kProjO, O - o0);
  const int b = blockIdx.z;
  for (int i = threadIdx.x; i < on * C; i += kThreads) wsm[i] = Wt[static_cast<size_t>(o0) * C + i];
  __syncthreads();
  const int p = blockIdx.x * kThreads + threadIdx.x;
  if (p >= P) return;
  float acc[kProjO];
#pragma unroll
  for (int o = 0; o < kProjO; ++o) acc[o] = 0.f;
  const float* xb = x + static_cast<size_t>(b) * C * P + p;
  int c = 0;
  for (; c + 8 <= C; c += 8) {  // 8 independent loads in flight per lane before the FMAs
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = xb[static_cast<size_t>(c + u) * P];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int o = 0; o < kProjO; ++o) acc[o] += wsm[o * C + c + u] * v[u];
  }
  for (; c < C; ++c) {
    const float v = xb[static_cast<size_t>(c) * P];
#pragma unroll
    for (int o = 0; o < kProjO; ++o) acc[o] += wsm[o * C + c] * v;
  }
#pragma unroll
  for (int o = 0; o < kProjO; ++o)
    if (o < on) out[(static_cast<size_t>(b) * O + o0 + o) * P + p] = acc[o] + (bias ? bias[o0 + o] : 0.f);
}

constexpr int kNout = 8;

inline int pick_dc(int D, int W) { return max(1, min(D, kNout * kThreads / W)); }

// gwc volume into `out` (B,G,D,H,W): the 4x4-blocked tile kernel when D and W
// are multiples of 4, else the general per-output kernel.
int launch_gwc(const float* fl, const float* fr, float* out, int B, int C, int G, int D, int H, int W,
               hipStream_t s) {
  const int Cg = C / G;
  const size_t lds = static_cast<size_t>(2) * Cg * W * sizeof(float);
  FSMI_CHECK_ARG(lds <= 160 * 1024, "gwc volume: row too large for LDS (Cg=%d W=%d)", Cg, W);
  const bool tile = (D % 4 == 0) && (W % 4 == 0);
  const void* fn = tile ? reinterpret_cast<const void*>(gwc_tile_kernel)
                        : reinterpret_cast<const void*>(gwc_kernel<kNout>);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    if (e != hipSuccess) return finish_launch("gwc volume: LDS attribute");
  }
  if (tile) {
    hipLaunchKernelGGL(gwc_tile_kernel, dim3(static_cast<unsigned>(B) * H * G), dim3(kThreads), lds, s, fl, fr, out,
                       C, G, D, H, W);
  } else {
    const int DC = pick_dc(D, W);
    const int nDC = (D + DC - 1) / DC;
    hipLaunchKernelGGL(gwc_kernel<kNout>, dim3(static_cast<unsigned>(B) * H * nDC), dim3(kThreads), lds, s, fl, fr,
                       out, C, G, D, H, W, DC, nDC);
  }
  return finish_launch("gwc volume");
}

}  // namespace
}  // namespace fsmi

using namespace fsmi;

extern "C" {

int fsmi_gwc_volume(const float* fl, const float* fr, float* out, int B, int C, int G, int D, int H, int W,
                    void* stream) {
  FSMI_CHECK_ARG(fl && fr && out, "fsmi_gwc_volume: null pointer");
  FSMI_CHECK_ARG(B > 0 && C > 0 && G > 0 && D > 0 && H > 0 && W > 0, "fsmi_gwc_volume: bad shape");
  FSMI_CHECK_ARG(C % G == 0, "C:%d, num_groups:%d", C, G);
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_GWC, s);
  return launch_gwc(fl, fr, out, B, C, G, D, H, W, s);
}

int fsmi_concat_volume(const float* pl, const float* pr, float* out, int B, int C, int D, int H, int W,
                       void* stream) {
  FSMI_CHECK_ARG(pl && pr && out, "fsmi_concat_volume: null pointer");
  FSMI_CHECK_ARG(B > 0 && C > 0 && D > 0 && H > 0 && W > 0, "fsmi_concat_volume: bad shape");
  const long long total = static_cast<long long>(B) * 2 * C * D * H * W;
  const unsigned grid = static_cast<unsigned>(std::min<long long>((total + kThreads - 1) / kThreads, 8192));
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_CONCAT, s);
  hipLaunchKernelGGL(concat_kernel, dim3(grid), dim3(kThreads), 0, s, pl, pr, out, C, D, H, W, total);
  return finish_launch("fsmi_concat_volume");
}

int fsmi_comb_volume_stem(const float* fl, const float* fr, const float* A, const float* Bm, const float* Wg,
                          float* gwc_ws, float* out, int B, int C, int G, int Cs, int D, int H, int W, void* stream) {
  FSMI_CHECK_ARG(fl && fr && A && Bm && Wg && out, "fsmi_comb_volume_stem: null pointer");
  FSMI_CHECK_ARG(B > 0 && C > 0 && Cs > 0 && D > 0 && H > 0 && W > 0, "fsmi_comb_volume_stem: bad shape");
  FSMI_CHECK_ARG(G == 8, "fsmi_comb_volume_stem: num_groups must be 8 (cv_group), got %d", G);
  FSMI_CHECK_ARG(C % G == 0, "C:%d, num_groups:%d", C, G);
  if (gwc_ws) {  // two streaming passes: gwc tile kernel -> workspace, then the stem stream
    hipStream_t s = as_stream(stream);
    LaunchTimer t(FSMI_K_COMB, s);
    const int rc = launch_gwc(fl, fr, gwc_ws, B, C, G, D, H, W, s);
    if (rc) return rc;
    const bool vec = (W % 4) == 0;
    const long long total = static_cast<long long>(B) * D * H * (vec ? W / 4 : W);
    if (vec)
      hipLaunchKernelGGL((stem_stream_kernel<8, 4>), dim3(ceil_div(total, kThreads)), dim3(kThreads), 0, s, gwc_ws, A,
                         Bm, Wg, out, Cs, D, H, W, total);
    else
      hipLaunchKernelGGL((stem_stream_kernel<8, 1>), dim3(ceil_div(total, kThreads)), dim3(kThreads), 0, s, gwc_ws, A,
                         Bm, Wg, out, Cs, D, H, W, total);
    return finish_launch("fsmi_comb_volume_stem");
  }
  const int Cg = C / G;
  // largest disparity chunk (<= 8) whose LDS image fits: staging/A-Bm rows + gwc tile + stem columns
  auto lds_for = [&](int dc) {
    return (static_cast<size_t>(std::max(2 * Cg * W, 2 * Cs * W)) + static_cast<size_t>(G) * dc * W + Cs * G) *
           sizeof(float);
  };
  int DC = std::min(D, 8);
  while (DC > 1 && lds_for(DC) > 160 * 1024) DC >>= 1;
  const size_t lds = lds_for(DC);
  FSMI_CHECK_ARG(lds <= 160 * 1024, "fsmi_comb_volume_stem: row too large for LDS (W=%d)", W);
  const int nDC = (D + DC - 1) / DC;
  const unsigned grid = static_cast<unsigned>(B) * H * nDC;
  hipStream_t s = as_stream(stream);
  const bool vec = (W % 4) == 0;
  const void* fn = vec ? reinterpret_cast<const void*>(comb_stem_kernel<8, 4>)
                       : reinterpret_cast<const void*>(comb_stem_kernel<8, 1>);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    if (e != hipSuccess) return finish_launch("fsmi_comb_volume_stem: LDS attribute");
  }
  LaunchTimer t(FSMI_K_COMB, s);
  if (vec)
    hipLaunchKernelGGL((comb_stem_kernel<8, 4>), dim3(grid), dim3(kThreads), lds, s, fl, fr, A, Bm, Wg, out, C, Cs, D,
                       H, W, DC, nDC);
  else
    hipLaunchKernelGGL((comb_stem_kernel<8, 1>), dim3(grid), dim3(kThreads), lds, s, fl, fr, A, Bm, Wg, out, C, Cs, D,
                       H, W, DC, nDC);
  return finish_launch("fsmi_comb_volume_stem");
}

int fsmi_pointwise_proj(const float* x, const float* Wt, const float* bias, float* out, int B, int C, int O, int H,
                        int W, void* stream) {
  FSMI_CHECK_ARG(x && Wt && out, "fsmi_pointwise_proj: null pointer");
  FSMI_CHECK_ARG(B > 0 && C > 0 && O > 0 && H > 0 && W > 0, "fsmi_pointwise_proj: bad shape");
  const int P = H * W;
  dim3 grid(ceil_div(P, kThreads), ceil_div(O, kProjO), B);
  const size_t lds = static_cast<size_t>(kProjO) * C * sizeof(float);
  FSMI_CHECK_ARG(lds <= 64 * 1024, "fsmi_pointwise_proj: C=%d too large", C);
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_PROJ, s);
  hipLaunchKernelGGL(proj_kernel, grid, dim3(kThreads), lds, s, x, Wt, bias, out, C, O, P);
  return finish_launch("fsmi_pointwise_proj");
}

}  // extern "C"
