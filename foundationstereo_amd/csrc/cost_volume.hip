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
#include <cstdlib>

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

// a1 + a2 + corr_stem[0] (1x1x1 conv 32 -> Cs) in ONE streaming pass, no gwc scratch:
//   out[b,o,d,h,w] = A[b,o,h,w] + Bm[b,o,h,w-d] (w >= d) + sum_g Wg[o,g] gwc_g(d,w)
// (A / Bm = the proj_cmb halves of the concat volume folded through the stem weight, bias in A).
//
// Block = (b, h, WT = 4*WQ column tile, DCH = 4*DQN disparity chunk); thread = 4 d x 4 w, so a
// wave-instruction store covers 4 rows of 256 contiguous bytes.  Measured per-block timeline
// (tools/build_phases.py) drove the structure: every block runs at once (~1 wave per SIMD at
// cfg2), so each dependent global round trip costs ~3 us and the volume stores, all issued in one
// phase, run at the chip's write rate (~7 TB/s); the kernel is therefore
//   1. ONE staging round trip: the fl rows (WT columns), the fr rows (the WT + DCH columns the
//      chunk's shifts reach), the A / Bm rows and the stem columns go global -> LDS by LDS-DMA
//      (global_load_lds_dwordx4, no VGPR staging), one s_waitcnt + barrier per phase (one phase
//      when the image fits ~80 KB -- ViT-S -- else groups in NPH phases);
//      columns outside [0, W) are written as zeros, so w < d needs no masking anywhere;
//   2. per channel one float4 of L and two aligned float4 of R (the 7-wide shift window) feed
//      16 packed-FMA dot products; one thread per staged column sums its squared norm;
//   3. F.normalize (eps 1e-12, core/submodule.py:395) applied after the dots:
//      gwc = (L . R) * inv|L| * inv|R|, then the Cs-channel stem epilogue and 16-B stores.
// Blocks of one row are neighbours in the XCD remap (shared L2 for the overlapping R rows).
constexpr int kBuildG = 8;
typedef __attribute__((address_space(3))) void lds_void_t;
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

// 4 columns [col, col+4) of a row; zeros outside [0, W)
__device__ __forceinline__ float4 build_quad1(const float* p, int col, int W) {
  float4 v;
  v.x = (col + 0 >= 0 && col + 0 < W) ? p[0] : 0.f;
  v.y = (col + 1 >= 0 && col + 1 < W) ? p[1] : 0.f;
  v.z = (col + 2 >= 0 && col + 2 < W) ? p[2] : 0.f;
  v.w = (col + 3 >= 0 && col + 3 < W) ? p[3] : 0.f;
  return v;
}

// rows x cols (multiple of 4) columns from col0 of channel-strided rows -> lds[rows][cols], element
// e = (row, column quad) at lds + 4e.  VEC 4 (W % 4 == 0, quads wholly in or out of [0, W)):
// LDS-DMA, one 1-KiB wave-instruction per 64 consecutive elements (destination = wave-uniform
// base + 16 * lane), zero quads by ds_write; VEC 1: register path with per-element bounds.
template <int VEC>
__device__ __forceinline__ void build_stage_rows(const float* __restrict__ f, size_t plane, int rows, int cols,
                                                 int col0, int W, float* lds, int tid, int nthr) {
  const int nq = cols / 4, n = rows * nq;
  const int sc = nthr / nq, sq = nthr - sc * nq;
  int c = tid / nq, q = tid - c * nq;
  const int wbase = tid & ~(kWave - 1);
  for (int e0 = 0; e0 < n; e0 += nthr) {
    const int e = e0 + tid;
    if (e < n) {
      const int col = col0 + 4 * q;
      const float* src = f + static_cast<size_t>(c) * plane + col;
      if constexpr (VEC == 4) {
        if (col >= 0 && col < W)
          __builtin_amdgcn_global_load_lds(src, (lds_void_t*)(lds + 4 * (e0 + wbase)), 16, 0, 0);
        else
          *reinterpret_cast<float4*>(lds + 4 * e) = make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        *reinterpret_cast<float4*>(lds + 4 * e) = build_quad1(src, col, W);
      }
    }
    q += sq;
    c += sc;
    if (q >= nq) {
      q -= nq;
      ++c;
    }
  }
}

// LDS image (floats): [A: Cs x WT][Bm: Cs x RS][Wg: Cs x G][invn: G x (WT+RS)][groups: GP x Cg x (WT+RS)]
__host__ __device__ inline int build_lds_floats(int Cg, int Cs, int WT, int RS, int GP) {
  return Cs * (WT + RS) + Cs * kBuildG + kBuildG * (WT + RS) + GP * Cg * (WT + RS);
}

template <int VEC, int GP>
__global__ __launch_bounds__(kThreads) void build_stem_kernel(const float* __restrict__ fl,
                                                              const float* __restrict__ fr,
                                                              const float* __restrict__ A,
                                                              const float* __restrict__ Bm,
                                                              const float* __restrict__ Wg,
                                                              float* __restrict__ out, int C, int Cs, int D,
                                                              int H, int W, int WQ, int DQN, int nwt, int ndc, int dbg,
                                                              unsigned long long* clk) {
  constexpr int G = kBuildG, NPH = G / GP;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Cg = C / G;
  const int WT = 4 * WQ, DCH = 4 * DQN, RS = WT + DCH, NC = WT + RS;
  clock_begin(clk);
  const unsigned item = xcd_remap(blockIdx.x, gridDim.x);
  const int dc = item % ndc;
  const int rest = item / ndc;
  const int wt = rest % nwt;
  const int row = rest / nwt;
  const int b = row / H, h = row - b * H;
  const int w0 = wt * WT, d0 = dc * DCH;
  const int rs0 = w0 - d0 - DCH;                   // first staged R column (a multiple of 4)
  const int tid = threadIdx.x, nthr = blockDim.x;
  const bool active = tid < WQ * DQN;
  const int wq = tid % WQ, dq = tid / WQ;
  const size_t plane = static_cast<size_t>(H) * W;
  float* As = smem;
  float* Bs = As + Cs * WT;
  float* Ws = Bs + Cs * RS;
  float* invn = Ws + Cs * G;                       // [G][WT + RS] inverse column norms (L then R)
  float* grp = invn + G * NC;                      // [GP][Cg][WT] L rows, then [GP][Cg][RS] R rows
  float* Rg = grp + GP * Cg * WT;
  const float* flb = fl + static_cast<size_t>(b) * C * plane + static_cast<size_t>(h) * W;
  const float* frb = fr + static_cast<size_t>(b) * C * plane + static_cast<size_t>(h) * W;
  // R window of this thread: positions base-4 .. base+3 of a staged row, base = 4(wq-dq) + DCH;
  // output (i, j) (d = d0+4dq+i, w = w0+4wq+j) uses position base + j - i = window slot j - i + 4
  const int base = 4 * (wq - dq) + DCH;
  const int wl0 = w0 + 4 * wq, dl0 = d0 + 4 * dq;
  // dbg bit 2: per-block phase timestamps (wall clock, 100 MHz) of thread 0 into output channel 0
  unsigned long long* ts = reinterpret_cast<unsigned long long*>(out) + static_cast<size_t>(blockIdx.x) * 16;
  const bool tsr = (dbg & 4) && tid == 0;
  if (tsr) ts[0] = wall_clock64();

  // epilogue operands travel with the first phase
  build_stage_rows<VEC>(A + static_cast<size_t>(b) * Cs * plane + static_cast<size_t>(h) * W, plane, Cs, WT, w0, W,
                        As, tid, nthr);
  build_stage_rows<VEC>(Bm + static_cast<size_t>(b) * Cs * plane + static_cast<size_t>(h) * W, plane, Cs, RS, rs0, W,
                        Bs, tid, nthr);
  for (int i = tid; i < Cs * G; i += nthr) Ws[i] = Wg[i];

  float gwc[G][4][4];
  const size_t oplane = static_cast<size_t>(D) * plane;
  float* dst = out + static_cast<size_t>(b) * Cs * oplane + static_cast<size_t>(dl0) * plane +
               static_cast<size_t>(h) * W + wl0;
  const bool wok = wl0 < W && !(dbg & 2);          // dbg bit 1: skip the stores (compute timing)

  // dot products of the thread's 4 d x 4 w outputs for groups [g0, g0 + GP) (staged at slots
  // 0..GP-1).  Output (i, j) is l_j * r_k, k = j - i + 4 (R window slot).  v_pk_fma_f32 takes
  // each half of each source from ONE aligned register pair (op_sel picks the halves), so two
  // outputs share a packed FMA when their l's lie in one of (l0,l1) / (l2,l3) and their r's in
  // one of (r0,r1) .. (r6,r7): 6 such pairs, all with a broadcast r, cover 12 outputs and the 4
  // left over are plain FMAs -- 10 VALU per channel, no register shuffles, and both R float4
  // reads stay whole ds_read_b128s.  (Pairing along w made the compiler re-read R at odd
  // offsets with ds_read2_b32; pairing through a shifted (l1,l2) pair cost 6 moves a channel.)
  auto dots = [&](int g0) {
#pragma unroll
    for (int gl = 0; gl < GP; ++gl) {
      const float* L = grp + gl * Cg * WT + 4 * wq;
      const float* R = Rg + gl * Cg * RS + base;
      f2 q10 = 0.f, q20 = 0.f, q00 = 0.f, q12 = 0.f, q22 = 0.f, q02 = 0.f;
      float s01 = 0.f, s30 = 0.f, s03 = 0.f, s32 = 0.f;
      const int cend = (dbg & 1) ? 0 : Cg;       // dbg bit 0: skip the dot products (store-path timing)
      auto step = [&](const f4& l, const f4& ra, const f4& rb) {   // ra: slots 0..3, rb: 4..7
        const f2 l01 = l.xy, l23 = l.zw;
        q10 += l01 * ra.ww;                        // (1,0) (2,1)  r3
        q20 += l01 * ra.zz;                        // (2,0) (3,1)  r2
        q00 += l01 * rb.xx;                        // (0,0) (1,1)  r4
        q12 += l23 * rb.yy;                        // (1,2) (2,3)  r5
        q22 += l23 * rb.xx;                        // (2,2) (3,3)  r4
        q02 += l23 * rb.zz;                        // (0,2) (1,3)  r6
        // singles as opaque FMAs: left to itself the SLP vectoriser pairs them through moves
        asm("v_fmac_f32 %0, %1, %2" : "+v"(s01) : "v"(l.y), "v"(rb.y));   // (0,1) r5
        asm("v_fmac_f32 %0, %1, %2" : "+v"(s30) : "v"(l.x), "v"(ra.y));   // (3,0) r1
        asm("v_fmac_f32 %0, %1, %2" : "+v"(s03) : "v"(l.w), "v"(rb.w));   // (0,3) r7
        asm("v_fmac_f32 %0, %1, %2" : "+v"(s32) : "v"(l.z), "v"(ra.w));   // (3,2) r3
      };
      // channels 4 at a time, all 12 LDS reads issued before the FMAs (the asm FMAs block the
      // compiler's own unrolling); the channel order of every sum is unchanged
      int c = 0;
      for (; c + 4 <= cend; c += 4, L += 4 * WT, R += 4 * RS) {
        f4 l[4], ra[4], rb[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          l[u] = *reinterpret_cast<const f4*>(L + u * WT);
          ra[u] = *reinterpret_cast<const f4*>(R + u * RS - 4);
          rb[u] = *reinterpret_cast<const f4*>(R + u * RS);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) step(l[u], ra[u], rb[u]);
      }
      for (; c < cend; ++c, L += WT, R += RS)
        step(*reinterpret_cast<const f4*>(L), *reinterpret_cast<const f4*>(R - 4), *reinterpret_cast<const f4*>(R));
      float (&o)[4][4] = gwc[g0 + gl];
      o[1][0] = q10.x; o[2][1] = q10.y; o[2][0] = q20.x; o[3][1] = q20.y;
      o[0][0] = q00.x; o[1][1] = q00.y; o[1][2] = q12.x; o[2][3] = q12.y;
      o[2][2] = q22.x; o[3][3] = q22.y; o[0][2] = q02.x; o[1][3] = q02.y;
      o[0][1] = s01; o[3][0] = s30; o[0][3] = s03; o[3][2] = s32;
    }
  };
  // inverse column norms of groups [g0, g0 + GP): one thread per staged column (idle threads
  // first) sums all GP groups, so GP x 4 independent LDS reads are in flight per step
  auto norms = [&](int g0) {
    for (int col = nthr - 1 - tid; col < NC; col += nthr) {
      const float* src = col < WT ? grp + col : Rg + (col - WT);
      const int stride = col < WT ? WT : RS;
      float ss[GP][4];
#pragma unroll
      for (int gl = 0; gl < GP; ++gl)
#pragma unroll
        for (int u = 0; u < 4; ++u) ss[gl][u] = 0.f;
      int c = 0;
      for (; c + 4 <= Cg; c += 4) {
#pragma unroll
        for (int gl = 0; gl < GP; ++gl) {
          float v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = src[(gl * Cg + c + u) * stride];
#pragma unroll
          for (int u = 0; u < 4; ++u) ss[gl][u] += v[u] * v[u];
        }
      }
      for (; c < Cg; ++c)
#pragma unroll
        for (int gl = 0; gl < GP; ++gl) {
          const float v = src[(gl * Cg + c) * stride];
          ss[gl][0] += v * v;
        }
#pragma unroll
      for (int gl = 0; gl < GP; ++gl) {
        const float t = (ss[gl][0] + ss[gl][1]) + (ss[gl][2] + ss[gl][3]);
        invn[(g0 + gl) * NC + col] = t > 1e-24f ? __builtin_amdgcn_rsqf(t) : 1e12f;   // 1 / max(|x|, 1e-12)
      }
    }
  };

#pragma unroll
  for (int ph = 0; ph < NPH; ++ph) {
    if (ph > 0) __syncthreads();                   // previous phase's groups fully consumed
    build_stage_rows<VEC>(flb + static_cast<size_t>(ph) * GP * Cg * plane, plane, GP * Cg, WT, w0, W, grp, tid, nthr);
    build_stage_rows<VEC>(frb + static_cast<size_t>(ph) * GP * Cg * plane, plane, GP * Cg, RS, rs0, W, Rg, tid, nthr);
    __builtin_amdgcn_s_waitcnt(0);                 // this thread's LDS-DMA pieces have landed
    __syncthreads();
    if (tsr) ts[1 + 2 * ph] = wall_clock64();
    norms(ph * GP);
    if (active) dots(ph * GP);
    if (tsr) ts[2 + 2 * ph] = wall_clock64();
  }
  __syncthreads();                                 // invn complete
  if (tsr) ts[9] = wall_clock64();
  if (!active) return;
  // normalise: gwc *= inv|L|[w] * inv|R|[w - d]
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const f4 il = *reinterpret_cast<const f4*>(invn + g * NC + 4 * wq);
    const f4 ia = *reinterpret_cast<const f4*>(invn + g * NC + WT + base - 4);
    const f4 ib = *reinterpret_cast<const f4*>(invn + g * NC + WT + base);
    const float rv[8] = {ia.x, ia.y, ia.z, ia.w, ib.x, ib.y, ib.z, ib.w};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) gwc[g][i][j] = gwc[g][i][j] * il[j] * rv[j - i + 4];
  }
#pragma unroll 2
  for (int o = 0; o < Cs; ++o) {
    const f4 av = *reinterpret_cast<const f4*>(As + o * WT + 4 * wq);
    const f4 ba = *reinterpret_cast<const f4*>(Bs + o * RS + base - 4);
    const f4 bb = *reinterpret_cast<const f4*>(Bs + o * RS + base);
    const f4 g0 = *reinterpret_cast<const f4*>(Ws + o * G);
    const f4 g1 = *reinterpret_cast<const f4*>(Ws + o * G + 4);
    const float bv[8] = {ba.x, ba.y, ba.z, ba.w, bb.x, bb.y, bb.z, bb.w};
    const float wv[G] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    float* po = dst + static_cast<size_t>(o) * oplane;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float sacc = 0.f;
#pragma unroll
        for (int g = 0; g < G; ++g) sacc += wv[g] * gwc[g][i][j];
        v[j] = av[j] + bv[j - i + 4] + sacc;       // Bm staged as 0 left of column 0: the w < d zeros
      }
      if (dl0 + i < D && wok && !((dbg & 4) && o == 0)) {   // dbg 4: channel 0 holds the timestamps
        float* pp = po + static_cast<size_t>(i) * plane;
        if constexpr (VEC == 4) {
          *reinterpret_cast<float4*>(pp) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (wl0 + j < W) pp[j] = v[j];
        }
      }
    }
  }
  if (tsr) {
    ts[10] = wall_clock64();
    __builtin_amdgcn_s_waitcnt(0);
    ts[11] = wall_clock64();
  }
  clock_end(clk);
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


// Single-pass build tile: thread grid WQ column quads x DQN disparity quads (<= 256 threads, one
// block per CU -- the LDS image is ~130 KB at cfg2 -- so the default aims for at most one block
// per CU and few column tiles).  Groups are staged in the fewest phases whose LDS image fits the
// CU's 160 KB.  FSMI_BUILD_TILE = "WQ,DQN" overrides (A/B measurement); FSMI_BUILD_DBG: 1 no dot
// products, 2 no stores, 4 phase timestamps (tools/build_phases.py).
int launch_build_stem(const float* fl, const float* fr, const float* A, const float* Bm, const float* Wg, float* out,
                      int B, int C, int Cs, int D, int H, int W, hipStream_t s) {
  const int Cg = C / kBuildG;
  // disparity quads in balanced chunks of at most 16 (cfg2's D4 = 48: one chunk of 12; D4 = 80:
  // two of 10)
  const int dq_all = (D + 3) / 4, nchunk = (dq_all + 15) / 16;
  int DQN = (dq_all + nchunk - 1) / nchunk, WQ = 8;
  const char* env = std::getenv("FSMI_BUILD_TILE");
  int ew = 0, ed = 0;
  if (env && std::sscanf(env, "%d,%d", &ew, &ed) == 2 && ew > 0 && ed > 0 && ew * ed <= kThreads) {
    WQ = ew;
    DQN = ed;
  } else {
    // widest column tile (fewest column tiles, least R-row overlap) the 256-thread block allows,
    // then balanced over the row: cfg2 (W4 = 160, D4 = 48) -> 2 tiles of 20 quads, 240 blocks
    const int wq_max = std::max(1, kThreads / DQN), nq = (W + 3) / 4;
    const int ntile = (nq + wq_max - 1) / wq_max;
    WQ = (nq + ntile - 1) / ntile;
  }
  const int WT = 4 * WQ, DCH = 4 * DQN, RS = WT + DCH;
  const int nthr = (WQ * DQN + kWave - 1) / kWave * kWave;
  // LDS budget of the image.  One round of tiles (<= 256 blocks, e.g. cfg2's 240): the whole CU,
  // so the groups take the fewest phases.  More tiles than CUs: at most 80 KB, two blocks per CU, so
  // one block's stores (the write-dominated half of the kernel) overlap the other's staging and dot
  // products -- cfg3 (4 pairs, 960 tiles): 0.40 -> 0.47-0.48 of HBM peak, while cfg2 at 80 KB loses
  // 0.49 -> 0.45.  (A persistent variant -- one block per CU walking its tiles and prefetching the
  // next tile by LDS-DMA during the current stores -- gained only 0.395 -> 0.402 at cfg3; dropped.)
  // FSMI_BUILD_LDS_KB overrides the budget (A/B).
  const int nwt0 = (W + WT - 1) / WT, ndc0 = (D + DCH - 1) / DCH;
  static const int lds_env = [] {
    const char* e = std::getenv("FSMI_BUILD_LDS_KB");
    return e ? std::atoi(e) : 0;
  }();
  const size_t lds_cap = static_cast<size_t>(lds_env > 0 && lds_env <= 160 ? lds_env
                                              : (B * H * nwt0 * ndc0 > 256 ? 80 : 160)) * 1024;
  int GP = kBuildG;
  while (GP > 1 && static_cast<size_t>(build_lds_floats(Cg, Cs, WT, RS, GP)) * sizeof(float) > lds_cap) GP /= 2;
  const size_t lds = static_cast<size_t>(build_lds_floats(Cg, Cs, WT, RS, GP)) * sizeof(float);
  FSMI_CHECK_ARG(lds <= 160 * 1024, "fsmi_comb_volume_stem: LDS image %zu B too large (C=%d)", lds, C);
  const int nwt = (W + WT - 1) / WT, ndc = (D + DCH - 1) / DCH;
  const unsigned grid = static_cast<unsigned>(B) * H * nwt * ndc;
  const bool vec = (W % 4) == 0;
  const char* dbs = std::getenv("FSMI_BUILD_DBG");
  const int dbg = dbs ? std::atoi(dbs) : 0;
  LaunchTimer t(FSMI_K_COMB, s);
  unsigned long long* clk = clock_slot(FSMI_K_COMB, s, static_cast<long long>(grid) * (nthr / kWave));
#define FSMI_BUILD_CASE(V, P)                                                                                     \
  do {                                                                                                            \
    const void* fn = reinterpret_cast<const void*>(build_stem_kernel<V, P>);                                      \
    if (lds > 64 * 1024 &&                                                                                        \
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)) != hipSuccess) \
      return finish_launch("fsmi_comb_volume_stem: LDS attribute");                                               \
    set_replay(FSMI_K_COMB, s, [=] {                                                                              \
      hipLaunchKernelGGL((build_stem_kernel<V, P>), dim3(grid), dim3(nthr), lds, s, fl, fr, A, Bm, Wg, out, C, Cs,  \
                         D, H, W, WQ, DQN, nwt, ndc, dbg, nullptr);                                               \
    });                                                                                                           \
    hipLaunchKernelGGL((build_stem_kernel<V, P>), dim3(grid), dim3(nthr), lds, s, fl, fr, A, Bm, Wg, out, C, Cs, D, \
                       H, W, WQ, DQN, nwt, ndc, dbg, clk);                                                        \
  } while (0)
  if (vec) {
    if (GP == 8) FSMI_BUILD_CASE(4, 8);
    else if (GP == 4) FSMI_BUILD_CASE(4, 4);
    else if (GP == 2) FSMI_BUILD_CASE(4, 2);
    else FSMI_BUILD_CASE(4, 1);
  } else {
    if (GP == 8) FSMI_BUILD_CASE(1, 8);
    else if (GP == 4) FSMI_BUILD_CASE(1, 4);
    else if (GP == 2) FSMI_BUILD_CASE(1, 2);
    else FSMI_BUILD_CASE(1, 1);
  }
#undef FSMI_BUILD_CASE
  return finish_launch("fsmi_comb_volume_stem");
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
  return launch_build_stem(fl, fr, A, Bm, Wg, out, B, C, Cs, D, H, W, as_stream(stream));
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
