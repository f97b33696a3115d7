// Backbone kernels: DepthAnythingV2's DINOv2 ViT + DPT head
// (core/extractor.py:286-320, depth_anything/dpt.py:24-190, dinov2/dinov2/models/vision_transformer.py)
// and the glue of Feature (core/extractor.py:323-369).  The dense layers (qkv / proj / fc1 / fc2, the
// DPT convs) run on the halo split-precision conv engine as 1x1 / 3x3 convs; this file holds what is
// not a dense conv:
//   * token-major LayerNorm over channels in the channel-major token layout (B, C, T) that lets every
//     Linear run as a 1x1 conv (a token = a pixel);
//   * multi-head self-attention (head dim 64) as one flash-style kernel on split-precision MFMA;
//   * the patch embedding's space-to-depth and the non-overlapping transposed convs' depth-to-space;
//   * the token assembly (patch embeddings + cls token + interpolated position embedding);
//   * bicubic resize (the backbone's input, F.interpolate(mode="bicubic", align_corners=False));
//   * InstanceNorm2d (+ activation, + residual) and a small elementwise kernel.
#include "fsmi_common.h"

namespace fsmi {
namespace {

typedef _Float16 bhalf8 __attribute__((ext_vector_type(8)));
typedef _Float16 bhalf4 __attribute__((ext_vector_type(4)));
typedef float bf32x16 __attribute__((ext_vector_type(16)));
typedef float bf32x8 __attribute__((ext_vector_type(8)));
typedef float bf32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- LayerNorm over channels
// x (B, C, Tx), out (B, C, To); token t < n of each image: out[b, c, t] = (x - mean) * rstd * w[c] + b[c]
// with the biased variance over the C channels of token t (nn.LayerNorm over the last dim of the
// reference's token-major (B, T, C) tensors, dinov2 layers/block.py:63,75, vision_transformer.py:96;
// LayerNorm2d / channels-last LayerNorm in EdgeNeXt).  Block = 16 tokens x 16 channel groups: lanes
// over consecutive tokens read 64-B runs of each channel row.  Each thread loads its C / 16 channel
// values of its token ONCE into registers (all loads issued before the first use), so the mean, the
// centred variance and the normalised output are computed from registers: one HBM read and one write
// per element (round 6; the three-pass form re-read the column twice and waited one load latency per
// channel: 13.8 us per ViT-S LayerNorm at cfg2).
constexpr int LN_TB = 16, LN_G = 16, LN_MAXN = 64;          // C <= LN_G * LN_MAXN = 1024

__global__ __launch_bounds__(256) void chan_ln_kernel(const float* __restrict__ x, float* __restrict__ out,
                                                      const float* __restrict__ w, const float* __restrict__ bias,
                                                      int C, int Tx, int To, int n, float eps, int ntiles) {
  __shared__ float red[LN_G][LN_TB + 1];
  const int tid = threadIdx.x, tok = tid % LN_TB, grp = tid / LN_TB;
  const int b = blockIdx.x / ntiles;
  const int t = (blockIdx.x - b * ntiles) * LN_TB + tok;
  const bool valid = t < n;
  const float* xp = x + static_cast<size_t>(b) * C * Tx + min(t, n - 1);
  const int cnt = (C - grp + LN_G - 1) / LN_G;              // channels grp, grp + 16, ...
  float v[LN_MAXN];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < LN_MAXN; ++k) v[k] = k < cnt ? xp[static_cast<size_t>(grp + LN_G * k) * Tx] : 0.f;
#pragma unroll
  for (int k = 0; k < LN_MAXN; ++k) s += v[k];
  red[grp][tok] = s;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int g = 0; g < LN_G; ++g) tot += red[g][tok];
  const float mean = tot / static_cast<float>(C);
  __syncthreads();
  float s2 = 0.f;
#pragma unroll
  for (int k = 0; k < LN_MAXN; ++k) {
    const float d = k < cnt ? v[k] - mean : 0.f;
    s2 = fmaf(d, d, s2);
  }
  red[grp][tok] = s2;
  __syncthreads();
  float var = 0.f;
#pragma unroll
  for (int g = 0; g < LN_G; ++g) var += red[g][tok];
  const float rstd = 1.f / sqrtf(var / static_cast<float>(C) + eps);
  if (!valid) return;
  float* op = out + static_cast<size_t>(b) * C * To + t;
#pragma unroll
  for (int k = 0; k < LN_MAXN; ++k) {
    if (k < cnt) {
      const int c = grp + LN_G * k;
      op[static_cast<size_t>(c) * To] = fmaf((v[k] - mean) * rstd, w ? w[c] : 1.f, bias ? bias[c] : 0.f);
    }
  }
}

// ---------------------------------------------------------------- multi-head self-attention
// softmax(q k^T * scale) v per head (dinov2 layers/attention.py:69-79, non-causal SDPA), head dim 64,
// on the channel-major qkv of the qkv 1x1 conv: qkv (B, 3*nh*64, Tp) = [q heads; k heads; v heads],
// out (B, nh*64, Tp).  Keys t >= T (token padding) are masked; every one of the Tp query columns is
// computed (the padding columns stay finite for the convs that read them).
//
// A block = (image, head, NW*32 queries); wave w owns 32 queries.  Per 64-key block:
//   S^T (keys x queries) = K Q^T on v_mfma_f32_32x32x16_f16 with 3 products per MAC (fp16 hi/lo
//   splits, ~22-bit operands, fp32 accumulation): A = K staged in LDS as [key][d] hi / lo images,
//   B = the wave's Q fragments, split once and kept in registers (q pre-scaled by scale*log2(e), so
//   the scores are in log2 units and exp2 gives the softmax);
//   online softmax per query column -- the 32 keys of a fragment sit in one lane's registers, the
//   other 32 in lane ^ 32 (one cross-half shuffle per max / sum);
//   O^T (d x queries) += V P^T: P^T straight from the S^T accumulators (column = query on the lane,
//   rows = keys in registers: the B operand with no data movement, k order permuted as the
//   accumulator layout dictates), scaled by 2^12 before its hi / lo split so small probabilities keep
//   their low half normal; A = V from an LDS [d][key] image, read in the matching key order.
// The next key block's K / V are loaded into registers before the current block's MFMAs.
// Key split (round 6): B * heads * Tp / 32 query waves is below one wave per SIMD at ViT-S cfg2 (744
// waves for 1024 SIMDs, every wave alone on its SIMD with nothing to hide its latencies: 78 us per
// launch), so the key blocks are divided into nsplit ranges, one block per (image, head, 128
// queries, range); each writes its unnormalised O^T with its running max m and sum l, and
// vit_attn_combine_kernel merges the ranges (in range order) with the 2^(m_s - max m) weights.
constexpr int ATT_HD = 64, ATT_KB = 64, ATT_KR = ATT_HD + 8, ATT_VR = ATT_KB + 4;
constexpr float ATT_PSCALE = 4096.f;

__device__ __forceinline__ void mma3b(bf32x16& acc, const bhalf8& ah, const bhalf8& al, const bhalf8& bh,
                                      const bhalf8& bl) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
}

template <int NW>
__global__ __launch_bounds__(NW * 64) void vit_attn_kernel(const float* __restrict__ qkv, float* __restrict__ out,
                                                           int nh, int T, int Tp, float qscale, int nqt, int nsplit,
                                                           int kbs, float* __restrict__ opart,
                                                           float* __restrict__ mlpart) {
  constexpr int NT = NW * 64, KT = ATT_KB * ATT_HD / 8 / NT, VT = ATT_KB * ATT_HD / 4 / NT;
  static_assert(KT >= 1 && VT >= 1, "vit_attn: block too large");
  __shared__ __attribute__((aligned(16))) _Float16 kt[2][ATT_KB][ATT_KR];   // [hi, lo][key][d]
  __shared__ __attribute__((aligned(16))) _Float16 vs[2][ATT_HD][ATT_VR];   // [hi, lo][d][key]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hh = lane >> 5, r32 = lane & 31;
  const int sp = blockIdx.x % nsplit, qb = blockIdx.x / nsplit;
  const int qt = qb % nqt, bh = qb / nqt;
  const int h = bh % nh, b = bh / nh;
  const size_t P = static_cast<size_t>(Tp);
  const float* Q = qkv + (static_cast<size_t>(b) * 3 * nh * ATT_HD + static_cast<size_t>(h) * ATT_HD) * P;
  const float* K = Q + static_cast<size_t>(nh) * ATT_HD * P;
  const float* V = K + static_cast<size_t>(nh) * ATT_HD * P;
  const int q0 = qt * NW * 32 + wave * 32;
  const int qi = min(q0 + r32, Tp - 1);

  // Q fragments: k-step s covers d = 16 s + 8 hh + j
  bhalf8 qh[4], ql[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    bf32x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = Q[static_cast<size_t>(16 * s + 8 * hh + j) * P + qi] * qscale;
    qh[s] = __builtin_convertvector(v, bhalf8);
    ql[s] = __builtin_convertvector(v - __builtin_convertvector(qh[s], bf32x8), bhalf8);
  }

  float kreg[KT][8];
  bf32x4 vreg[VT];
  auto gload = [&](int j0) {
#pragma unroll
    for (int u = 0; u < KT; ++u) {
      const int task = u * NT + tid, key = task & (ATT_KB - 1), dg = task / ATT_KB;
#pragma unroll
      for (int t = 0; t < 8; ++t) kreg[u][t] = K[static_cast<size_t>(8 * dg + t) * P + j0 + key];
    }
#pragma unroll
    for (int u = 0; u < VT; ++u) {
      const int task = u * NT + tid, quad = task & (ATT_KB / 4 - 1), d = task / (ATT_KB / 4);
      vreg[u] = *reinterpret_cast<const bf32x4*>(V + static_cast<size_t>(d) * P + j0 + 4 * quad);
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int u = 0; u < KT; ++u) {
      const int task = u * NT + tid, key = task & (ATT_KB - 1), dg = task / ATT_KB;
      bf32x8 v;
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = kreg[u][t];
      const bhalf8 hi = __builtin_convertvector(v, bhalf8);
      *reinterpret_cast<bhalf8*>(&kt[0][key][8 * dg]) = hi;
      *reinterpret_cast<bhalf8*>(&kt[1][key][8 * dg]) = __builtin_convertvector(v - __builtin_convertvector(hi, bf32x8), bhalf8);
    }
#pragma unroll
    for (int u = 0; u < VT; ++u) {
      const int task = u * NT + tid, quad = task & (ATT_KB / 4 - 1), d = task / (ATT_KB / 4);
      const bhalf4 hi = __builtin_convertvector(vreg[u], bhalf4);
      *reinterpret_cast<bhalf4*>(&vs[0][d][4 * quad]) = hi;
      *reinterpret_cast<bhalf4*>(&vs[1][d][4 * quad]) =
          __builtin_convertvector(vreg[u] - __builtin_convertvector(hi, bf32x4), bhalf4);
    }
  };

  float m = -INFINITY, l = 0.f;
  bf32x16 o[2];
#pragma unroll
  for (int r = 0; r < 16; ++r) o[0][r] = o[1][r] = 0.f;
  const int kb_begin = sp * kbs, nkb = min((T + ATT_KB - 1) / ATT_KB, kb_begin + kbs);
  gload(kb_begin * ATT_KB);
  for (int kb = kb_begin; kb < nkb; ++kb) {
    __syncthreads();                 // every wave is done reading the previous block's images
    lstore();
    __syncthreads();
    if (kb + 1 < nkb) gload((kb + 1) * ATT_KB);
    bf32x16 sc[2];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[f][r] = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bhalf8 ah = *reinterpret_cast<const bhalf8*>(&kt[0][f * 32 + r32][16 * s + 8 * hh]);
        const bhalf8 al = *reinterpret_cast<const bhalf8*>(&kt[1][f * 32 + r32][16 * s + 8 * hh]);
        mma3b(sc[f], ah, al, qh[s], ql[s]);
      }
    }
    const int j0 = kb * ATT_KB;
    if (j0 + ATT_KB > T) {           // the last block: keys past T do not exist
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (j0 + f * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh >= T) sc[f][r] = -INFINITY;
    }
    float mx = -INFINITY;
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc[f][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float mnew = fmaxf(m, mx);
    const float alpha = __builtin_amdgcn_exp2f(m - mnew);
    float ps = 0.f;
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(sc[f][r] - mnew);
        sc[f][r] = p;
        ps += p;
      }
    ps += __shfl_xor(ps, 32);
    l = fmaf(l, alpha, ps);
    m = mnew;
    o[0] *= alpha;
    o[1] *= alpha;
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        bf32x8 pv;
#pragma unroll
        for (int j = 0; j < 8; ++j) pv[j] = sc[f][8 * ss + j] * ATT_PSCALE;
        const bhalf8 ph = __builtin_convertvector(pv, bhalf8);
        const bhalf8 pl = __builtin_convertvector(pv - __builtin_convertvector(ph, bf32x8), bhalf8);
        const int ks = 2 * f + ss;
#pragma unroll
        for (int df = 0; df < 2; ++df) {
          const int d = df * 32 + r32;
          const bhalf4 h0 = *reinterpret_cast<const bhalf4*>(&vs[0][d][16 * ks + 4 * hh]);
          const bhalf4 h1 = *reinterpret_cast<const bhalf4*>(&vs[0][d][16 * ks + 8 + 4 * hh]);
          const bhalf4 l0 = *reinterpret_cast<const bhalf4*>(&vs[1][d][16 * ks + 4 * hh]);
          const bhalf4 l1 = *reinterpret_cast<const bhalf4*>(&vs[1][d][16 * ks + 8 + 4 * hh]);
          const bhalf8 vh = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
          const bhalf8 vl = {l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
          mma3b(o[df], vh, vl, ph, pl);
        }
      }
  }
  const int qo = q0 + r32;
  if (qo >= Tp) return;
  if (nsplit > 1) {                // this key range's partial: O^T unnormalised, m, l
    const int nbh = gridDim.x / (nsplit * nqt);                                     // B * nh
    const size_t slot = static_cast<size_t>(sp) * nbh + bh;
    float* op = opart + slot * ATT_HD * P + qo;
#pragma unroll
    for (int df = 0; df < 2; ++df)
#pragma unroll
      for (int r = 0; r < 16; ++r) op[static_cast<size_t>(df * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh) * P] = o[df][r];
    if (hh == 0) {
      mlpart[slot * 2 * P + qo] = m;
      mlpart[slot * 2 * P + P + qo] = l;
    }
    return;
  }
  const float inv = 1.f / (l * ATT_PSCALE);
  float* op = out + (static_cast<size_t>(b) * nh + h) * ATT_HD * P + qo;
#pragma unroll
  for (int df = 0; df < 2; ++df)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      op[static_cast<size_t>(df * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh) * P] = o[df][r] * inv;
}

// out[bh, d, q] = sum_s 2^(m_s - M) O_s[d, q] / (sum_s 2^(m_s - M) l_s * PSCALE), M = max_s m_s; one
// thread per (bh, 8 channels, query)
__global__ __launch_bounds__(256) void vit_attn_combine_kernel(const float* __restrict__ opart,
                                                               const float* __restrict__ mlpart,
                                                               float* __restrict__ out, int nbh, int Tp, int nsplit) {
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  const int q = static_cast<int>(i % Tp);
  const long long r = i / Tp;
  const int dg = static_cast<int>(r % (ATT_HD / 8));
  const int bh = static_cast<int>(r / (ATT_HD / 8));
  if (bh >= nbh) return;
  const size_t P = static_cast<size_t>(Tp);
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, mlpart[(static_cast<size_t>(s) * nbh + bh) * 2 * P + q]);
  float L = 0.f, acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const size_t slot = static_cast<size_t>(s) * nbh + bh;
    const float w = __builtin_amdgcn_exp2f(mlpart[slot * 2 * P + q] - M);
    L = fmaf(mlpart[slot * 2 * P + P + q], w, L);
    const float* op = opart + (slot * ATT_HD + 8 * dg) * P + q;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = fmaf(op[j * P], w, acc[j]);
  }
  const float inv = 1.f / (L * ATT_PSCALE);
  float* o = out + (static_cast<size_t>(bh) * ATT_HD + 8 * dg) * P + q;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j * P] = acc[j] * inv;
}

// key ranges per (image, head, 128-query tile): enough blocks for two per CU, >= 4 key blocks each
int vit_attn_splits(int B, int heads, int T, int Tp, int* kbs) {
  const int nkb = (T + ATT_KB - 1) / ATT_KB;
  const long long nb = static_cast<long long>(B) * heads * ((Tp + 127) / 128);
  int ns = static_cast<int>(std::min<long long>(8, (512 + nb - 1) / nb));
  ns = std::max(1, std::min(ns, nkb / 4));
  const int per = (nkb + ns - 1) / ns;
  *kbs = per;
  return (nkb + per - 1) / per;
}

// ---------------------------------------------------------------- layout kernels
// space-to-depth (the im2col of a conv whose stride equals its kernel: DINOv2's patch embedding
// Conv2d(3, D, 14, stride 14), EdgeNeXt's stem Conv2d(3, 48, 4, 4) and downsampling Conv2d(k2, s2)):
// out[b, (c*k + ky)*k + kx, y, x] = in[b, c, y*k + ky, x*k + kx] -- the channel order of
// weight.reshape(Cout, -1), so the conv becomes a 1x1 conv over the k*k*C channels.
__global__ __launch_bounds__(256) void s2d_kernel(const float* __restrict__ x, float* __restrict__ out, int C, int H,
                                                  int W, int k, long long n) {
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const int Ho = H / k, Wo = W / k;
  const int xo = static_cast<int>(i % Wo);
  long long r = i / Wo;
  const int yo = static_cast<int>(r % Ho);
  r /= Ho;
  const int ch = static_cast<int>(r % (static_cast<long long>(C) * k * k));
  const long long b = r / (static_cast<long long>(C) * k * k);
  const int kx = ch % k, ky = (ch / k) % k, c = ch / (k * k);
  out[i] = x[((b * C + c) * H + (yo * k + ky)) * W + xo * k + kx];
}

// depth-to-space (a transposed conv whose stride equals its kernel, DPT's resize_layers[0] / [1]:
// ConvTranspose2d(k4, s4) / (k2, s2), depth_anything/dpt.py:41-53, run as a 1x1 conv with k*k*C
// outputs ordered (ky*k + kx)*C + c): out[b, c, y*k + ky, x*k + kx] = in[b, (ky*k + kx)*C + c, y, x]
__global__ __launch_bounds__(256) void d2s_kernel(const float* __restrict__ x, float* __restrict__ out, int C, int H,
                                                  int W, int k, long long n) {
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const int Wo = W * k, Ho = H * k;
  const int X = static_cast<int>(i % Wo);
  long long r = i / Wo;
  const int Y = static_cast<int>(r % Ho);
  r /= Ho;
  const int c = static_cast<int>(r % C);
  const long long b = r / C;
  const int ky = Y % k, kx = X % k;
  out[i] = x[((b * k * k * C + (ky * k + kx) * C + c) * H + Y / k) * W + X / k];
}

// token assembly (vision_transformer.py:214-233 with the class token stored AFTER the N patch tokens
// -- attention, LayerNorm and the Linears are permutation-equivariant over tokens, and the patch
// tokens then form a contiguous NCHW-able run): out (B, C, Tp), pos (C, Tp) the interpolated position
// embedding in the same token order (zero past N + 1).
__global__ __launch_bounds__(256) void vit_tokens_kernel(const float* __restrict__ emb, const float* __restrict__ cls,
                                                         const float* __restrict__ pos, float* __restrict__ out,
                                                         int C, int N, int Tp, long long n) {
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const int t = static_cast<int>(i % Tp);
  const long long bc = i / Tp;
  const int c = static_cast<int>(bc % C);
  const float v = t < N ? emb[bc * N + t] : (t == N ? cls[c] : 0.f);
  out[i] = v + (t <= N ? pos[static_cast<size_t>(c) * Tp + t] : 0.f);
}

// F.interpolate(mode="bicubic", align_corners=False) (core/extractor.py:352): cubic convolution with
// A = -0.75, source x = (dst + 0.5) * in/out - 0.5 (not clamped), taps clamped to the border
__device__ __forceinline__ void cubic_w(float t, float (&w)[4]) {
  constexpr float A = -0.75f;
  const float x1 = t + 1.f, x2 = 1.f - t, x3 = 2.f - t;
  w[0] = ((A * x1 - 5.f * A) * x1 + 8.f * A) * x1 - 4.f * A;
  w[1] = ((A + 2.f) * t - (A + 3.f)) * t * t + 1.f;
  w[2] = ((A + 2.f) * x2 - (A + 3.f)) * x2 * x2 + 1.f;
  w[3] = ((A * x3 - 5.f * A) * x3 + 8.f * A) * x3 - 4.f * A;
}

__global__ __launch_bounds__(256) void bicubic_kernel(const float* __restrict__ x, float* __restrict__ out, int Hi,
                                                      int Wi, int Ho, int Wo, float sh, float sw, long long n) {
#pragma clang fp contract(off)
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const int ox = static_cast<int>(i % Wo);
  const int oy = static_cast<int>((i / Wo) % Ho);
  const long long p = i / (static_cast<long long>(Ho) * Wo);
  // one rounding (fma), as the reference's vectorised CPU kernel computes it: at source coordinates of
  // a few hundred pixels one fp32 ulp of the coordinate moves the taps' weights by ~3e-5
  const float fy = fmaf(sh, oy + 0.5f, -0.5f), fx = fmaf(sw, ox + 0.5f, -0.5f);
  const int iy = static_cast<int>(floorf(fy)), ix = static_cast<int>(floorf(fx));
  float wy[4], wx[4];
  cubic_w(fy - iy, wy);
  cubic_w(fx - ix, wx);
  const float* xp = x + p * Hi * Wi;
  float acc = 0.f;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int yy = min(max(iy - 1 + a, 0), Hi - 1);
    float row = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int xx = min(max(ix - 1 + c, 0), Wi - 1);
      row += xp[static_cast<size_t>(yy) * Wi + xx] * wx[c];
    }
    acc += row * wy[a];
  }
  out[i] = acc;
}

// ---------------------------------------------------------------- InstanceNorm2d (+ act, + residual)
// out = act2(act1((x - mean) * rstd) + res) per (b, c) plane, biased variance, no affine
// (nn.InstanceNorm2d defaults; BasicConv_IN / Conv2x_IN / ResnetBasicBlock / ResidualBlock with
// norm 'instance', core/submodule.py:320-385, core/extractor.py:20-80).  act: 0 none, 1 ReLU,
// 6 LeakyReLU(0.01).  One block per plane; the plane is read three times (from L2 after the first).
__device__ __forceinline__ float act_f(float v, int act) {
  return act == 1 ? fmaxf(v, 0.f) : act == 6 ? (v >= 0.f ? v : 0.01f * v) : v;
}

__device__ __forceinline__ float block_sum256(float v, float* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// REG: planes of HW <= 256 * IN_MAXN are read once into registers (all loads in flight together) and
// normalised from them -- one HBM read and one write per element; larger planes take three passes.
constexpr int IN_MAXN = 80;               // 20480 px: a 1/4-resolution plane at 640x480

template <bool REG>
__global__ __launch_bounds__(256) void instnorm_kernel(const float* __restrict__ x, const float* __restrict__ res,
                                                       float* __restrict__ out, int HW, float eps, int act1,
                                                       int act2) {
  __shared__ float red[4];
  const float* xp = x + static_cast<size_t>(blockIdx.x) * HW;
  float* op = out + static_cast<size_t>(blockIdx.x) * HW;
  const float* rp = res ? res + static_cast<size_t>(blockIdx.x) * HW : nullptr;
  const int tid = threadIdx.x;
  if constexpr (REG) {
    float v[IN_MAXN];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < IN_MAXN; ++k) v[k] = tid + 256 * k < HW ? xp[tid + 256 * k] : 0.f;
#pragma unroll
    for (int k = 0; k < IN_MAXN; ++k) s += v[k];
    const float mean = block_sum256(s, red) / static_cast<float>(HW);
    float s2 = 0.f;
#pragma unroll
    for (int k = 0; k < IN_MAXN; ++k) {
      const float d = tid + 256 * k < HW ? v[k] - mean : 0.f;
      s2 = fmaf(d, d, s2);
    }
    const float rstd = 1.f / sqrtf(block_sum256(s2, red) / static_cast<float>(HW) + eps);
#pragma unroll
    for (int k = 0; k < IN_MAXN; ++k) {
      const int i = tid + 256 * k;
      if (i < HW) {
        float y = act_f((v[k] - mean) * rstd, act1);
        if (rp) y = act_f(y + rp[i], act2);
        op[i] = y;
      }
    }
  } else {
    float s = 0.f;
    for (int i = tid; i < HW; i += 256) s += xp[i];
    const float mean = block_sum256(s, red) / static_cast<float>(HW);
    float s2 = 0.f;
    for (int i = tid; i < HW; i += 256) {
      const float d = xp[i] - mean;
      s2 = fmaf(d, d, s2);
    }
    const float rstd = 1.f / sqrtf(block_sum256(s2, red) / static_cast<float>(HW) + eps);
    for (int i = tid; i < HW; i += 256) {
      float y = act_f((xp[i] - mean) * rstd, act1);
      if (rp) y = act_f(y + rp[i], act2);
      op[i] = y;
    }
  }
}

// ---------------------------------------------------------------- elementwise
// op 0: a + b, 1: relu(a), 2: relu(a + b), 3: a * b; b is indexed modulo bper (a per-image operand
// broadcast over the batch, e.g. a position embedding)
__global__ __launch_bounds__(256) void ew_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                 float* __restrict__ out, long long n, long long bper, int op) {
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const float x = a[i];
  const float y = b ? b[bper > 0 ? i % bper : i] : 0.f;
  out[i] = op == 0 ? x + y : op == 1 ? fmaxf(x, 0.f) : op == 2 ? fmaxf(x + y, 0.f) : x * y;
}

// ---------------------------------------------------------------- cross-covariance attention
// EdgeNeXt's XCA (timm edgenext CrossCovarianceAttn, the SplitTransposeBlock of core/extractor.py:327's
// edgenext_small): per head, a ch x ch channel attention over the N tokens,
//   attn = softmax_j( <q_i, k_j> / (max(|q_i|, 1e-12) max(|k_j|, 1e-12)) * temperature[h] ),
//   out_i = sum_j attn_ij v_j,
// on the channel-major qkv (B, 3C, N) of its qkv 1x1 conv (q / k / v channel h*ch + i of their third).
// xca_gram_kernel: block (image, head, split) accumulates the Gram matrix <q_i, k_j> and the squared
// row norms over its 1/XCA_NS of the tokens (128-token chunks staged in LDS, one thread per pair) into
// a partial; xca_softmax_kernel: one block per (image, head) sums the XCA_NS partials in split order and
// writes the softmaxed ch x ch map; xca_apply_kernel: one thread per token applies it to the v column.
// ch <= 40.  (Round 6: one block per (image, head) -- 16 blocks for the whole chip -- took 153 us at the
// 1/8-resolution stage; the split spreads the same pairs over B * heads * 16 blocks.)
constexpr int XCA_MAXCH = 40, XCA_NC = 128, XCA_NS = 16;
constexpr int XCA_NPAIR = XCA_MAXCH * XCA_MAXCH + 2 * XCA_MAXCH;

__global__ __launch_bounds__(256) void xca_gram_kernel(const float* __restrict__ qkv, float* __restrict__ part, int C,
                                                       int nh, int N) {
  __shared__ float qs[XCA_MAXCH][XCA_NC + 1];
  __shared__ float ks[XCA_MAXCH][XCA_NC + 1];
  const int ch = C / nh;
  const int bh = blockIdx.x / XCA_NS, sp = blockIdx.x - bh * XCA_NS, h = bh % nh, b = bh / nh;
  const int npair = ch * ch + 2 * ch;
  const int per = (N + XCA_NS - 1) / XCA_NS;
  const int t_begin = sp * per, t_end = min(N, t_begin + per);
  const float* q = qkv + (static_cast<size_t>(b) * 3 * C + static_cast<size_t>(h) * ch) * N;
  const float* k = q + static_cast<size_t>(C) * N;
  constexpr int NP = (XCA_NPAIR + 255) / 256;
  float acc[NP];
#pragma unroll
  for (int u = 0; u < NP; ++u) acc[u] = 0.f;
  for (int n0 = t_begin; n0 < t_end; n0 += XCA_NC) {
    const int nc = min(XCA_NC, t_end - n0);
    __syncthreads();
    for (int e = threadIdx.x; e < ch * XCA_NC; e += 256) {
      const int i = e / XCA_NC, t = e - i * XCA_NC;
      qs[i][t] = t < nc ? q[static_cast<size_t>(i) * N + n0 + t] : 0.f;
      ks[i][t] = t < nc ? k[static_cast<size_t>(i) * N + n0 + t] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      const int pr = u * 256 + threadIdx.x;
      if (pr >= npair) break;
      const float* x;
      const float* y;
      if (pr < ch * ch) {
        x = qs[pr / ch];
        y = ks[pr % ch];
      } else if (pr < ch * ch + ch) {
        x = y = qs[pr - ch * ch];
      } else {
        x = y = ks[pr - ch * ch - ch];
      }
      float s = acc[u];
      for (int t = 0; t < nc; ++t) s = fmaf(x[t], y[t], s);
      acc[u] = s;
    }
  }
  float* pp = part + static_cast<size_t>(blockIdx.x) * npair;
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    const int pr = u * 256 + threadIdx.x;
    if (pr < npair) pp[pr] = acc[u];
  }
}

__global__ __launch_bounds__(256) void xca_softmax_kernel(const float* __restrict__ part,
                                                          const float* __restrict__ temp, float* __restrict__ attn,
                                                          int C, int nh) {
  __shared__ float g[XCA_NPAIR];
  const int ch = C / nh, bh = blockIdx.x, h = bh % nh;
  const int npair = ch * ch + 2 * ch;
  const float* pp = part + static_cast<size_t>(bh) * XCA_NS * npair;
  for (int pr = threadIdx.x; pr < npair; pr += 256) {
    float s = 0.f;
#pragma unroll
    for (int sp = 0; sp < XCA_NS; ++sp) s += pp[sp * npair + pr];
    g[pr] = s;
  }
  __syncthreads();
  // row i: softmax over j of the normalised scores (one thread per row)
  const float tp = temp[h];
  float* ap = attn + static_cast<size_t>(bh) * ch * ch;
  if (threadIdx.x < ch) {
    const int i = threadIdx.x;
    const float qn = fmaxf(sqrtf(g[ch * ch + i]), 1e-12f);
    float mx = -INFINITY;
    for (int j = 0; j < ch; ++j) {
      const float kn = fmaxf(sqrtf(g[ch * ch + ch + j]), 1e-12f);
      const float v = g[i * ch + j] / (qn * kn) * tp;
      g[i * ch + j] = v;
      mx = fmaxf(mx, v);
    }
    float sum = 0.f;
    for (int j = 0; j < ch; ++j) {
      const float e = expf(g[i * ch + j] - mx);
      g[i * ch + j] = e;
      sum += e;
    }
    for (int j = 0; j < ch; ++j) ap[i * ch + j] = g[i * ch + j] / sum;
  }
}

__global__ __launch_bounds__(256) void xca_apply_kernel(const float* __restrict__ qkv, const float* __restrict__ attn,
                                                        float* __restrict__ out, int C, int nh, int N, int ntile) {
  __shared__ float a[XCA_MAXCH * XCA_MAXCH];
  const int ch = C / nh;
  const int bh = blockIdx.x / ntile, h = bh % nh, b = bh / nh;
  const int n = (blockIdx.x - bh * ntile) * 256 + threadIdx.x;
  for (int e = threadIdx.x; e < ch * ch; e += 256) a[e] = attn[static_cast<size_t>(bh) * ch * ch + e];
  __syncthreads();
  if (n >= N) return;
  const float* v = qkv + (static_cast<size_t>(b) * 3 * C + 2 * C + static_cast<size_t>(h) * ch) * N + n;
  float vc[XCA_MAXCH];
#pragma unroll
  for (int j = 0; j < XCA_MAXCH; ++j)
    if (j < ch) vc[j] = v[static_cast<size_t>(j) * N];
  float* op = out + (static_cast<size_t>(b) * C + static_cast<size_t>(h) * ch) * N + n;
  for (int i = 0; i < ch; ++i) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < XCA_MAXCH; ++j)
      if (j < ch) s = fmaf(a[i * ch + j], vc[j], s);
    op[static_cast<size_t>(i) * N] = s;
  }
}

}  // namespace
}  // namespace fsmi

using namespace fsmi;

extern "C" int fsmi_channel_layernorm(const float* x, float* out, const float* w, const float* b, int B, int C, int Tx,
                                      int To, int n, float eps, void* stream) {
  FSMI_CHECK_ARG(x && out, "fsmi_channel_layernorm: null pointer");
  FSMI_CHECK_ARG(B > 0 && C > 0 && n > 0 && n <= Tx && n <= To, "fsmi_channel_layernorm: bad shape (n %d, Tx %d, To %d)",
                 n, Tx, To);
  FSMI_CHECK_ARG(x != out || Tx == To, "fsmi_channel_layernorm: in place needs Tx == To");
  FSMI_CHECK_ARG(C <= LN_G * LN_MAXN, "fsmi_channel_layernorm: C %d > %d", C, LN_G * LN_MAXN);
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_NORM, s);
  const int ntiles = (n + LN_TB - 1) / LN_TB;
  hipLaunchKernelGGL(chan_ln_kernel, dim3(static_cast<unsigned>(B) * ntiles), dim3(256), 0, s, x, out, w, b, C, Tx, To,
                     n, eps, ntiles);
  return finish_launch("fsmi_channel_layernorm");
}

extern "C" long long fsmi_vit_attention_ws_floats(int B, int heads, int T, int Tp) {
  if (B <= 0 || heads <= 0 || T <= 0 || Tp <= 0) return 0;
  int kbs = 0;
  const int ns = vit_attn_splits(B, heads, T, Tp, &kbs);
  return ns > 1 ? static_cast<long long>(ns) * B * heads * (ATT_HD + 2) * Tp : 0;
}

extern "C" int fsmi_vit_attention(const float* qkv, float* out, int B, int heads, int head_dim, int T, int Tp,
                                  float scale, float* ws, long long ws_floats, void* stream) {
  FSMI_CHECK_ARG(qkv && out && qkv != out, "fsmi_vit_attention: null or aliased pointers");
  FSMI_CHECK_ARG(head_dim == ATT_HD, "fsmi_vit_attention: head dim %d (built for 64)", head_dim);
  FSMI_CHECK_ARG(B > 0 && heads > 0 && T > 0 && T <= Tp && Tp % ATT_KB == 0,
                 "fsmi_vit_attention: T %d, Tp %d (Tp a multiple of %d, T <= Tp)", T, Tp, ATT_KB);
  FSMI_CHECK_ARG(reinterpret_cast<uintptr_t>(qkv) % 16 == 0, "fsmi_vit_attention: qkv must be 16-B aligned");
  const long long need = fsmi_vit_attention_ws_floats(B, heads, T, Tp);
  FSMI_CHECK_ARG(ws_floats >= need && (need == 0 || ws), "fsmi_vit_attention: workspace %lld floats < %lld",
                 ws_floats, need);
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_DT, s);
  const float qs = scale * 1.4426950408889634f;
  int kbs = 0;
  const int ns = vit_attn_splits(B, heads, T, Tp, &kbs);
  const int nqt = (Tp + 127) / 128;
  float* opart = ns > 1 ? ws : nullptr;
  float* mlpart = ns > 1 ? ws + static_cast<size_t>(ns) * B * heads * ATT_HD * Tp : nullptr;
  hipLaunchKernelGGL(vit_attn_kernel<4>, dim3(static_cast<unsigned>(B * heads * nqt * ns)), dim3(256), 0, s, qkv, out,
                     heads, T, Tp, qs, nqt, ns, kbs, opart, mlpart);
  if (ns > 1) {
    const long long n = static_cast<long long>(B) * heads * (ATT_HD / 8) * Tp;
    hipLaunchKernelGGL(vit_attn_combine_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, opart,
                       mlpart, out, B * heads, Tp, ns);
  }
  return finish_launch("fsmi_vit_attention");
}

extern "C" int fsmi_space_to_depth(const float* x, float* out, int B, int C, int H, int W, int k, void* stream) {
  FSMI_CHECK_ARG(x && out, "fsmi_space_to_depth: null pointer");
  FSMI_CHECK_ARG(B > 0 && C > 0 && k > 0 && H % k == 0 && W % k == 0 && H > 0 && W > 0,
                 "fsmi_space_to_depth: %dx%d not divisible by %d", H, W, k);
  hipStream_t s = as_stream(stream);
  const long long n = static_cast<long long>(B) * C * H * W;
  hipLaunchKernelGGL(s2d_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, s, x, out, C, H, W, k, n);
  return finish_launch("fsmi_space_to_depth");
}

extern "C" int fsmi_depth_to_space(const float* x, float* out, int B, int C, int H, int W, int k, void* stream) {
  FSMI_CHECK_ARG(x && out, "fsmi_depth_to_space: null pointer");
  FSMI_CHECK_ARG(B > 0 && C > 0 && H > 0 && W > 0 && k > 0, "fsmi_depth_to_space: bad shape");
  hipStream_t s = as_stream(stream);
  const long long n = static_cast<long long>(B) * C * H * W * k * k;
  hipLaunchKernelGGL(d2s_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, s, x, out, C, H, W, k, n);
  return finish_launch("fsmi_depth_to_space");
}

extern "C" int fsmi_vit_tokens(const float* emb, const float* cls, const float* pos, float* out, int B, int C, int N,
                               int Tp, void* stream) {
  FSMI_CHECK_ARG(emb && cls && pos && out, "fsmi_vit_tokens: null pointer");
  FSMI_CHECK_ARG(B > 0 && C > 0 && N > 0 && Tp > N, "fsmi_vit_tokens: Tp %d must exceed N %d", Tp, N);
  hipStream_t s = as_stream(stream);
  const long long n = static_cast<long long>(B) * C * Tp;
  hipLaunchKernelGGL(vit_tokens_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, s, emb, cls, pos, out, C, N, Tp, n);
  return finish_launch("fsmi_vit_tokens");
}

extern "C" int fsmi_resize_bicubic(const float* x, float* out, int B, int C, int Hi, int Wi, int Ho, int Wo,
                                   void* stream) {
  FSMI_CHECK_ARG(x && out && x != out, "fsmi_resize_bicubic: null or aliased pointers");
  FSMI_CHECK_ARG(B > 0 && C > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0, "fsmi_resize_bicubic: bad shape");
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_RESIZE, s);
  const long long n = static_cast<long long>(B) * C * Ho * Wo;
  hipLaunchKernelGGL(bicubic_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, s, x, out, Hi, Wi, Ho, Wo,
                     static_cast<float>(Hi) / static_cast<float>(Ho), static_cast<float>(Wi) / static_cast<float>(Wo),
                     n);
  return finish_launch("fsmi_resize_bicubic");
}

extern "C" int fsmi_instance_norm(const float* x, const float* res, float* out, int planes, int HW, float eps, int act1,
                                  int act2, void* stream) {
  FSMI_CHECK_ARG(x && out, "fsmi_instance_norm: null pointer");
  FSMI_CHECK_ARG(planes > 0 && HW > 0, "fsmi_instance_norm: bad shape");
  FSMI_CHECK_ARG((act1 == 0 || act1 == 1 || act1 == 6) && (act2 == 0 || act2 == 1 || act2 == 6),
                 "fsmi_instance_norm: act 0 / 1 / 6");
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_NORM, s);
  if (HW <= 256 * IN_MAXN)
    hipLaunchKernelGGL(instnorm_kernel<true>, dim3(static_cast<unsigned>(planes)), dim3(256), 0, s, x, res, out, HW,
                       eps, act1, act2);
  else
    hipLaunchKernelGGL(instnorm_kernel<false>, dim3(static_cast<unsigned>(planes)), dim3(256), 0, s, x, res, out, HW,
                       eps, act1, act2);
  return finish_launch("fsmi_instance_norm");
}

extern "C" int fsmi_elementwise(const float* a, const float* b, float* out, long long n, long long bper, int op,
                                void* stream) {
  FSMI_CHECK_ARG(a && out && n > 0, "fsmi_elementwise: null pointer / empty");
  FSMI_CHECK_ARG(op >= 0 && op <= 3 && (b || op == 1), "fsmi_elementwise: op %d", op);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(ew_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, s, a, b, out, n, bper, op);
  return finish_launch("fsmi_elementwise");
}

extern "C" long long fsmi_xca_workspace_floats(int B, int C, int heads) {
  if (B <= 0 || heads <= 0 || C % heads) return 0;
  const long long ch = C / heads;
  return static_cast<long long>(B) * heads * (ch * ch + XCA_NS * (ch * ch + 2 * ch));
}

extern "C" int fsmi_xca(const float* qkv, const float* temperature, float* ws, float* out, int B, int C, int heads,
                        int N, void* stream) {
  FSMI_CHECK_ARG(qkv && temperature && ws && out && out != qkv, "fsmi_xca: null or aliased pointers");
  FSMI_CHECK_ARG(B > 0 && heads > 0 && N > 0 && C % heads == 0 && C / heads <= XCA_MAXCH,
                 "fsmi_xca: C %d over %d heads (<= %d channels per head)", C, heads, XCA_MAXCH);
  hipStream_t s = as_stream(stream);
  const int ch = C / heads;
  float* attn = ws;                                          // B * heads * ch * ch
  float* part = ws + static_cast<size_t>(B) * heads * ch * ch;   // B * heads * XCA_NS * (ch * ch + 2 ch)
  hipLaunchKernelGGL(xca_gram_kernel, dim3(static_cast<unsigned>(B * heads * XCA_NS)), dim3(256), 0, s, qkv, part,
                     C, heads, N);
  hipLaunchKernelGGL(xca_softmax_kernel, dim3(static_cast<unsigned>(B * heads)), dim3(256), 0, s, part, temperature,
                     attn, C, heads);
  const int ntile = (N + 255) / 256;
  hipLaunchKernelGGL(xca_apply_kernel, dim3(static_cast<unsigned>(B * heads * ntile)), dim3(256), 0, s, qkv, attn,
                     out, C, heads, N, ntile);
  return finish_launch("fsmi_xca");
}
