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
                                                             float* __restrict__ o1, int C, int HW, long long P,
                                                             unsigned long long* clk) {
  clock_begin(clk);
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
  clock_end(clk);
}

// all-pairs on pre-normalised operands: no LDS, no barriers.  Block = (b, h,
// w1 tile), one wave per w2 tile; each wave streams its two 32-column slabs
// from L2 (row-major blocks of a row share one XCD) 16 k-steps of loads ahead
// of the MFMAs that consume them.
template <int MAXT>
__global__ __launch_bounds__(MAXT * kWave) void allpairs_corr_direct_kernel(
    const float* __restrict__ nl, const float* __restrict__ nr, float* __restrict__ lv0, float* __restrict__ lv1,
    float* __restrict__ lv2, float* __restrict__ lv3, int L, int C, int H, int W, int T, unsigned long long* clk) {
  clock_begin(clk);
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
  clock_end(clk);
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
                                                             int HW, int nq, long long total,
                                                             unsigned long long* clk) {
  clock_begin(clk);
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
  clock_end(clk);
}

// ---------------------------------------------------------------------------
// a6: fused lookup (core/geometry.py:43-65 + core/utils/utils.py:44-55).  Grid = (B * ceil(HW/64),
// L, nchunk/4); one wave = 64 consecutive pixels of one image x 4 geo channels (or the corr
// channel) of one level.  Coordinates follow bilinear_sampler: x -> 2x/(n-1)-1 -> (x'+1) *
// ((n-1)/2) (the CPU grid_sampler's align_corners unnormalise), then linear interpolation with
// zero padding.  (2 or 7 channels per wave, FSMI_LOOKUP_CPC: within 1 % back to back and in the
// step, round 4.)
// ---------------------------------------------------------------------------
struct LookupArgs {
  const float* vol[FSMI_MAX_LEVELS];
  const float* cor[FSMI_MAX_LEVELS];
  const float* disp;
  const float* coords;       // (B,H,W) column coordinates of the corr taps; nullptr: the pixel column w
  float* out;
  int L, Cv, D, H, W, W2, B;
  unsigned long long* clk;   // in-kernel launch clock (nullptr: off)
};

// Branch-free buffer addressing (round 4; replaced per-lane exec-masked global loads and a 64-bit
// division per lane: 43.9 -> 37.7 us in the cfg2 step, 36.3 -> 30.9 us back to back).
// Grid = (B * ceil(HW/64), L, nchunk/4): the pixel tile never straddles two images, so b comes
// from blockIdx.  Every element is a raw buffer load from a per-channel resource (base = the
// channel's (D_i, HW) plane, wave-uniform, num_records = its size): an element outside [0, D_i)
// or a lane past the image gets the offset 0x80000000, which the buffer unit answers with 0 without
// a memory access -- grid_sample's zero padding from the hardware range check, no exec-mask
// branches.  The offsets are channel-invariant (only the resource base moves), so every channel
// costs 2r+2 loads + K stores and no address VALU.  Outputs go through the same mechanism
// (per-channel resource over its K tap planes; tail lanes out of range).
constexpr unsigned kOOB = 0x80000000u;
constexpr int kBufFlags = 0x00020000;   // raw buffer, 32-bit data format (gfx9 resource word 3)

// base and size are wave-uniform by construction; readfirstlane states it, so the resource is built
// in SGPRs (a resource the compiler believes divergent costs a waterfall loop per buffer access)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const float* base, unsigned bytes) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(base);
  const unsigned lo = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(v));
  const unsigned hi = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(v >> 32));
  float* p = reinterpret_cast<float*>((static_cast<unsigned long long>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, static_cast<int>(__builtin_amdgcn_readfirstlane(bytes)), kBufFlags);
}

// a kernel-argument array indexed by a uniform level: a select chain keeps the pointer in SGPRs
// (a dynamic index into the by-value argument copies the array to scratch and makes it divergent)
__device__ __forceinline__ const float* level_ptr(const float* const (&arr)[FSMI_MAX_LEVELS], int i) {
  const float* r = arr[0];
#pragma unroll
  for (int l = 1; l < FSMI_MAX_LEVELS; ++l) r = i == l ? arr[l] : r;
  return r;
}

// Tap interpolation without data-dependent selects (a per-tap select between window elements is
// folded by the compiler into a dynamically indexed private array: scratch traffic).  A lane's taps
// sit at window pairs (k + sel, k + sel + 1); sel differs from 1 only where the unnormalise round
// trip crosses an integer.  FAST (wave-uniform: every lane's every tap at sel = 1): the 2r+2 inner
// window loads, each tap from fixed window slots.  Otherwise each tap loads its own pair at the
// element it needs (2 loads per tap, the extra ones served by the caches) -- same products, same
// add order, same values.
struct PlaneAddr {          // byte offset of element x of a lane's row: (x * rstride + col) * 4
  int rstride, col, n;
  bool live;
  __device__ __forceinline__ unsigned off(int x) const {
    return (live && x >= 0 && x < n) ? static_cast<unsigned>(x * rstride + col) * 4u : kOOB;
  }
};

template <int R, bool FAST>
__device__ __forceinline__ void lookup_plane(__amdgpu_buffer_rsrc_t src, const Taps<R>& tp, const PlaneAddr& pa,
                                             __amdgpu_buffer_rsrc_t dst, const unsigned (&so)[2 * R + 1]) {
#pragma clang fp contract(off)
  constexpr int K = 2 * R + 1;
  float o[K];
  if constexpr (FAST) {
    float win[2 * R + 2];
#pragma unroll
    for (int j = 0; j < 2 * R + 2; ++j)
      win[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(src, pa.off(tp.xb + 1 + j), 0, 0));
#pragma unroll
    for (int k = 0; k < K; ++k) o[k] = win[k] * (1.f - tp.f[k]) + win[k + 1] * tp.f[k];
  } else {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int x0 = tp.xb + k + tp.sel[k];
      const float v0 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(src, pa.off(x0), 0, 0));
      const float v1 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(src, pa.off(x0 + 1), 0, 0));
      o[k] = v0 * (1.f - tp.f[k]) + v1 * tp.f[k];
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o[k]), dst, so[k], 0, 0);
}

template <int R, int CPC>
__global__ __launch_bounds__(256) void geo_lookup_kernel(LookupArgs a, int tiles) {
  constexpr int K = 2 * R + 1;
  // the wave index is uniform: readfirstlane tells the compiler, so every resource below stays scalar
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = blockIdx.y;  // level
  clock_begin(a.clk);
  const int chunk = blockIdx.z * 4 + wave;
  const int nchunk_geo = (a.Cv + CPC - 1) / CPC;
  if (chunk > nchunk_geo) return;                       // wave-uniform
  const int b = blockIdx.x / tiles;
  const int HW = a.H * a.W;
  const int hw = (blockIdx.x - b * tiles) * 64 + lane;
  const bool live = hw < HW;
  const int hwc = live ? hw : HW - 1;
  const float inv_s = 1.f / static_cast<float>(1 << i);  // exact: x * 2^-i == x / 2^i
  const float ds = a.disp[static_cast<size_t>(b) * HW + hwc] * inv_s;
  const int CH = a.L * K * (a.Cv + 1);
  const float* outb = a.out + (static_cast<size_t>(b) * CH + static_cast<size_t>(i) * K * (a.Cv + 1)) * HW;
  unsigned so[K];                                        // store offsets (bytes) in a channel's K planes
#pragma unroll
  for (int k = 0; k < K; ++k) so[k] = live ? static_cast<unsigned>(k * HW + hw) * 4u : kOOB;
  Taps<R> tp;
  PlaneAddr pa;
  pa.live = live;
  const float* src_base;
  unsigned src_bytes;
  int nplanes, first_plane;
  size_t src_step;
  if (chunk < nchunk_geo) {
    const int Di = a.D >> i;
    tp.init(ds, Di);
    pa.rstride = HW;
    pa.col = hw;
    pa.n = Di;
    const int c0 = chunk * CPC;
    first_plane = c0;
    nplanes = min(CPC, a.Cv - c0);
    src_step = static_cast<size_t>(Di) * HW;
    src_base = level_ptr(a.vol, i) + (static_cast<size_t>(b) * a.Cv + c0) * src_step;
    src_bytes = static_cast<unsigned>(Di * HW) * 4u;
  } else {
    // correlation channel: each lane's row of the W2 pyramid level, contiguous over x
    const int W2i = a.W2 >> i;
    // the reference's init_x0 = coords / 2^i - disp / 2^i + dx (core/geometry.py:57); the model passes
    // coords = arange(W) per row (core/foundation_stereo.py:231), derived here without a load
    const int w = hwc - (hwc / a.W) * a.W;
    const float cw = a.coords ? a.coords[static_cast<size_t>(b) * HW + hwc] : static_cast<float>(w);
    tp.init(cw * inv_s - ds, W2i);
    const int p0 = (blockIdx.x - b * tiles) * 64;        // first pixel of the tile
    pa.rstride = 1;
    pa.col = lane * W2i;
    pa.n = W2i;
    first_plane = a.Cv;
    nplanes = 1;
    src_step = 0;
    src_base = level_ptr(a.cor, i) + (static_cast<size_t>(b) * HW + p0) * W2i;
    src_bytes = static_cast<unsigned>(min(64, HW - p0) * W2i) * 4u;
  }
  bool odd = false;
#pragma unroll
  for (int k = 0; k < K; ++k) odd |= tp.sel[k] != 1;
  const bool fast = __builtin_amdgcn_ballot_w64(odd) == 0;   // wave-uniform
#pragma unroll
  for (int u = 0; u < CPC; ++u) {
    if (u < nplanes) {                                   // wave-uniform (ragged last chunk)
      const __amdgpu_buffer_rsrc_t src = buf_rsrc(src_base + u * src_step, src_bytes);
      const __amdgpu_buffer_rsrc_t dst =
          buf_rsrc(outb + static_cast<size_t>(first_plane + u) * K * HW, static_cast<unsigned>(K * HW) * 4u);
      if (fast)
        lookup_plane<R, true>(src, tp, pa, dst, so);
      else
        lookup_plane<R, false>(src, tp, pa, dst, so);
    }
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
    const unsigned ngrid = ceil_div(P, 64), cgrid = static_cast<unsigned>(B) * H * T;
    hipLaunchKernelGGL(normalize_cols_kernel, dim3(ngrid, 2), dim3(64), 0, s, fl, fr, nl, nr, C, H * W, P,
                       clock_slot(FSMI_K_NORM, s, 2ll * ngrid));
    // up to 8 w2 tiles (W <= 256) with a 512-thread bound: 128 VGPRs (the 1024-thread bound) spilled
    unsigned long long* clk = clock_slot(FSMI_K_CORR, s, static_cast<long long>(cgrid) * T, "allpairs_corr");
    if (T <= 8)
      hipLaunchKernelGGL(allpairs_corr_direct_kernel<8>, dim3(cgrid), dim3(T * kWave), 0, s, nl, nr, lv[0], lv[1],
                         lv[2], lv[3], num_levels, C, H, W, T, clk);
    else
      hipLaunchKernelGGL(allpairs_corr_direct_kernel<kCorrMaxT>, dim3(cgrid), dim3(T * kWave), 0, s, nl, nr, lv[0],
                         lv[1], lv[2], lv[3], num_levels, C, H, W, T, clk);
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
  unsigned long long* clk = clock_slot(FSMI_K_VOLPYR, s, 4ll * grid);
  switch (S) {
    case 2: hipLaunchKernelGGL(volume_pyramid_kernel<2>, dim3(grid), dim3(256), 0, s, vol, o[0], o[1], o[2], D, HW, nq, total, clk); break;
    case 4: hipLaunchKernelGGL(volume_pyramid_kernel<4>, dim3(grid), dim3(256), 0, s, vol, o[0], o[1], o[2], D, HW, nq, total, clk); break;
    default: hipLaunchKernelGGL(volume_pyramid_kernel<8>, dim3(grid), dim3(256), 0, s, vol, o[0], o[1], o[2], D, HW, nq, total, clk); break;
  }
  return finish_launch("fsmi_volume_pyramid");
}

int fsmi_geo_lookup(const float* const* vol_levels, const float* const* corr_levels, const float* disp, float* out,
                    int num_levels, int radius, int B, int Cv, int D, int H, int W, int W2, void* stream) {
  return fsmi_geo_lookup_coords(vol_levels, corr_levels, disp, nullptr, out, num_levels, radius, B, Cv, D, H, W, W2,
                                stream);
}

int fsmi_geo_lookup_coords(const float* const* vol_levels, const float* const* corr_levels, const float* disp,
                           const float* coords, float* out, int num_levels, int radius, int B, int Cv, int D, int H,
                           int W, int W2, void* stream) {
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
  a.coords = coords;
  a.out = out;
  a.L = num_levels;
  a.Cv = Cv;
  a.D = D;
  a.H = H;
  a.W = W;
  a.W2 = W2;
  a.B = B;
  const int HW = H * W;
  const int tiles = (HW + 63) / 64;
  // buffer offsets inside one channel plane, one channel's K tap planes and one tile's corr rows
  // are 31-bit
  FSMI_CHECK_ARG(static_cast<long long>(D) * HW * 4 < (1ll << 31) &&
                     static_cast<long long>(2 * radius + 1) * HW * 4 < (1ll << 31) &&
                     static_cast<long long>(B) * tiles < (1ll << 31),
                 "fsmi_geo_lookup: a channel plane exceeds 2 GB (D=%d, H*W=%d)", D, HW);
  // geo channels per wave (FSMI_LOOKUP_CPC: 2 / 4 / 7 at radius 4, an A/B knob)
  static const int env_cpc = [] { const char* e = getenv("FSMI_LOOKUP_CPC"); const int v = e ? atoi(e) : 4;
                                  return (v == 2 || v == 7) ? v : 4; }();
  const int cpc = radius == 4 ? env_cpc : 4;
  const int nchunk = (Cv + cpc - 1) / cpc + 1;
  dim3 grid(static_cast<unsigned>(B * tiles), num_levels, (nchunk + 3) / 4);
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_LOOKUP, s);
  auto launch = [grid, radius, s, tiles, cpc](const LookupArgs& la) {
    if (radius == 4 && cpc == 2) {
      hipLaunchKernelGGL((geo_lookup_kernel<4, 2>), grid, dim3(256), 0, s, la, tiles);
    } else if (radius == 4 && cpc == 7) {
      hipLaunchKernelGGL((geo_lookup_kernel<4, 7>), grid, dim3(256), 0, s, la, tiles);
    } else {
      switch (radius) {
        case 2: hipLaunchKernelGGL((geo_lookup_kernel<2, 4>), grid, dim3(256), 0, s, la, tiles); break;
        case 3: hipLaunchKernelGGL((geo_lookup_kernel<3, 4>), grid, dim3(256), 0, s, la, tiles); break;
        default: hipLaunchKernelGGL((geo_lookup_kernel<4, 4>), grid, dim3(256), 0, s, la, tiles); break;
      }
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
