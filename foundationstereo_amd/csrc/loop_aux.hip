// Refinement-loop auxiliaries that MIOpen / ATen run poorly at these shapes:
//  * depthwise KxK conv (EdgeNeXt dwconv of DispHead, core/submodule.py:565-591, and of the backbone's
//    EdgeNeXt-S ConvBlocks / SplitTransposeBlocks, core/extractor.py:327):
//    MIOpen routes it through NCHW->NHWC transposes and a grouped CK kernel
//    (~105 us at 128x120x160); here it is one LDS-tiled pass (HBM-bound: one
//    read + one write of the plane);
//  * bilinear resize with align_corners=True (interp(), core/update.py:80).
#include "fsmi_common.h"

namespace fsmi {
namespace {

constexpr int DW_TR = 16, DW_TC = 64;   // conv_1in output tile per block (rows x cols), 4 rows per thread
// dwconv: 32 x 64 output tile, 8 rows per thread -- the (KS-1)-row halo is re-read for half as many
// outputs and each LDS window row feeds up to 8 accumulators (16 x 64 with 4 rows: 1 TB/s at cfg2)
constexpr int DWK_TR = 32, DWK_RPT = 8;

// Stage the zero-padded IR x IC input window at (r0 - P, c0 - P) of a plane (plus an optional second
// plane summed in) into LDS.  Unrolled: every thread issues all of its global loads before its first
// LDS store (a rolled loop waits one HBM latency per element -- 11 of them for the 7x7 window, which
// made the depthwise conv ~4x its streaming time)
template <int IR, int IC, int LDW>
__device__ __forceinline__ void stage_window(float (*tile)[LDW], const float* __restrict__ xp,
                                             const float* __restrict__ ap, int r0, int c0, int P, int H, int W) {
  constexpr int NE = (IR * IC + 255) / 256;
  float v[NE];
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    const int e = threadIdx.x + 256 * k;
    const int ir = e / IC, ic = e - ir * IC;
    const int hh = r0 + ir - P, ww = c0 + ic - P;
    v[k] = 0.f;
    if (e < IR * IC && hh >= 0 && hh < H && ww >= 0 && ww < W) {
      v[k] = xp[hh * W + ww];
      if (ap) v[k] += ap[hh * W + ww];
    }
  }
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    const int e = threadIdx.x + 256 * k;
    const int ir = e / IC, ic = e - ir * IC;
    if (e < IR * IC) tile[ir][ic] = v[k];
  }
}

// x / add / out planes (b, c) at (b * ctot + c) * H * W of their tensors (channel slices of wider maps);
// add (optional) is summed into the input as it is staged (EdgeNeXt's multi-scale split, the
// `sp = sp + spx[i]` before each depthwise conv, timm edgenext SplitTransposeBlock)
template <int KS>
__global__ __launch_bounds__(256) void dwconv_kernel(const float* __restrict__ x, const float* __restrict__ add,
                                                     const float* __restrict__ w,
                                                     const float* __restrict__ bias, float* __restrict__ out,
                                                     int C, int H, int W, int ntr, int ntc, int xct, int adct,
                                                     int oct, unsigned long long* clk) {
  FSMI_TIMELINE_CLOCK(clk);
  constexpr int P = KS / 2, IR = DWK_TR + KS - 1, IC = DW_TC + KS - 1, RPT = DWK_RPT;
  __shared__ float tile[IR][IC + 1];
  const int plane = blockIdx.x / (ntr * ntc);
  const int t = blockIdx.x - plane * ntr * ntc;
  const int r0 = (t / ntc) * DWK_TR, c0 = (t % ntc) * DW_TC;
  const int c = plane % C, bimg = plane / C;
  const float* xp = x + (static_cast<size_t>(bimg) * xct + c) * H * W;
  const float* ap = add ? add + (static_cast<size_t>(bimg) * adct + c) * H * W : nullptr;
  stage_window<IR, IC, IC + 1>(tile, xp, ap, r0, c0, P, H, W);
  float wk[KS * KS];
#pragma unroll
  for (int k = 0; k < KS * KS; ++k) wk[k] = w[c * KS * KS + k];   // block-uniform: scalar loads
  __syncthreads();
  const int col = threadIdx.x & 63, rb = (threadIdx.x >> 6) * RPT;
  const float b0 = bias ? bias[c] : 0.f;
  float acc[RPT];
#pragma unroll
  for (int o = 0; o < RPT; ++o) acc[o] = b0;
#pragma unroll
  for (int ir = 0; ir < RPT + KS - 1; ++ir) {
    float v[KS];
#pragma unroll
    for (int kw = 0; kw < KS; ++kw) v[kw] = tile[rb + ir][col + kw];
#pragma unroll
    for (int o = 0; o < RPT; ++o) {
      const int kh = ir - o;
      if (kh >= 0 && kh < KS) {
#pragma unroll
        for (int kw = 0; kw < KS; ++kw) acc[o] = fmaf(wk[kh * KS + kw], v[kw], acc[o]);
      }
    }
  }
  float* op = out + (static_cast<size_t>(bimg) * oct + c) * H * W;
#pragma unroll
  for (int o = 0; o < RPT; ++o) {
    const int hh = r0 + rb + o, ww = c0 + col;
    if (hh < H && ww < W) op[hh * W + ww] = acc[o];
  }
}

// Single-input-channel KSxKS conv (+ bias, optional ReLU): the motion encoder's convd1,
// Conv2d(1, 64, 7, padding=3) + ReLU (core/update.py:57,67).  Block = 16x64 output pixels x
// CO_PER output channels (blockIdx.y); the thread's (4 + KS - 1) x KS input window is read from
// LDS into registers once and reused for every output channel; weights are block-uniform.
constexpr int C1_CO = 8;
template <int KS>
__global__ __launch_bounds__(256) void conv_1in_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                       const float* __restrict__ bias, float* __restrict__ out,
                                                       int Cout, int H, int W, int ntr, int ntc, int relu,
                                                       unsigned long long* clk) {
  FSMI_TIMELINE_CLOCK(clk);
  constexpr int P = KS / 2, IR = DW_TR + KS - 1, IC = DW_TC + KS - 1;
  __shared__ float tile[IR][IC + 1];
  const int b = blockIdx.x / (ntr * ntc);
  const int t = blockIdx.x - b * ntr * ntc;
  const int r0 = (t / ntc) * DW_TR, c0 = (t % ntc) * DW_TC;
  const float* xp = x + static_cast<size_t>(b) * H * W;
  stage_window<IR, IC, IC + 1>(tile, xp, nullptr, r0, c0, P, H, W);
  __syncthreads();
  const int col = threadIdx.x & 63, rb = (threadIdx.x >> 6) * 4;
  float v[4 + KS - 1][KS];
#pragma unroll
  for (int ir = 0; ir < 4 + KS - 1; ++ir)
#pragma unroll
    for (int kw = 0; kw < KS; ++kw) v[ir][kw] = tile[rb + ir][col + kw];
  const int co_end = min(Cout, static_cast<int>(blockIdx.y + 1) * C1_CO);
  for (int co = blockIdx.y * C1_CO; co < co_end; ++co) {
    const float* wk = w + co * KS * KS;                 // uniform: scalar loads
    const float b0 = bias ? bias[co] : 0.f;
    float acc[4] = {b0, b0, b0, b0};
#pragma unroll
    for (int kh = 0; kh < KS; ++kh)
#pragma unroll
      for (int kw = 0; kw < KS; ++kw) {
        const float wv = wk[kh * KS + kw];
#pragma unroll
        for (int o = 0; o < 4; ++o) acc[o] = fmaf(wv, v[o + kh][kw], acc[o]);
      }
    float* op = out + (static_cast<size_t>(b) * Cout + co) * H * W;
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const int hh = r0 + rb + o, ww = c0 + col;
      if (hh < H && ww < W) op[hh * W + ww] = relu ? fmaxf(acc[o], 0.f) : acc[o];
    }
  }
}

// pool2x: F.avg_pool2d(x, 3, stride=2, padding=1) with count_include_pad (every window / 9),
// core/update.py:72-73.  One thread per output; the 3 input rows are contiguous 3-float runs.
__global__ __launch_bounds__(256) void pool2x_kernel(const float* __restrict__ x, float* __restrict__ out,
                                                     int H, int W, int Ho, int Wo, long long n,
                                                     unsigned long long* clk) {
  FSMI_TIMELINE_CLOCK(clk);
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const int ox = static_cast<int>(i % Wo);
  const int oy = static_cast<int>((i / Wo) % Ho);
  const long long p = i / (static_cast<long long>(Ho) * Wo);
  const float* xp = x + p * H * W;
  float s = 0.f;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy) {
    const int y = 2 * oy + dy;
    if (y < 0 || y >= H) continue;
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      const int xx = 2 * ox + dx;
      if (xx >= 0 && xx < W) s += xp[y * W + xx];
    }
  }
  out[i] = s / 9.f;
}

// F.interpolate(mode="bilinear", align_corners=True): src = dst * (in-1)/(out-1)
__global__ __launch_bounds__(256) void resize_kernel(const float* __restrict__ x, float* __restrict__ out,
                                                     long long planes, int Hi, int Wi, int Ho, int Wo, float sh,
                                                     float sw,
                                                     unsigned long long* clk) {
#pragma clang fp contract(off)
  FSMI_TIMELINE_CLOCK(clk);
  const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  const long long n = planes * Ho * Wo;
  if (i >= n) return;
  const int ox = static_cast<int>(i % Wo);
  const int oy = static_cast<int>((i / Wo) % Ho);
  const long long p = i / (static_cast<long long>(Ho) * Wo);
  const float fy = sh * oy, fx = sw * ox;
  const int y0 = static_cast<int>(fy), x0 = static_cast<int>(fx);
  const int y1 = y0 + (y0 < Hi - 1 ? 1 : 0), x1 = x0 + (x0 < Wi - 1 ? 1 : 0);
  const float ly = fy - y0, lx = fx - x0;
  const float hy = 1.f - ly, hx = 1.f - lx;
  const float* xp = x + p * Hi * Wi;
  const float top = hx * xp[y0 * Wi + x0] + lx * xp[y0 * Wi + x1];
  const float bot = hx * xp[y1 * Wi + x0] + lx * xp[y1 * Wi + x1];
  out[i] = hy * top + ly * bot;
}


// Conv2d(Cin, 1, 3, padding=1) + bias (+ res): DispHead's last layer (core/update.py:28), the loop's
// disp + delta.  One output channel leaves 31 of 32 MFMA rows of a halo tile idle (19 us at cfg2 on
// the 32-cout tile); here it is a VALU dot product per pixel in fp32: a block is a 2 x 64 pixel tile,
// its four waves each sum a quarter of the channels (9 taps from global memory, L1-resident) and
// combine through LDS in wave order (deterministic).
constexpr int C1O_TR = 2, C1O_TC = 64;
__global__ __launch_bounds__(256) void conv3x3_cout1_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ bias, const float* __restrict__ res,
                                                            long long res_bstride, float* __restrict__ out,
                                                            long long out_bstride, int Cin, int H, int W, int ntr,
                                                            int ntc, unsigned long long* clk) {
  FSMI_TIMELINE_CLOCK(clk);
  __shared__ float part[4][C1O_TR * C1O_TC];
  const int b = blockIdx.x / (ntr * ntc);
  const int t = blockIdx.x - b * ntr * ntc;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c0 = (t % ntc) * C1O_TC + lane, r0 = (t / ntc) * C1O_TR;
  const int cq = (Cin + 3) / 4, cb = wave * cq, ce = min(Cin, cb + cq);
  const long long HW = static_cast<long long>(H) * W;
  const float* xb = x + (static_cast<long long>(b) * Cin) * HW;
  // per tap: offset and validity of the (r0 + rr + dh - 1, c0 + dw - 1) input pixel, rr in [0, TR)
  float acc[C1O_TR];
#pragma unroll
  for (int rr = 0; rr < C1O_TR; ++rr) acc[rr] = 0.f;
#pragma unroll 4
  for (int c = cb; c < ce; ++c) {
    const float* xc = xb + c * HW;
    const float* wc = w + c * 9;                   // uniform: scalar loads
    float v[C1O_TR + 2][3];
#pragma unroll
    for (int ir = 0; ir < C1O_TR + 2; ++ir) {
      const int hh = r0 + ir - 1;
#pragma unroll
      for (int dw = 0; dw < 3; ++dw) {
        const int ww = c0 + dw - 1;
        v[ir][dw] = (hh >= 0 && hh < H && ww >= 0 && ww < W) ? xc[hh * W + ww] : 0.f;
      }
    }
#pragma unroll
    for (int rr = 0; rr < C1O_TR; ++rr)
#pragma unroll
      for (int dh = 0; dh < 3; ++dh)
#pragma unroll
        for (int dw = 0; dw < 3; ++dw) acc[rr] = fmaf(wc[dh * 3 + dw], v[rr + dh][dw], acc[rr]);
  }
#pragma unroll
  for (int rr = 0; rr < C1O_TR; ++rr) part[wave][rr * C1O_TC + lane] = acc[rr];
  __syncthreads();
  if (wave < C1O_TR) {
    const int rr = wave, hh = r0 + rr;
    if (hh < H && c0 < W) {
      float s = part[0][rr * C1O_TC + lane];
#pragma unroll
      for (int q = 1; q < 4; ++q) s += part[q][rr * C1O_TC + lane];
      if (bias) s += bias[0];
      const long long p = static_cast<long long>(hh) * W + c0;
      if (res) s += res[b * res_bstride + p];
      out[b * out_bstride + p] = s;
    }
  }
}
}  // namespace
}  // namespace fsmi

using namespace fsmi;

extern "C" int fsmi_dwconv2d_ex(const float* x, int x_ctot, const float* add, int add_ctot, const float* w,
                                const float* bias, float* out, int out_ctot, int B, int C, int KS, int H, int W,
                                void* stream) {
  FSMI_CHECK_ARG(x && w && out, "fsmi_dwconv2d: null pointer");
  FSMI_CHECK_ARG(B > 0 && C > 0 && H > 0 && W > 0, "fsmi_dwconv2d: bad shape");
  FSMI_CHECK_ARG(x_ctot >= C && out_ctot >= C && (!add || add_ctot >= C), "fsmi_dwconv2d: channel slice wider than "
                 "its tensor");
  FSMI_CHECK_ARG(KS == 3 || KS == 5 || KS == 7 || KS == 9, "fsmi_dwconv2d: kernel %d unsupported (3, 5, 7, 9)", KS);
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_DWCONV, s);
  const int ntr = (H + DWK_TR - 1) / DWK_TR, ntc = (W + DW_TC - 1) / DW_TC;
  const dim3 grid(static_cast<unsigned>(B) * C * ntr * ntc);
  unsigned long long* clk = clock_slot(FSMI_K_DWCONV, s, 4ll * grid.x * grid.y * grid.z, "dwconv", true);
#define FSMI_DW_LAUNCH(K) hipLaunchKernelGGL(dwconv_kernel<K>, grid, dim3(256), 0, s, x, add, w, bias, out, C, H, W, \
                                             ntr, ntc, x_ctot, add_ctot, out_ctot, clk)
  if (KS == 7) FSMI_DW_LAUNCH(7);
  else if (KS == 5) FSMI_DW_LAUNCH(5);
  else if (KS == 9) FSMI_DW_LAUNCH(9);
  else FSMI_DW_LAUNCH(3);
#undef FSMI_DW_LAUNCH
  return finish_launch("fsmi_dwconv2d");
}

extern "C" int fsmi_dwconv2d(const float* x, const float* w, const float* bias, float* out, int B, int C, int KS,
                             int H, int W, void* stream) {
  return fsmi_dwconv2d_ex(x, C, nullptr, C, w, bias, out, C, B, C, KS, H, W, stream);
}

extern "C" int fsmi_conv2d_1in(const float* x, const float* w, const float* bias, float* out, int B, int Cout, int KS,
                               int H, int W, int relu, void* stream) {
  FSMI_CHECK_ARG(x && w && out, "fsmi_conv2d_1in: null pointer");
  FSMI_CHECK_ARG(B > 0 && Cout > 0 && H > 0 && W > 0, "fsmi_conv2d_1in: bad shape");
  FSMI_CHECK_ARG(KS == 3 || KS == 5 || KS == 7, "fsmi_conv2d_1in: kernel %d unsupported (3, 5, 7)", KS);
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_DWCONV, s);
  const int ntr = (H + DW_TR - 1) / DW_TR, ntc = (W + DW_TC - 1) / DW_TC;
  const dim3 grid(static_cast<unsigned>(B) * ntr * ntc, (Cout + C1_CO - 1) / C1_CO);
  unsigned long long* clk = clock_slot(FSMI_K_DWCONV, s, 4ll * grid.x * grid.y * grid.z, "conv_1in", true);
  if (KS == 7) hipLaunchKernelGGL(conv_1in_kernel<7>, grid, dim3(256), 0, s, x, w, bias, out, Cout, H, W, ntr, ntc, relu, clk);
  else if (KS == 5) hipLaunchKernelGGL(conv_1in_kernel<5>, grid, dim3(256), 0, s, x, w, bias, out, Cout, H, W, ntr, ntc, relu, clk);
  else hipLaunchKernelGGL(conv_1in_kernel<3>, grid, dim3(256), 0, s, x, w, bias, out, Cout, H, W, ntr, ntc, relu, clk);
  return finish_launch("fsmi_conv2d_1in");
}

extern "C" int fsmi_pool2x(const float* x, float* out, int B, int C, int H, int W, void* stream) {
  FSMI_CHECK_ARG(x && out, "fsmi_pool2x: null pointer");
  FSMI_CHECK_ARG(B > 0 && C > 0 && H > 0 && W > 0, "fsmi_pool2x: bad shape");
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_RESIZE, s);
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const long long n = static_cast<long long>(B) * C * Ho * Wo;
  hipLaunchKernelGGL(pool2x_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, s, x, out, H, W, Ho, Wo, n,
                     clock_slot(FSMI_K_RESIZE, s, 4ll * ceil_div(n, 256), "pool2x", true));
  return finish_launch("fsmi_pool2x");
}

extern "C" int fsmi_resize_bilinear(const float* x, float* out, int B, int C, int Hi, int Wi, int Ho, int Wo,
                                    void* stream) {
  FSMI_CHECK_ARG(x && out, "fsmi_resize_bilinear: null pointer");
  FSMI_CHECK_ARG(B > 0 && C > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0, "fsmi_resize_bilinear: bad shape");
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_RESIZE, s);
  const float sh = Ho > 1 ? static_cast<float>(Hi - 1) / static_cast<float>(Ho - 1) : 0.f;
  const float sw = Wo > 1 ? static_cast<float>(Wi - 1) / static_cast<float>(Wo - 1) : 0.f;
  const long long planes = static_cast<long long>(B) * C;
  const long long n = planes * Ho * Wo;
  hipLaunchKernelGGL(resize_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, x, out, planes,
                     Hi, Wi, Ho, Wo, sh, sw, clock_slot(FSMI_K_RESIZE, s, 4ll * ((n + 255) / 256), "resize", true));
  return finish_launch("fsmi_resize_bilinear");
}

extern "C" int fsmi_conv3x3_cout1(const float* x, int Cin, const float* w, const float* bias, const float* res,
                                  long long res_bstride, float* out, long long out_bstride, int B, int H, int W,
                                  void* stream) {
  FSMI_CHECK_ARG(x && w && out, "fsmi_conv3x3_cout1: null pointer");
  FSMI_CHECK_ARG(B > 0 && Cin > 0 && H > 0 && W > 0, "fsmi_conv3x3_cout1: bad shape");
  hipStream_t s = as_stream(stream);
  LaunchTimer t(FSMI_K_CONV2D, s);
  const int ntr = (H + C1O_TR - 1) / C1O_TR, ntc = (W + C1O_TC - 1) / C1O_TC;
  const unsigned nb = static_cast<unsigned>(B) * ntr * ntc;
  hipLaunchKernelGGL(conv3x3_cout1_kernel, dim3(nb), dim3(256), 0, s, x, w, bias, res, res_bstride, out, out_bstride,
                     Cin, H, W, ntr, ntc, clock_slot(FSMI_K_CONV2D, s, 4ll * nb, "conv3x3_cout1", true));
  return finish_launch("fsmi_conv3x3_cout1");
}
