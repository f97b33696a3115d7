/*
 * fsmi.h -- C ABI of libfsmi.so, the MI355X-native (gfx950) hot path of
 * FoundationStereo: cost-volume build, geometry encoding, per-iteration
 * correlation lookup, soft-argmin, convex upsampling and ConvGRU gates.
 *
 * Conventions (every entry point):
 *   - all tensors are fp32, contiguous, row-major, already resident in device
 *     memory (HBM); pointers are device pointers, shapes are plain ints;
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream);
 *     launches are asynchronous on that stream, nothing allocates, nothing
 *     synchronises, so every call is hipGraph-capturable;
 *   - return 0 on success, FSMI_ERR_ARG (1001) when an argument violates the
 *     contract (message in fsmi_last_error()), or the hipError_t of a failed
 *     launch.
 *
 * Reference interfaces replaced are cited as path:line in TongZhe2016/
 * FoundationStereo (snapshot 2025-06-29).  See INTEGRATION.md for bindings.
 */
#ifndef FSMI_H_
#define FSMI_H_

#ifdef __cplusplus
extern "C" {
#endif

#define FSMI_OK 0
#define FSMI_ERR_ARG 1001
#define FSMI_MAX_LEVELS 4

/* ---- library ---------------------------------------------------------- */
int fsmi_version(void);                /* 100*major + minor */
const char* fsmi_last_error(void);     /* thread-local, "" when none */
const char* fsmi_arch(void);           /* "gfx950" */

/* ---- a1: group-wise correlation volume --------------------------------
 * replaces build_gwc_volume / groupwise_correlation, core/submodule.py:388-412
 * fl, fr: (B,C,H,W); out: (B,G,D,H,W).  out[b,g,d,h,w] = <nL,nR(w-d)> over
 * the C/G channels of group g after L2 normalisation (eps 1e-12), 0 for w<d.
 * Requires C % G == 0 (reference: AssertionError at core/submodule.py:390). */
int fsmi_gwc_volume(const float* fl, const float* fr, float* out,
                    int B, int C, int G, int D, int H, int W, void* stream);

/* ---- a2: concat volume -------------------------------------------------
 * replaces build_concat_volume, core/submodule.py:416-427
 * pl, pr: (B,C,H,W); out: (B,2C,D,H,W): left half copied for all w, right
 * half shifted by d and zero for w<d. */
int fsmi_concat_volume(const float* pl, const float* pr, float* out,
                       int B, int C, int D, int H, int W, void* stream);

/* ---- a1+a2+corr_stem[0] fused ------------------------------------------
 * replaces core/foundation_stereo.py:207-213 up to and including the
 * 1x1x1 Conv3d(32 -> Cs) of corr_stem (core/foundation_stereo.py:165):
 *   out[b,o,d,h,w] = A[b,o,h,w] + [w>=d] Bm[b,o,h,w-d] + sum_g Wg[o,g] gwc[b,g,d,h,w]
 * where A, Bm: (B,Cs,H,W) are the proj_cmb features already multiplied by the
 * concat columns of the stem weight (A also carries the stem bias), and
 * Wg: (Cs,G) the gwc columns.  out: (B,Cs,D,H,W).  gwc_ws: optional
 * (B,G,D,H,W) scratch; with it the build runs as two streaming passes (gwc
 * tile kernel, then the stem stream), without it as one LDS-staged kernel. */
int fsmi_comb_volume_stem(const float* fl, const float* fr, const float* A, const float* Bm,
                          const float* Wg, float* gwc_ws, float* out,
                          int B, int C, int G, int Cs, int D, int H, int W, void* stream);

/* pointwise 2-output projection used to form A / Bm above:
 * out[b,o,h,w] = bias[o] + sum_c Wt[o,c] x[b,c,h,w];  x: (B,C,H,W), out: (B,O,H,W) */
int fsmi_pointwise_proj(const float* x, const float* Wt, const float* bias, float* out,
                        int B, int C, int O, int H, int W, void* stream);

/* ---- a5: all-pairs correlation + W2 pyramid (fp32 MFMA) ----------------
 * replaces Combined_Geo_Encoding_Volume.corr + its avg-pool pyramid,
 * core/geometry.py:24-40,68-77.  fl, fr: (B,C,H,W).  levels[i]: (B,H,W,W>>i')
 * with W_i = floor(W_{i-1}/2); level 0 is the full (B,H,W1,W2) correlation of
 * the channel-L2-normalised features.  ws: optional 2*B*C*H*W-float scratch;
 * with it the features are normalised once and the MFMA pass reads them
 * straight from L2, without it one LDS-staged kernel normalises per block. */
int fsmi_allpairs_corr(const float* fl, const float* fr, float* const* levels, int num_levels,
                       int B, int C, int H, int W, float* ws, void* stream);

/* ---- a5: filtered-volume pyramid over D ---------------------------------
 * replaces core/geometry.py:29,34-36 without the permute copy.  vol:
 * (B,Cv,D,H,W) native layout; levels[i-1]: (B,Cv,D_i,H,W), i=1..num_levels-1,
 * D_i = floor(D_{i-1}/2), value = mean of the two parents (iterated). */
int fsmi_volume_pyramid(const float* vol, float* const* levels, int num_levels,
                        int B, int Cv, int D, int H, int W, void* stream);

/* ---- a6: per-iteration multi-level lookup ------------------------------
 * replaces Combined_Geo_Encoding_Volume.__call__ + bilinear_sampler,
 * core/geometry.py:43-65, core/utils/utils.py:44-55.
 * vol_levels[i]: (B,Cv,D_i,H,W); corr_levels[i]: (B,H,W,W2_i); disp: (B,1,H,W);
 * out: (B, L*(2r+1)*(Cv+1), H, W) with channel order per level
 * [geo (c*(2r+1)+k) ..., corr k ...] (core/geometry.py:62-65).
 * Taps at x = disp/2^i + k and x = w/2^i - disp/2^i + k, k in [-r,r]; linear
 * interpolation, align_corners=True, zero padding.  Requires D_i >= 2, W2_i >= 2. */
int fsmi_geo_lookup(const float* const* vol_levels, const float* const* corr_levels,
                    const float* disp, float* out,
                    int num_levels, int radius, int B, int Cv, int D, int H, int W, int W2,
                    void* stream);
/* the same with the reference's `coords` argument (core/geometry.py:43,57): coords (B,H,W) fp32, the
 * column coordinate of each pixel on the left image (core/foundation_stereo.py:231 passes arange(W)
 * per row), so the corr taps sit at x = coords/2^i - disp/2^i + k.  coords == NULL: the pixel column
 * w (what fsmi_geo_lookup does, without the load). */
int fsmi_geo_lookup_coords(const float* const* vol_levels, const float* const* corr_levels,
                           const float* disp, const float* coords, float* out,
                           int num_levels, int radius, int B, int Cv, int D, int H, int W, int W2,
                           void* stream);

/* 1-D stereo specialisation of bilinear_sampler (core/utils/utils.py:44-55):
 * img (P,C,1,Lx); x (P,K) pixel x-coordinates (y == 0); out (P,C,1,K). */
int fsmi_bilinear_sampler_1d(const float* img, const float* x, float* out,
                             int P, int C, int Lx, int K, void* stream);

/* ---- a4: soft-argmin ---------------------------------------------------
 * fsmi_disparity_regression: core/submodule.py:431-435, prob (B,D,H,W) -> (B,1,H,W)
 * fsmi_softmax_regression:  core/foundation_stereo.py:218-220 fused
 *                           (softmax over D of logits, then sum d*p_d). */
int fsmi_disparity_regression(const float* prob, float* out, int B, int D, int H, int W, void* stream);
int fsmi_softmax_regression(const float* logits, float* out, int B, int D, int H, int W, void* stream);

/* ---- a9: convex upsampling ---------------------------------------------
 * fsmi_context_upsample: core/submodule.py:456-468; disp (B,1,h,w),
 *   w (B,9,4h,4w) -> out (B,4h,4w).
 * fsmi_softmax_context_upsample: core/foundation_stereo.py:187-189 fused:
 *   softmax over the 9 logits, scale disp by `scale` (4.0), convex combine. */
int fsmi_context_upsample(const float* disp, const float* w, float* out, int B, int h, int w_, void* stream);
int fsmi_softmax_context_upsample(const float* disp, const float* logits, float* out, float scale,
                                  int B, int h, int w_, void* stream);

/* ---- a7: selective ConvGRU gates (core/update.py:83-119) ----------------
 * zr_s / zr_l: (B, 2*Hd, H, W) pre-activations [z | r] of the small (k=1) and
 * large (k=3) RaftConvGRU; h: (B,Hd,H,W); x: (B,Cx,H,W).
 * fsmi_gru_reset: qin_s/qin_l (B, Hd+Cx, H, W) <- [sigmoid(r)*h , x]   (update.py:92-93)
 * fsmi_gru_blend: hout <- att*((1-zs)h+zs*tanh(qs)) + (1-att)*((1-zl)h+zl*tanh(ql))
 *                 with z = sigmoid(z_pre); q_s/q_l: (B,Hd,H,W); att (B,1,H,W);
 *                 (update.py:91,94-95,117). hout may alias h. */
int fsmi_gru_reset(const float* zr_s, const float* zr_l, const float* h, const float* x,
                   float* qin_s, float* qin_l, int B, int Hd, int Cx, int H, int W, void* stream);
int fsmi_gru_blend(const float* zr_s, const float* zr_l, const float* q_s, const float* q_l,
                   const float* h, const float* att, float* hout,
                   int B, int Hd, int H, int W, void* stream);

/* ---- a3: few-output-channel direct 3D convolution ------------------------
 * replaces the classifier's final nn.Conv3d(14, 1, kernel_size=7, padding=3)
 * (core/foundation_stereo.py:175): x (B,Cin,D,H,W), w (Cout,Cin,KS,KS,KS),
 * bias (Cout) or NULL -> out (B,Cout,D,H,W); stride 1, zero padding KS/2.
 * Supported (KS, Cout): (7,1), (3,1). */
int fsmi_conv3d_direct(const float* x, const float* w, const float* bias, float* out,
                       int B, int Cin, int Cout, int KS, int D, int H, int W, void* stream);

/* Convolution of the refinement loop, halo-tiled split-precision MFMA.
 * replaces the nn.Conv2d / nn.Linear stacks of the refinement loop
 * (core/update.py:20-159: motion encoder, SelectiveConvGRU convs, DispHead,
 * mask head) plus the elementwise passes that follow them.
 * Input: nseg NCHW channel segments concatenated along C (zero-copy cat):
 *   segment i = seg_ch[i] channels starting at seg_ptr[i] inside a tensor with
 *   seg_ctot[i] channels per image (batch stride seg_ctot[i]*H*W).
 * out[b, co0+co] (tensor with out_ctot channels) =
 *   res[b,co] + gamma[co] * alpha * act(conv + bias[co]);  act 0 none, 1 ReLU, 2 GELU(erf),
 *   6 LeakyReLU 0.01; gamma/res may be NULL (res has res_ctot channels per image).
 *   act 7: out = ReLU(conv + bias[co] + res[b,co]) (res required, gamma NULL, alpha 1): the
 *   remaining input channels of a conv whose loop-invariant channels were convolved once
 *   into res (SelectiveConvGRU.conv0's context segment, core/update.py:112-113).
 * Split-precision operands on the fp16 MFMA ("3 x fp16"): x = hi + lo (two fp16),
 * product = hi*hi + hi*lo + lo*hi accumulated in fp32 (~22-bit operands).  whi/wlo:
 * _Float16 weights packed [KS*KS][Cin32/32][Cout32][32] (Cin32/Cout32 = Cin/Cout rounded
 * up to 32, zero padded).  Square KS in {1, 3}.  Range-safe split: each output channel's weights are packed
 * x 2^wexp[co] (its max |w| in [1, 2)); scale_bias (2*Cout floats, device, 8-B
 * aligned) holds the pairs (2^-wexp[co], bias[co]) the epilogue applies as
 * conv * scale + bias; activations get a block exponent per 32-channel chunk in the
 * kernel (conv_halo.h, chunk_exp), so neither overflows fp16 nor loses its low
 * half to fp16 subnormals.  A block stages a (rows+2)x34 input halo once per
 * 32-channel chunk and runs all taps from LDS.  Inner segments must hold a
 * multiple of 8 channels.  cfg 0: 64 couts x 8x32 px, 1: 128 couts x 4x32 px
 * (weights staged per tap through LDS); 2 / 3: the same tiles with each wave's
 * weight fragments loaded into registers one tap ahead; 4: 128 couts x 2x32 px,
 * 5: 64 couts x 4x32 px (registers, one pixel fragment per wave: 3 waves/SIMD);
 * 8: 128 couts x 8x32 px, 9: 256 couts x 4x32 px (registers, 2x4 fragments per wave);
 * 16 + c (c in 3, 4, 5, 7): tile c with two K groups -- 512-thread blocks whose two wave
 * groups take alternate 32-channel chunks and sum through LDS (split-K inside the block);
 * -1: measured default.
 * nsplit: split-K over 32-channel chunks (<0: auto, sized to fill the chip);
 * partial sums go to ws (nsplit*B*Cout*H*W floats, ws_floats available) and
 * a second kernel sums them in split order (deterministic) and applies the
 * epilogue.  ws may be NULL when nsplit is 0/1 (or auto: then no split).
 * (A last-arriving-block fixup inside the conv kernel was measured 4x slower:
 * the agent-scope fences it needs flush and invalidate the per-XCD L2.) */
/* Launches of the halo / pointwise / depth conv tiles since the last reset, per tile config as
 * launched: counts[c] for c < n (n <= 64): 0..9 and 11 register / LDS tiles, 10 stride-2 tiles,
 * 16 + c K-group tiles, 24..29 pointwise tiles, 30 the depth-blocked (17,1,1) tile, 32 + c the
 * pipelined variant of tile c.  reset != 0 zeroes them after the read.  (Which tile the tuning table
 * or the policy picked for a layer, checked by tests.) */
int fsmi_conv_launch_counts(long long* counts, int n, int reset);

/* Debug: while buf != NULL, every halo-conv launch stores per-block wall-clock
 * stamps (100 MHz) into buf[block*40 + 0..39]: start, each chunk's staging
 * barrier, before/after the epilogue, (chunks << 32 | block).  NULL disables. */
int fsmi_debug_conv_timestamps(unsigned long long* buf);

int fsmi_conv2d_halo_x3(const float* const* seg_ptr, const int* seg_ch, const int* seg_ctot, int nseg,
                        const void* whi, const void* wlo, const float* scale_bias, const float* gamma,
                        const float* res, int res_ctot, float* out, int out_ctot, int co0, int B, int Cout,
                        int KS, int H, int W, int act, float alpha, int cfg, int nsplit, float* ws,
                        long long ws_floats, void* stream);

/* The same halo conv with a SelectiveConvGRU gate as its epilogue (replaces
 * the gate elementwise passes of core/update.py:88-95,117; Hd = hidden channels,
 * h / z / rh / out (B,Hd,H,W), att (B,1,H,W), all written/read in place):
 *   mode 0 (convz|convr stacked, Cout = 2Hd): z = sigmoid(conv[:Hd]),
 *          rh = sigmoid(conv[Hd:]) * h   (rh then feeds convq as a segment beside x);
 *   mode 1 (small GRU convq, Cout = Hd): out[:, co0:] = ((1-z)h + z tanh(conv)) * att;
 *   mode 2 (large GRU convq):            out[:, co0:] += ((1-z)h + z tanh(conv)) * (1-att).
 * conv includes the bias.  Other arguments as fsmi_conv2d_halo_x3. */
int fsmi_conv2d_halo_x3_gate(const float* const* seg_ptr, const int* seg_ch, const int* seg_ctot, int nseg,
                             const void* whi, const void* wlo, const float* scale_bias, int mode,
                             const float* h, float* z, const float* att, float* rh, int Hd, float* out,
                             int out_ctot, int co0, int B, int Cout, int KS, int H, int W, int cfg, int nsplit,
                             float* ws, long long ws_floats, void* stream);

/* ---- a3: 3D cost filtering (stride-1 Conv3d + folded BatchNorm) ----------
 * replaces the stride-1 Conv3d+BN(+act) layers of core/submodule.py:51-195
 * (BasicConv, Conv3dNormActReduced, ResnetBasicBlock3D) on MIOpen.  The same
 * halo split-precision kernel: a KD x KS x KS conv (KS in {1,3}, KD odd, zero
 * padding KD/2, KS/2) is the sum over kd of 2D convs on depth plane d+kd-KD/2.
 * x (B,Cin,D,H,W), out / res (B,Cout,D,H,W); whi/wlo packed as for
 * fsmi_conv2d_halo_x3 with taps = (kd, kh, kw), kd major; bias = folded conv bias +
 * BatchNorm shift.  out = act(conv + bias) + res, or with res_pre
 * act(conv + bias + res); act 0 none, 1 ReLU, 6 LeakyReLU(0.01).
 * cfg as fsmi_conv2d_halo_x3 plus 6: 32 couts x 8x32 px, 7: 32 x 4x32. */
int fsmi_conv3d_halo_x3(const float* x, int Cin, const void* whi, const void* wlo, const float* scale_bias,
                        const float* res, float* out, int B, int Cout, int D, int H, int W, int KD, int KS,
                        int act, int res_pre, int cfg, int nsplit, float* ws, long long ws_floats, void* stream);

/* ---- a3: stride-2 Conv3d and the fused FeatureAtt gate ----------------------
 * fsmi_conv3d_halo_x3 with two more terms:
 *   stride 2: the hourglass BasicConv(is_3d, kernel_size=3, stride=2, padding=1) + BN + LeakyReLU
 *     (core/foundation_stereo.py:50-58), and with D = KD = 1 the context net's 3x3 s2 p1 convs and
 *     1x1 s2 projections (core/extractor.py:20-80): KS, KD in {1, 3} with padding KS/2, KD/2;
 *     D, H, W are the INPUT's, out / res are (B, Cout, (D-1)/2+1, (H-1)/2+1, (W-1)/2+1); cfg -1 or
 *     the stride-2 tiles 4 (128 couts x 2x32 px), 5 (64 x 4x32), 7 (32 x 4x32), 10 (64 x 2x32).
 *   res_pre needs a volume (D or KD > 1) or stride 2 (FSMI_ERR_ARG otherwise).
 *   fatt: FeatureAtt (core/submodule.py:438-454) folded into the epilogue -- the final value of
 *     output channel co at (d, h, w) is multiplied by sigmoid(fatt[b, co, h, w]); fatt is the
 *     gate's pre-sigmoid (B, Cout, Ho, Wo) map (contiguous) or NULL. */
int fsmi_conv3d_halo_x3_ex(const float* x, int Cin, const void* whi, const void* wlo, const float* scale_bias,
                           const float* res, const float* fatt, float* out, int B, int Cout, int D, int H, int W,
                           int KD, int KS, int stride, int act, int res_pre, int cfg, int nsplit, float* ws,
                           long long ws_floats, void* stream);

/* ---- refinement-loop auxiliaries ---------------------------------------
 * fsmi_dwconv2d: depthwise KSxKS conv (KS in {3,5,7}, stride 1, zero pad KS/2)
 *   x, out (B,C,H,W); w (C,1,KS,KS); bias (C) or NULL.  Replaces the EdgeNeXt
 *   dwconv of DispHead (core/submodule.py:565-591 via core/update.py:24-31).
 * fsmi_resize_bilinear: F.interpolate(x, (Ho,Wo), mode="bilinear",
 *   align_corners=True) on (B,C,Hi,Wi) -> (B,C,Ho,Wo) (interp, core/update.py:80). */
/* ---- a3: ConvTranspose3d(k=4, s=2, p=1) + folded BatchNorm + activation -------------
 * replaces the hourglass *_up BasicConv(deconv=True, is_3d=True), core/foundation_stereo.py:62-68
 * with core/submodule.py:51-86: x (B,Cin,D,H,W) -> out (B,Cout,2D,2H,2W).  Output phase
 * p = 4*pd + 2*ph + pw (voxels (2d+pd, 2h+ph, 2w+pw)) is a 2x2x2 stride-1 conv over x:
 * whi[p] / wlo[p] packed as fsmi_conv3d_halo_x3's weights (KD = KS = 2, taps at input offsets
 * {-1, 0} for phase 0 and {0, +1} for phase 1 of each dimension; ops.pack_deconv_phases),
 * scale_bias[p] its (2^-wexp, bias) pairs.  act 0 none / 1 ReLU / 6 LeakyReLU(0.01); cfg tile
 * (2, 3, 5, 6, 7) or -1. */
int fsmi_conv3d_up2_halo_x3(const float* x, int Cin, const void* const* whi, const void* const* wlo,
                            const float* const* scale_bias, float* out, int B, int Cout, int D, int H, int W,
                            int act, int cfg, void* stream);
/* ConvTranspose2d(k=4, s=2, p=1) (+ bias / folded BN, activation 0 / 1 ReLU / 6 LeakyReLU) on 2x2
 * phase tiles: x (B,Cin,H,W) -> out (B,Cout,2H,2W); whi / wlo / scale_bias: the 4 phase packs
 * (phase p = 2*oh + ow writes output pixels (2h + oh, 2w + ow)).  Replaces the spx upsampling
 * deconvs spx_2_gru.conv1 and spx_gru (core/foundation_stereo.py:183-191, core/submodule.py:281-317). */
int fsmi_conv2d_up2_halo_x3(const float* x, int Cin, const void* const* whi, const void* const* wlo,
                            const float* const* scale_bias, float* out, int B, int Cout, int H, int W,
                            int act, int cfg, void* stream);

int fsmi_dwconv2d(const float* x, const float* w, const float* bias, float* out, int B, int C, int KS,
                  int H, int W, void* stream);
/* fsmi_edgenext_mlp: the inverted-bottleneck MLP of EdgeNextConvEncoder (core/submodule.py:583-590,
 *   replacing pwconv1 -> GELU -> pwconv2 -> gamma -> residual):
 *   out[b,:,p] = res[b,:,p] + gamma * (W2 gelu(W1 x[b,:,p] + b1) + b2), x / res / out (B,C,H,W)
 *   (out may alias res, not x); w1hi/w1lo = ops.PackedConv of W1 (E x C) as a 1x1 conv,
 *   sb1 its (2^-wexp, b1) pairs (E float2), w2hi/w2lo / sb2 the same for W2 (C x E); gamma (C) or
 *   NULL.  Split-precision MFMA (3 fp16 products per MAC) with fp32 accumulation; the 4C hidden
 *   map stays in LDS.  Built for C = 128, E = 4C (DispHead). */
int fsmi_edgenext_mlp(const float* x, const float* res, float* out, const void* w1hi, const void* w1lo,
                      const float* sb1, const void* w2hi, const void* w2lo, const float* sb2, const float* gamma,
                      int B, int C, int E, int H, int W, void* stream);
int fsmi_resize_bilinear(const float* x, float* out, int B, int C, int Hi, int Wi, int Ho, int Wo, void* stream);
/* fsmi_conv3x3_cout1: Conv2d(Cin, 1, 3, padding=1) + bias (+ res) in fp32 on (B,Cin,H,W) (dense NCHW):
 * out[b*out_bstride + p] = res[b*res_bstride + p] + bias[0] + sum_c,tap w[c*9 + tap] * x[b, c, p + tap];
 * bias (device, 1 float) and res may be NULL.  DispHead's last layer (core/update.py:28), whose caller adds disp (the loop's
 * disp + delta, core/foundation_stereo.py:240-241) and writes it into the next motion-feature buffer. */
int fsmi_conv3x3_cout1(const float* x, int Cin, const float* w, const float* bias, const float* res, long long res_bstride,
                       float* out, long long out_bstride, int B, int H, int W, void* stream);

/* fsmi_conv2d_1in: Conv2d(1, Cout, KS, padding=KS//2) (+ ReLU when relu != 0) on (B,1,H,W) ->
 *   (B,Cout,H,W): the motion encoder's convd1 + ReLU (core/update.py:57,67); KS in {3,5,7}. */
int fsmi_conv2d_1in(const float* x, const float* w, const float* bias, float* out, int B, int Cout, int KS,
                    int H, int W, int relu, void* stream);
/* fsmi_pool2x: F.avg_pool2d(x, 3, stride=2, padding=1) (count_include_pad) on (B,C,H,W) ->
 *   (B,C,(H-1)/2+1,(W-1)/2+1): pool2x, core/update.py:72-73. */
int fsmi_pool2x(const float* x, float* out, int B, int C, int H, int W, void* stream);

/* ---- disparity transformer of the hourglass ---------
 * fsmi_dt_patch_embed: conv_patch = depthwise Conv3d(C, C, 4, stride 4) + eval
 *   BatchNorm3d (core/foundation_stereo.py:85-88) with bias and BN folded into
 *   per-channel scale / shift; x (B,C,D,H,W) -> out (B,C,D/4,H/4,W/4); w (C,4,4,4).
 * fsmi_disparity_transformer: CostVolumeDisparityAttention.forward
 *   (core/submodule.py:506-528): tokens = the L disparities of each (b,h,w),
 *   x + pe[:L], then nlayers post-norm encoder layers (core/submodule.py:233-257;
 *   attention = FlashMultiheadAttention, :198-229, non-causal, scale 1/sqrt(C/nheads),
 *   FFN with exact GELU, LayerNorm eps).  x, out (B,C,L,HW) NCDHW; pe (L,C);
 *   params = nlayers x fsmi_dt_layer_floats() floats, each layer
 *   [Wq bq Wk bk Wv bv Wo bo ln1.w ln1.b W1 b1 W2 b2 ln2.w ln2.b] (Linear weights
 *   (out,in) row-major).  Built for C=28, 4 heads, FFN 28, L <= 64.
 * fsmi_upsample4_add: vol (B,C,4D,4H,4W) += F.interpolate(t, scale_factor=4,
 *   mode="trilinear", align_corners=False) of t (B,C,D,H,W)
 *   (core/foundation_stereo.py:119-120). */
int fsmi_dt_layer_floats(void);
int fsmi_dt_patch_embed(const float* x, const float* w, const float* scale, const float* shift, float* out,
                        int B, int C, int D, int H, int W, void* stream);
int fsmi_disparity_transformer(const float* x, float* out, const float* params, const float* pe, int B, int C,
                               int L, int HW, int nheads, int ffdim, int nlayers, float eps, void* stream);
int fsmi_upsample4_add(const float* t, float* vol, int B, int C, int D, int H, int W, void* stream);

/* ---- backbone: DepthAnythingV2 ViT + DPT, EdgeNeXt-S, Feature fusion --------
 * replaces Feature / DepthAnythingFeature (core/extractor.py:286-369), the DINOv2 ViT
 * (dinov2/dinov2/models/vision_transformer.py, layers/{attention,block,patch_embed}.py), the DPT head
 * (depth_anything/dpt.py:24-190, depth_anything/blocks.py) and timm's edgenext_small (core/extractor.py:327).
 * The ViT runs on the channel-major token layout (B, C, Tp): token t of channel c at c*Tp + t, the N patch
 * tokens first, the class token at N, zero padding up to Tp; every Linear is then a 1x1 conv of
 * fsmi_conv2d_halo_x3 over a (Tp/32) x 32 "image".
 * fsmi_channel_layernorm: nn.LayerNorm over channels per token (eps), x (B,C,Tx) -> out (B,C,To), tokens
 *   [0, n) (n <= Tx, To); w / b (C) or NULL.  Also LayerNorm2d / channels-last LayerNorm of NCHW maps
 *   (Tx = To = n = H*W).
 * fsmi_vit_attention: softmax(q k^T * scale) v per head (layers/attention.py:69-79): qkv (B, 3*heads*64, Tp)
 *   = [q; k; v] channel-major, out (B, heads*64, Tp); keys >= T masked; head_dim 64; Tp % 64 == 0.
 *   Split-precision MFMA (3 fp16 products per MAC), fp32 softmax.  ws: fsmi_vit_attention_ws_floats(B, heads,
 *   T, Tp) floats (0: NULL allowed) for the key-range partials when the keys are split over several blocks.
 * fsmi_space_to_depth: out[b, (c*k+ky)*k+kx, y, x] = x[b, c, y*k+ky, x*k+kx] (B,C,H,W) -> (B,C*k*k,H/k,W/k):
 *   the im2col of a conv with stride == kernel (patch embed k14, EdgeNeXt stem k4 / downsample k2).
 * fsmi_depth_to_space: out[b, c, y*k+ky, x*k+kx] = x[b, (ky*k+kx)*C + c, y, x]: a ConvTranspose2d with
 *   stride == kernel (DPT resize_layers[0..1]) after its 1x1-conv form.
 * fsmi_vit_tokens: out[b,c,t] = (emb[b,c,t] for t < N | cls[c] for t == N | 0) + pos[c,t] (pos (C,Tp), zero
 *   past N): prepare_tokens_with_masks (vision_transformer.py:214-233) in the layout above.
 * fsmi_resize_bicubic: F.interpolate(mode="bicubic", align_corners=False), A = -0.75, border-clamped taps
 *   (core/extractor.py:352).
 * fsmi_instance_norm: out = act2(act1(InstanceNorm(x)) + res) per plane (planes = B*C, biased variance, no
 *   affine), res may be NULL; act 0 none, 1 ReLU, 6 LeakyReLU(0.01) (core/submodule.py:320-385,
 *   core/extractor.py:20-80 with norm 'instance').
 * fsmi_elementwise: op 0 a+b, 1 relu(a), 2 relu(a+b), 3 a*b; b indexed modulo bper when bper > 0.
 * fsmi_xca: EdgeNeXt cross-covariance attention core (timm CrossCovarianceAttn): qkv (B,3C,N) channel-major,
 *   temperature (heads), ws (fsmi_xca_workspace_floats(B, C, heads) floats: the softmaxed maps, then the
 *   per-split Gram partials), out (B,C,N); C/heads <= 40.
 * fsmi_dwconv2d_ex: fsmi_dwconv2d on channel slices (x / add / out planes at (b*ctot + c)*H*W), KS in
 *   {3,5,7,9}, with add (or NULL) summed into the input first. */
int fsmi_channel_layernorm(const float* x, float* out, const float* w, const float* b, int B, int C, int Tx, int To,
                           int n, float eps, void* stream);
int fsmi_vit_attention(const float* qkv, float* out, int B, int heads, int head_dim, int T, int Tp, float scale,
                       float* ws, long long ws_floats, void* stream);
long long fsmi_vit_attention_ws_floats(int B, int heads, int T, int Tp);
int fsmi_space_to_depth(const float* x, float* out, int B, int C, int H, int W, int k, void* stream);
int fsmi_depth_to_space(const float* x, float* out, int B, int C, int H, int W, int k, void* stream);
int fsmi_vit_tokens(const float* emb, const float* cls, const float* pos, float* out, int B, int C, int N, int Tp,
                    void* stream);
int fsmi_resize_bicubic(const float* x, float* out, int B, int C, int Hi, int Wi, int Ho, int Wo, void* stream);
int fsmi_instance_norm(const float* x, const float* res, float* out, int planes, int HW, float eps, int act1, int act2,
                       void* stream);
int fsmi_elementwise(const float* a, const float* b, float* out, long long n, long long bper, int op, void* stream);
int fsmi_xca(const float* qkv, const float* temperature, float* ws, float* out, int B, int C, int heads, int N,
             void* stream);
long long fsmi_xca_workspace_floats(int B, int C, int heads);
int fsmi_dwconv2d_ex(const float* x, int x_ctot, const float* add, int add_ctot, const float* w, const float* bias,
                     float* out, int out_ctot, int B, int C, int KS, int H, int W, void* stream);

/* ---- live kernel timing (bench.py roofline) -----------------------------
 * When enabled, every launch of the kernels below is bracketed by a pair of
 * hipEvents recorded on the launch stream (skipped while the stream is being
 * captured).  fsmi_timer_query synchronises those events and returns the
 * summed duration and launch count since the last reset. */
enum {
  FSMI_K_GWC = 0, FSMI_K_CONCAT, FSMI_K_COMB, FSMI_K_PROJ, FSMI_K_CORR, FSMI_K_VOLPYR,
  FSMI_K_LOOKUP, FSMI_K_SAMPLER, FSMI_K_REG, FSMI_K_UPSAMPLE, FSMI_K_GRU_RESET, FSMI_K_GRU_BLEND,
  FSMI_K_CONV3D, FSMI_K_CONV2D, FSMI_K_DWCONV, FSMI_K_RESIZE, FSMI_K_DT, FSMI_K_NORM, FSMI_K_COUNT
};
/* Range guard of the split-precision convs: a block scales its activations by a power of two
 * fixed from its first 32-channel chunk (8 bits of headroom); a later value that would still
 * leave fp16's range sets a host-mapped flag instead of silently becoming inf.  *overflowed =
 * the flag (1 once any conv since the last reset overflowed); reset != 0 clears it.  The flag
 * is written asynchronously: synchronise the streams that ran the convs before reading it. */
int fsmi_range_status(int reset, int* overflowed);
/* Safe range mode: while set, every split-precision 2D conv launched (or captured) afterwards takes
 * a per-chunk block exponent with exact accumulator rescaling (the volumes' mode), which cannot
 * overflow; ~3 % slower.  FoundationStereo.forward switches it on and re-runs a forward whose
 * range flag came back set (the reference has no such mode: its convs are fp32 / fp16 autocast,
 * core/update.py:83-159).  Sticky until cleared. */
int fsmi_set_range_safe(int safe);
/* Fill out[0..n) with NaN on `stream` when the range flag is set (a device-side check, no host
 * synchronisation): FoundationStereo.forward appends it to a CAPTURED forward, so a graph replay
 * whose convs overflowed returns NaN, never a silently wrong disparity. */
int fsmi_range_poison(float* out, long long n, void* stream);
int fsmi_get_range_safe(int* safe);

/* on: 0 off, 1 on (events + kernel clocks outside stream capture), 2 also the kernel clocks of
 * launches captured into a hipGraph (their stamps are rewritten by every replay: a query after the
 * replays reads the last replay's launches -- bench.py's in-step lookup timing), 3 as 2 with every
 * instrumented kernel clocked, not only the geometry kernels (fsmi_timer_dump_captured). */
int fsmi_timer_enable(int on);
int fsmi_timer_reset(void);
int fsmi_timer_query(int kernel, double* total_ms, long long* count);
/* Same launches timed by the kernels themselves (lookup, cost-volume build, all-pairs correlation
 * and its normalisation, volume pyramid): each
 * instrumented launch records its first block start and last wave end (stores acknowledged) in
 * s_memrealtime ticks; returns the summed durations -- execution time without the latency of
 * the event records around the launch. */
int fsmi_timer_query_clock(int kernel, double* total_ms, long long* count);
/* The same over the launches captured into hipGraphs while timing was in mode 2: their stamps hold
 * the last replay of each graph.  Kept across fsmi_timer_reset / fsmi_timer_enable (the graphs keep
 * writing their slots) until fsmi_timer_release_captured, which the caller may call only once every
 * graph captured in mode 2 is destroyed (their slots are then handed out again).  Either query fails
 * (FSMI_ERR_ARG) when a launch of the kernel found the clock arena full (16M stamps; 64M in timer mode 3). */
int fsmi_timer_query_clock_captured(int kernel, double* total_ms, long long* count);
int fsmi_timer_release_captured(void);
/* The replay's timeline: one text line per launch captured in timer mode 2, in capture order,
 * "<kernel id> <stream> <first wave start> <last wave end> <tag>" (s_memrealtime ticks, 100 MHz;
 * 0 0 for a launch no replay has run).  Writes at most size bytes (NUL-terminated); *needed = the
 * full length + 1.  Instrumented: the halo / pointwise conv kernels and their split-K reduce, the
 * EdgeNeXt MLP, depthwise / 1-input convs, pool / resize, and the geometry kernels. */
int fsmi_timer_dump_captured(char* buf, long long size, long long* needed);
/* The number of lines fsmi_timer_dump_captured would print so far (launches captured with clocks),
 * without touching the device: callable while a capture is in progress (positions a cross-stream wait
 * among the captured launches; tools/replay_timeline.py). */
int fsmi_timer_captured_count(long long* n);
/* Re-issue the last timed launch of `kernel` (lookup, cost-volume build) `reps` times back to
 * back on its stream between two hipEvents; *avg_ms = span / reps.  The kernels are pure
 * functions of their inputs, so the replays rewrite identical outputs.
 * Lifetime contract: the replay reuses the raw device pointers of the recorded launch, so the
 * CALLER must keep every input and output buffer of that launch allocated until the replay has
 * finished (ops.py holds references to the last timed launch's tensors until the next
 * fsmi_timer_reset / fsmi_timer_enable, which also drop the recorded launch). */
int fsmi_timer_replay(int kernel, int reps, double* avg_ms);

#ifdef __cplusplus
}
#endif
#endif /* FSMI_H_ */
