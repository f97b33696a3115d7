"""Torch-tensor front end of the HIP hot path (libfsmi.so, include/fsmi.h).

Each op takes ROCm-resident fp32 tensors, allocates its output through the
PyTorch caching allocator, and launches on the current HIP stream -- no host
synchronisation, so a whole refinement loop can be captured in a hipGraph.
There is no CPU path: CPU tensors raise (the CPU restatement lives in the
test-only ``oracle`` package).  The ops are inference-only (the reference's
training backprop is out of scope): inputs that require grad
while grad mode is on raise.
"""
from __future__ import annotations

from typing import List, Sequence

import json
import os

import torch

from . import _lib

Tensor = torch.Tensor


def _stream(t: Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _check(name: str, *ts: Tensor):
    for t in ts:
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"{name}: expected tensors")
        if not t.is_cuda:
            raise RuntimeError(f"{name}: fsmi ops run on ROCm (HIP) device tensors only; got {t.device}")
        if t.dtype != torch.float32:
            raise RuntimeError(f"{name}: expected float32, got {t.dtype}")
        if torch.is_grad_enabled() and t.requires_grad:
            raise RuntimeError(f"{name}: fsmi ops are inference-only (input requires grad)")


def _c(t: Tensor) -> Tensor:
    """Contiguous and 16-byte aligned (the kernels issue float4 accesses)."""
    if t.is_contiguous() and t.data_ptr() % 16 == 0:
        return t
    return t.contiguous() if not t.is_contiguous() else t.clone()


def _p(t: Tensor) -> int:
    return t.data_ptr()


def _overlaps(a: Tensor, b: Tensor) -> bool:
    """Whether the byte ranges a and b span on the same device intersect."""
    if a.device != b.device or a.numel() == 0 or b.numel() == 0:
        return False
    a0, b0 = a.data_ptr(), b.data_ptr()
    a1 = a0 + (sum((n - 1) * st for n, st in zip(a.shape, a.stride())) + 1) * a.element_size()
    b1 = b0 + (sum((n - 1) * st for n, st in zip(b.shape, b.stride())) + 1) * b.element_size()
    return a0 < b1 and b0 < a1


# ---------------------------------------------------------------- cost volume

def gwc_volume(fl: Tensor, fr: Tensor, maxdisp: int, num_groups: int) -> Tensor:
    """core/submodule.py:399-412 -> (B,G,D,H,W)."""
    _check("gwc_volume", fl, fr)
    B, C, H, W = fl.shape
    assert C % num_groups == 0, f"C:{C}, num_groups:{num_groups}"
    fl, fr = _c(fl), _c(fr)
    out = torch.empty((B, num_groups, maxdisp, H, W), device=fl.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_gwc_volume(_p(fl), _p(fr), _p(out), B, C, num_groups, maxdisp, H, W,
                                           _stream(fl)), "gwc_volume")
    return out


def concat_volume(pl: Tensor, pr: Tensor, maxdisp: int) -> Tensor:
    """core/submodule.py:416-427 -> (B,2C,D,H,W)."""
    _check("concat_volume", pl, pr)
    B, C, H, W = pl.shape
    pl, pr = _c(pl), _c(pr)
    out = torch.empty((B, 2 * C, maxdisp, H, W), device=pl.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_concat_volume(_p(pl), _p(pr), _p(out), B, C, maxdisp, H, W, _stream(pl)),
               "concat_volume")
    return out


def pointwise_proj(x: Tensor, wt: Tensor, bias: Tensor = None) -> Tensor:
    """out[b,o] = bias[o] + sum_c wt[o,c] x[b,c]  (1x1 conv)."""
    _check("pointwise_proj", x, wt, *([bias] if bias is not None else []))
    B, C, H, W = x.shape
    O = wt.shape[0]
    x, wt = _c(x), _c(wt)
    out = torch.empty((B, O, H, W), device=x.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_pointwise_proj(_p(x), _p(wt), _p(bias) if bias is not None else None, _p(out),
                                               B, C, O, H, W, _stream(x)), "pointwise_proj")
    return out


def comb_volume_stem(fl: Tensor, fr: Tensor, A: Tensor, Bm: Tensor, Wg: Tensor, maxdisp: int,
                     two_pass: bool = False) -> Tensor:
    """Fused gwc + concat + corr_stem[0] (core/foundation_stereo.py:207-213,165) -> (B,Cs,D,H,W).

    Default: one LDS-staged streaming kernel (no scratch); ``two_pass`` (or
    FSMI_BUILD_TWO_PASS=1): gwc into a (B,G,D,H,W) scratch, then a stem pass."""
    _check("comb_volume_stem", fl, fr, A, Bm, Wg)
    B, C, H, W = fl.shape
    Cs, G = Wg.shape
    assert C % G == 0, f"C:{C}, num_groups:{G}"
    fl, fr, A, Bm, Wg = _c(fl), _c(fr), _c(A), _c(Bm), _c(Wg)
    out = torch.empty((B, Cs, maxdisp, H, W), device=fl.device, dtype=torch.float32)
    two_pass = two_pass or os.environ.get("FSMI_BUILD_TWO_PASS", "0") == "1"
    ws = torch.empty((B, G, maxdisp, H, W), device=fl.device, dtype=torch.float32) if two_pass else None
    _lib.check(_lib.load().fsmi_comb_volume_stem(_p(fl), _p(fr), _p(A), _p(Bm), _p(Wg),
                                                 _p(ws) if ws is not None else None, _p(out), B, C, G, Cs,
                                                 maxdisp, H, W, _stream(fl)), "comb_volume_stem")
    _keep_for_replay("comb", fl, fr, A, Bm, Wg, ws, out)
    return out


# ---------------------------------------------------------------- geometry

def allpairs_corr(fl: Tensor, fr: Tensor, num_levels: int, two_pass: bool = True) -> List[Tensor]:
    """core/geometry.py:24-40,68-77 -> [(B,H,W,W_i)] with W_i = W >> i.

    ``two_pass`` (default): normalise into a scratch, then the barrier-free MFMA
    pass; otherwise one LDS-staged kernel."""
    _check("allpairs_corr", fl, fr)
    B, C, H, W = fl.shape
    fl, fr = _c(fl), _c(fr)
    levels = [torch.empty((B, H, W, W >> i), device=fl.device, dtype=torch.float32) for i in range(num_levels)]
    ws = torch.empty((2, B, C, H, W), device=fl.device, dtype=torch.float32) if two_pass else None
    pp, keep = _lib.ptr_array([_p(t) for t in levels])
    _lib.check(_lib.load().fsmi_allpairs_corr(_p(fl), _p(fr), pp, num_levels, B, C, H, W,
                                              _p(ws) if ws is not None else None, _stream(fl)), "allpairs_corr")
    del keep
    return levels


def volume_pyramid(vol: Tensor, num_levels: int) -> List[Tensor]:
    """core/geometry.py:29,34-36 in the native (B,Cv,D,H,W) layout -> [vol, lvl1, ...]."""
    _check("volume_pyramid", vol)
    B, Cv, D, H, W = vol.shape
    vol = _c(vol)
    levels = [torch.empty((B, Cv, D >> i, H, W), device=vol.device, dtype=torch.float32)
              for i in range(1, num_levels)]
    if levels:
        pp, keep = _lib.ptr_array([_p(t) for t in levels])
        _lib.check(_lib.load().fsmi_volume_pyramid(_p(vol), pp, num_levels, B, Cv, D, H, W, _stream(vol)),
                   "volume_pyramid")
        del keep
    return [vol] + levels


def geo_lookup(vol_levels: Sequence[Tensor], corr_levels: Sequence[Tensor], disp: Tensor, radius: int,
               out: Tensor = None, coords: Tensor = None) -> Tensor:
    """core/geometry.py:43-65 -> (B, L*(2r+1)*(Cv+1), H, W).  ``coords``: the reference's column
    coordinates (any layout with B*H*W elements, e.g. its (B,H,W,1)); None = the pixel column w, which
    is what the reference passes (core/foundation_stereo.py:231)."""
    _check("geo_lookup", disp, *vol_levels, *corr_levels, *([coords] if coords is not None else []))
    L = len(vol_levels)
    B, Cv, D, H, W = vol_levels[0].shape
    W2 = corr_levels[0].shape[-1]
    assert disp.shape == (B, 1, H, W), f"disp {tuple(disp.shape)} vs volume {(B, 1, H, W)}"
    for i in range(L):
        assert vol_levels[i].shape == (B, Cv, D >> i, H, W) and vol_levels[i].is_contiguous()
        assert corr_levels[i].shape == (B, H, W, W2 >> i) and corr_levels[i].is_contiguous()
    disp = _c(disp)
    if coords is not None:
        assert coords.numel() == B * H * W, f"coords {tuple(coords.shape)}: expected B*H*W = {B * H * W} values"
        coords = _c(coords.reshape(B, H, W))
    K = 2 * radius + 1
    if out is None:
        out = torch.empty((B, L * K * (Cv + 1), H, W), device=disp.device, dtype=torch.float32)
    pv, kv = _lib.ptr_array([_p(t) for t in vol_levels])
    pc, kc = _lib.ptr_array([_p(t) for t in corr_levels])
    _lib.check(_lib.load().fsmi_geo_lookup_coords(pv, pc, _p(disp), _p(coords) if coords is not None else None,
                                                  _p(out), L, radius, B, Cv, D, H, W, W2, _stream(disp)),
               "geo_lookup")
    del kv, kc
    _keep_for_replay("lookup", *vol_levels, *corr_levels, disp, out, coords)
    return out


def bilinear_sampler_1d(img: Tensor, x: Tensor) -> Tensor:
    """core/utils/utils.py:44-55 (H == 1): img (P,C,1,Lx), x (P,K) -> (P,C,1,K)."""
    _check("bilinear_sampler", img, x)
    P, C, Hh, Lx = img.shape
    assert Hh == 1
    K = x.shape[-1]
    img, x = _c(img), _c(x.reshape(P, K))
    out = torch.empty((P, C, 1, K), device=img.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_bilinear_sampler_1d(_p(img), _p(x), _p(out), P, C, Lx, K, _stream(img)),
               "bilinear_sampler")
    return out


# ---------------------------------------------------------------- heads

def disparity_regression(prob: Tensor, maxdisp: int) -> Tensor:
    """core/submodule.py:431-435."""
    assert len(prob.shape) == 4
    _check("disparity_regression", prob)
    B, D, H, W = prob.shape
    assert D == maxdisp
    prob = _c(prob)
    out = torch.empty((B, 1, H, W), device=prob.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_disparity_regression(_p(prob), _p(out), B, D, H, W, _stream(prob)),
               "disparity_regression")
    return out


def softmax_regression(logits: Tensor) -> Tensor:
    """softmax over D then disparity_regression (core/foundation_stereo.py:218-220)."""
    _check("softmax_regression", logits)
    B, D, H, W = logits.shape
    logits = _c(logits)
    out = torch.empty((B, 1, H, W), device=logits.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_softmax_regression(_p(logits), _p(out), B, D, H, W, _stream(logits)),
               "softmax_regression")
    return out


def context_upsample(disp_low: Tensor, up_weights: Tensor) -> Tensor:
    """core/submodule.py:456-468 -> (B,4h,4w)."""
    _check("context_upsample", disp_low, up_weights)
    b, c, h, w = disp_low.shape
    assert c == 1 and up_weights.shape == (b, 9, 4 * h, 4 * w)
    disp_low, up_weights = _c(disp_low), _c(up_weights)
    out = torch.empty((b, 4 * h, 4 * w), device=disp_low.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_context_upsample(_p(disp_low), _p(up_weights), _p(out), b, h, w,
                                                 _stream(disp_low)), "context_upsample")
    return out


def softmax_context_upsample(disp_low: Tensor, logits: Tensor, scale: float = 4.0) -> Tensor:
    """softmax(9) + context_upsample(scale*disp) fused (core/foundation_stereo.py:187-189) -> (B,4h,4w)."""
    _check("softmax_context_upsample", disp_low, logits)
    b, c, h, w = disp_low.shape
    assert c == 1 and logits.shape == (b, 9, 4 * h, 4 * w)
    disp_low, logits = _c(disp_low), _c(logits)
    out = torch.empty((b, 4 * h, 4 * w), device=disp_low.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_softmax_context_upsample(_p(disp_low), _p(logits), _p(out), float(scale), b, h, w,
                                                         _stream(disp_low)), "softmax_context_upsample")
    return out


def gru_reset(zr_s: Tensor, zr_l: Tensor, h: Tensor, x: Tensor):
    """[sigmoid(r)*h, x] for the small and large GRU (core/update.py:92-93)."""
    _check("gru_reset", zr_s, zr_l, h, x)
    B, Hd, H, W = h.shape
    Cx = x.shape[1]
    zr_s, zr_l, h, x = _c(zr_s), _c(zr_l), _c(h), _c(x)
    qs = torch.empty((B, Hd + Cx, H, W), device=h.device, dtype=torch.float32)
    ql = torch.empty_like(qs)
    _lib.check(_lib.load().fsmi_gru_reset(_p(zr_s), _p(zr_l), _p(h), _p(x), _p(qs), _p(ql), B, Hd, Cx, H, W,
                                          _stream(h)), "gru_reset")
    return qs, ql


def gru_blend(zr_s: Tensor, zr_l: Tensor, q_s: Tensor, q_l: Tensor, h: Tensor, att: Tensor) -> Tensor:
    """att*GRU_small + (1-att)*GRU_large state update (core/update.py:91,94-95,117)."""
    _check("gru_blend", zr_s, zr_l, q_s, q_l, h, att)
    B, Hd, H, W = h.shape
    zr_s, zr_l, q_s, q_l, h, att = (_c(t) for t in (zr_s, zr_l, q_s, q_l, h, att))
    out = torch.empty_like(h)
    _lib.check(_lib.load().fsmi_gru_blend(_p(zr_s), _p(zr_l), _p(q_s), _p(q_l), _p(h), _p(att), _p(out), B, Hd,
                                          H, W, _stream(h)), "gru_blend")
    return out


def conv3d_direct(x: Tensor, w: Tensor, bias: Tensor = None) -> Tensor:
    """Stride-1, zero-padded (KS//2) 3D conv for Cout == 1 (the classifier head, core/foundation_stereo.py:175)."""
    _check("conv3d_direct", x, w, *([bias] if bias is not None else []))
    B, Cin, D, H, W = x.shape
    Cout, Cw, KS = w.shape[0], w.shape[1], w.shape[2]
    assert Cw == Cin and tuple(w.shape[2:]) == (KS, KS, KS)
    x, w = _c(x), _c(w)
    out = torch.empty((B, Cout, D, H, W), device=x.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_conv3d_direct(_p(x), _p(w), _p(bias) if bias is not None else None, _p(out), B, Cin,
                                              Cout, KS, D, H, W, _stream(x)), "conv3d_direct")
    return out


# leaky: halo kernel only; relu_pre: ReLU(conv + bias + res), res added BEFORE the activation (2D halo /
# pointwise tiles; SelectiveConvGRU.conv0 with its loop-invariant context segment precomputed into res)
ACT = {None: 0, "none": 0, "relu": 1, "gelu": 2, "leaky": 6, "relu_pre": 7}


class PackedConv:
    """Conv weights packed once for the halo-tiled split-precision kernels
    (``fsmi_conv2d_halo_x3`` / ``fsmi_conv3d_halo_x3_ex``): fp16 hi / lo halves of each output
    channel's weights pre-scaled by 2^wexp[co] (square 1x1 / 2x2 / 3x3 taps, optionally KD deep).
    Several weight tensors stacked along Cout form one conv (e.g. convz|convr).
    """

    def __init__(self, *weights: Tensor, mode: str = "halo"):
        assert mode == "halo", f"PackedConv: mode {mode!r} (only the halo kernels remain)"
        w = torch.cat([x.detach().float() for x in weights], 0)
        if w.dim() == 5:                    # Conv3d (Cout, Cin, KD, KS, KS): taps kd-major
            self.kd = w.shape[2]
            w = w.permute(0, 1, 3, 4, 2)    # taps are packed as (kd, kh, kw) below
        else:
            self.kd = 1
            w = w.unsqueeze(-1)
        self.cout, self.cin, self.k, kw, _ = w.shape
        assert self.k == kw
        self.mode = mode
        assert self.k in (1, 2, 3), "halo conv: 1x1, 2x2 (transposed-conv phases) or 3x3"
        cinp = (self.cin + 31) // 32 * 32
        coutp = (self.cout + 31) // 32 * 32
        # per output channel: row max |w| * 2^e[co] in [1, 2) -- BN folding spreads the rows'
        # scales over decades, and a per-tensor exponent would leave the small rows' lo halves
        # fp16-subnormal (~11-bit weights).  The kernel multiplies row co by wscale[co] = 2^-e[co].
        rmax = w.abs().reshape(self.cout, -1).amax(1).double()
        e = torch.where(rmax > 0, -torch.floor(torch.log2(torch.where(rmax > 0, rmax, torch.ones_like(rmax)))),
                        torch.zeros_like(rmax)).clamp(-100, 100)
        row_scale = torch.pow(2.0, e).float().view(-1, 1, 1, 1, 1)
        self.wscale = torch.pow(2.0, -e).float().contiguous()
        ws = torch.zeros((coutp, cinp, self.kd, self.k, self.k), device=w.device, dtype=torch.float32)
        ws[:self.cout, :self.cin] = w.permute(0, 1, 4, 2, 3) * row_scale
        # [tap = (kd, kh, kw)][cin chunk][cout][32]
        ws = ws.permute(2, 3, 4, 1, 0).reshape(self.kd * self.k * self.k, cinp // 32, 32, coutp) \
            .permute(0, 1, 3, 2).contiguous()
        hi = ws.half()
        lo = (ws - hi.float()).half()
        self.whi, self.wlo = hi.contiguous(), lo.contiguous()
        self._sb = {}
        self._sb_retired = []            # pinned (scale, bias) buffers whose key was reused: kept alive

    def scale_bias(self, bias: Tensor = None) -> Tensor:
        """(2^-wexp[co], bias[co]) pairs, 2*Cout floats, for the halo kernels' epilogue, cached per
        bias tensor and version so that a captured graph keeps reading one stable buffer.

        Entries for parameters (and for biases first seen during a stream capture, whose buffer a
        graph node now holds) live as long as this PackedConv.  A per-call temporary bias (e.g.
        ``bias.float()`` under a half model) keeps only its latest entry: an entry is valid only for
        the very tensor object it was built from (a weak reference, so a recycled address is never
        a false hit), and each eager use records the current stream on the buffer, so dropping it
        later cannot hand its memory to a new allocation while a kernel on another stream may still
        read it."""
        import weakref
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        key = None if bias is None else (bias.data_ptr(), bias._version)
        hit = self._sb.get(key)
        if hit is not None and hit[1] is not None and hit[1]() is not bias:
            # the address now belongs to another tensor.  A pinned entry's buffer may still be read by
            # a captured graph node: it is retired, never dropped, before the key is reused
            if hit[2]:
                self._sb_retired.append(hit[0])
            hit = None
        if hit is None:
            b = torch.zeros_like(self.wscale) if bias is None else bias.detach().float().reshape(-1)
            assert b.numel() == self.cout, f"bias of {b.numel()} for {self.cout} output channels"
            pinned = bias is None or isinstance(bias, torch.nn.Parameter) or capturing
            if not pinned:
                for k in [k for k, v in self._sb.items() if not v[2]]:
                    del self._sb[k]
            hit = self._sb[key] = (torch.stack([self.wscale, b], 1).contiguous(),
                                   None if bias is None else weakref.ref(bias), pinned)
        if not hit[2] and not capturing and hit[0].is_cuda:
            hit[0].record_stream(torch.cuda.current_stream(hit[0].device))
        return hit[0]


def _segments(segs):
    import ctypes
    norm = []
    for s in segs:
        t, c0, n = (s, 0, s.shape[1]) if isinstance(s, torch.Tensor) else s
        norm.append((t, c0, n))
    t0 = norm[0][0]
    B, _, H, W = t0.shape
    HW = H * W
    for t, c0, n in norm:
        assert t.is_contiguous() and t.shape[0] == B and t.shape[2:] == (H, W) and c0 + n <= t.shape[1], \
            "conv2d: segment shape mismatch"
    nseg = len(norm)
    ptrs = (ctypes.c_void_p * nseg)(*[t.data_ptr() + 4 * c0 * HW for t, c0, _ in norm])
    chs = (ctypes.c_int * nseg)(*[n for _, _, n in norm])
    tots = (ctypes.c_int * nseg)(*[t.shape[1] for t, _, _ in norm])
    return norm, (ctypes.cast(ptrs, ctypes.POINTER(ctypes.c_void_p)), chs, tots, ptrs), sum(n for _, _, n in norm)


_ACT3D = {None: 0, "relu": 1, "leaky": 6}


def conv3d(x: Tensor, pk, bias: Tensor = None, act=None, res: Tensor = None, res_pre: bool = False,
           cfg: int = -1, nsplit: int = -1, stride: int = 1, fatt: Tensor = None) -> Tensor:
    """'Same' Conv3d (KD x K x K, K in {1, 3}, KD odd) on the halo split-precision kernel
    (``fsmi_conv3d_halo_x3_ex``); NCDHW in and out.  ``act`` None / "relu" / "leaky" (0.01);
    ``res`` is added after the activation, or before it with ``res_pre`` (ResNet block tail).
    ``stride`` 2: KD x K x K with K, KD in {1, 3}, padding K // 2, KD // 2 and stride 2 (output
    (n - 1) // 2 + 1 per dimension; 2D convs as volumes of depth 1).
    ``fatt``: FeatureAtt's pre-sigmoid gate (B, Cout, Ho, Wo); the output is multiplied by
    sigmoid(fatt) broadcast over depth (core/submodule.py:452-453)."""
    assert pk.mode == "halo" and x.dim() == 5
    assert stride in (1, 2) and (stride == 1 or (pk.k in (1, 3) and pk.kd in (1, 3))), \
        "conv3d: stride 2 needs K, KD in {1, 3}"
    _check("conv3d", x, *[t for t in (bias, res, fatt) if t is not None])
    B, Cin, D, H, W = x.shape
    assert Cin == pk.cin, f"conv3d: {Cin} input channels for a conv packed with {pk.cin}"
    x = _c(x)
    Do, Ho, Wo = (D, H, W) if stride == 1 else ((D - 1) // 2 + 1, (H - 1) // 2 + 1, (W - 1) // 2 + 1)
    out = torch.empty((B, pk.cout, Do, Ho, Wo), device=x.device, dtype=torch.float32)
    if res is not None:
        res = _c(res)
        assert res.shape == out.shape
    if fatt is not None:
        fatt = _c(fatt)
        assert tuple(fatt.shape) == (B, pk.cout, Ho, Wo), f"conv3d: gate {tuple(fatt.shape)} for output {tuple(out.shape)}"
    if _CONV_FLOPS["on"]:
        _CONV_FLOPS["flops"] += 2 * Cin * pk.cout * pk.kd * pk.k * pk.k * B * Do * Ho * Wo
    stream = _stream(x)
    ws = _split_workspace(x.device, stream, 8 * B * pk.cout * Do * Ho * Wo)
    cfg, nsplit = _tuned(pk.k if stride == 1 else f"{pk.k}s2", pk.kd, Cin, pk.cout, B, D, H, W, cfg, nsplit)
    if cfg == 30 and not _DEPTH_TILE:
        cfg, nsplit = -1, -1           # A/B: the generic volume tiles (the C side picks)
    _lib.check(_lib.load().fsmi_conv3d_halo_x3_ex(
        _p(x), Cin, _p(pk.whi), _p(pk.wlo), _p(pk.scale_bias(bias)),
        _p(res) if res is not None else None, _p(fatt) if fatt is not None else None, _p(out), B, pk.cout,
        D, H, W, pk.kd, pk.k, stride, _ACT3D[act], 1 if res_pre else 0, cfg, nsplit, _p(ws), ws.numel(), stream),
        "conv3d")
    return out


# kernel index of each 2-tap phase conv of ConvTranspose3d(k=4, s=2, p=1): output 2m + p reads input
# m - 1 + t (+1 for p = 1) through kernel element _UP2_K[p][t]
_UP2_K = ((3, 1), (2, 0))


def pack_deconv_phases(weight: Tensor, scale: Tensor = None):
    """ConvTranspose3d(k=4, s=2, p=1) weight (Cin, Cout, 4, 4, 4), optionally scaled per output
    channel (folded BatchNorm), as the 8 phase convs of ``fsmi_conv3d_up2_halo_x3``."""
    w = weight.detach().double()
    assert w.dim() == 5 and tuple(w.shape[2:]) == (4, 4, 4), "pack_deconv_phases: k = 4 only"
    if scale is not None:
        w = w * scale.detach().double().view(1, -1, 1, 1, 1)
    packs = []
    for p in range(8):
        pd, ph, pw = p >> 2, (p >> 1) & 1, p & 1
        kd = [_UP2_K[pd][t] for t in range(2)]
        kh = [_UP2_K[ph][t] for t in range(2)]
        kw = [_UP2_K[pw][t] for t in range(2)]
        wp = w[:, :, kd][:, :, :, kh][:, :, :, :, kw]            # (Cin, Cout, 2, 2, 2)
        packs.append(PackedConv(wp.permute(1, 0, 2, 3, 4).float().contiguous(), mode="halo"))
    return packs


def conv3d_up2(x: Tensor, packs, bias: Tensor = None, act=None, cfg: int = -1) -> Tensor:
    """ConvTranspose3d(k=4, s=2, p=1) (+ bias / folded BN, activation) on the halo kernel's 2x2x2
    phase tiles: (B, Cin, D, H, W) -> (B, Cout, 2D, 2H, 2W)."""
    assert len(packs) == 8 and all(pk.mode == "halo" and pk.k == 2 and pk.kd == 2 for pk in packs)
    _check("conv3d_up2", x, *([bias] if bias is not None else []))
    B, Cin, D, H, W = x.shape
    pk0 = packs[0]
    assert Cin == pk0.cin, f"conv3d_up2: {Cin} input channels for a conv packed with {pk0.cin}"
    x = _c(x)
    out = torch.empty((B, pk0.cout, 2 * D, 2 * H, 2 * W), device=x.device, dtype=torch.float32)
    if _CONV_FLOPS["on"]:
        _CONV_FLOPS["flops"] += 2 * Cin * pk0.cout * 64 * B * D * H * W
    whi, k1 = _lib.ptr_array([_p(pk.whi) for pk in packs])
    wlo, k2 = _lib.ptr_array([_p(pk.wlo) for pk in packs])
    sbs = [pk.scale_bias(bias) for pk in packs]
    sb, k3 = _lib.ptr_array([_p(t) for t in sbs])
    _lib.check(_lib.load().fsmi_conv3d_up2_halo_x3(_p(x), Cin, whi, wlo, sb, _p(out), B, pk0.cout, D, H, W,
                                                   _ACT3D[act], cfg, _stream(x)), "conv3d_up2")
    del k1, k2, k3
    return out


def pack_deconv2d_phases(weight: Tensor, scale: Tensor = None):
    """ConvTranspose2d(k=4, s=2, p=1) weight (Cin, Cout, 4, 4), optionally scaled per output channel
    (folded BatchNorm), as the 4 phase convs (2x2, stride 1) of ``fsmi_conv2d_up2_halo_x3``."""
    w = weight.detach().double()
    assert w.dim() == 4 and tuple(w.shape[2:]) == (4, 4), "pack_deconv2d_phases: k = 4 only"
    if scale is not None:
        w = w * scale.detach().double().view(1, -1, 1, 1)
    packs = []
    for p in range(4):
        ph, pw = p >> 1, p & 1
        kh = [_UP2_K[ph][t] for t in range(2)]
        kw = [_UP2_K[pw][t] for t in range(2)]
        wp = w[:, :, kh][:, :, :, kw]                            # (Cin, Cout, 2, 2)
        packs.append(PackedConv(wp.permute(1, 0, 2, 3).float().contiguous(), mode="halo"))
    return packs


def conv2d_up2(x: Tensor, packs, bias: Tensor = None, act=None, cfg: int = -1) -> Tensor:
    """ConvTranspose2d(k=4, s=2, p=1) (+ bias / folded BN, activation) on the halo kernel's 2x2 phase
    tiles: (B, Cin, H, W) -> (B, Cout, 2H, 2W)."""
    assert len(packs) == 4 and all(pk.mode == "halo" and pk.k == 2 and pk.kd == 1 for pk in packs)
    _check("conv2d_up2", x, *([bias] if bias is not None else []))
    B, Cin, H, W = x.shape
    pk0 = packs[0]
    assert Cin == pk0.cin, f"conv2d_up2: {Cin} input channels for a conv packed with {pk0.cin}"
    x = _c(x)
    out = torch.empty((B, pk0.cout, 2 * H, 2 * W), device=x.device, dtype=torch.float32)
    if _CONV_FLOPS["on"]:
        _CONV_FLOPS["flops"] += 2 * Cin * pk0.cout * 16 * B * H * W
    whi, k1 = _lib.ptr_array([_p(pk.whi) for pk in packs])
    wlo, k2 = _lib.ptr_array([_p(pk.wlo) for pk in packs])
    sbs = [pk.scale_bias(bias) for pk in packs]
    sb, k3 = _lib.ptr_array([_p(t) for t in sbs])
    _lib.check(_lib.load().fsmi_conv2d_up2_halo_x3(_p(x), Cin, whi, wlo, sb, _p(out), B, pk0.cout, H, W,
                                                   _ACT3D[act], cfg, _stream(x)), "conv2d_up2")
    del k1, k2, k3
    return out


_GATE_MODE = {"zr": 0, "blend_small": 1, "blend_large": 2}

_RANGE_DEBUG = os.environ.get("FSMI_RANGE_DEBUG", "0") == "1"   # diagnostics: sync + check after each conv


def _range_debug(what, segs, out=None, ch=None):
    if not _RANGE_DEBUG or torch.cuda.is_current_stream_capturing():
        return
    if range_overflowed(reset=True):
        desc = [(tuple(t.shape), c0, n, float(t[:, c0:c0 + n].abs().max())) for t, c0, n in segs]
        print(f"[fsmi range] {what}: segments (shape, c0, n, max|x|) {desc}", flush=True)
    if out is not None:                  # an output far beyond any activation: report its producer
        o = out if ch is None else out[:, ch[0]:ch[1]]
        m = float(o.abs().max())
        if not m < 1e15:
            desc = [(tuple(t.shape), c0, n, float(t[:, c0:c0 + n].abs().max())) for t, c0, n in segs]
            print(f"[fsmi range] {what}: OUTPUT max|y| {m:.3g}; inputs {desc}", flush=True)


def conv2d_gate(segs, pk, bias: Tensor, mode: str, h: Tensor, z: Tensor, att: Tensor = None, rh: Tensor = None,
                out: Tensor = None, nsplit: int = -1, cfg: int = -1):
    """Halo conv with a SelectiveConvGRU gate epilogue (``fsmi_conv2d_halo_x3_gate``).

    ``mode`` "zr": ``pk`` = [convz; convr] stacked; writes ``z = sigmoid(.)`` and ``rh = sigmoid(r)*h``.
    "blend_small": ``out = ((1-z)h + z*tanh(convq)) * att``; "blend_large": ``out += (...) * (1-att)``
    (core/update.py:88-95,117)."""
    assert pk.mode == "halo", "conv2d_gate: needs a PackedConv(mode='halo')"
    norm, (pp, chs, tots, keep), cin = _segments(segs)
    t0 = norm[0][0]
    B, _, H, W = t0.shape
    Hd = h.shape[1]
    m = _GATE_MODE[mode]
    extra = [x for x in (bias, h, z, att, rh, out) if x is not None]
    _check("conv2d_gate", *[t for t, _, _ in norm], *extra)
    assert cin == pk.cin, f"conv2d_gate: {cin} input channels for a conv packed with {pk.cin}"
    for x in (h, z, att, rh, out):
        assert x is None or (x.is_contiguous() and x.shape[0] == B and x.shape[2:] == (H, W)), \
            "conv2d_gate: shape mismatch"
    if m == 0:
        assert pk.cout == 2 * Hd and rh is not None
    else:
        assert pk.cout == Hd and att is not None and out is not None
    if _CONV_FLOPS["on"]:
        _CONV_FLOPS["flops"] += 2 * cin * pk.cout * pk.k * pk.k * B * H * W
    stream = _stream(t0)
    ws = _split_workspace(t0.device, stream, 8 * B * pk.cout * H * W)
    cfg, nsplit = _tuned(pk.k, 1, cin, pk.cout, B, 1, H, W, cfg, nsplit)
    _lib.check(_lib.load().fsmi_conv2d_halo_x3_gate(
        pp, chs, tots, len(norm), _p(pk.whi), _p(pk.wlo), _p(pk.scale_bias(bias)), m, _p(h), _p(z),
        _p(att) if att is not None else None, _p(rh) if rh is not None else None, Hd,
        _p(out) if out is not None else None, out.shape[1] if out is not None else 0, 0, B, pk.cout, pk.k, H, W,
        cfg, nsplit, _p(ws), ws.numel(), stream), "conv2d_gate")
    _range_debug(f"conv2d_gate {mode} k{pk.k} {cin}->{pk.cout}", norm)
    del keep


# ---- measured tile / split-K choices per conv shape (tools/tune_conv.py -> tuning/fsmi_conv.json):
# consulted when a caller leaves cfg / nsplit on auto; shapes not in the table use the C-side policy
_TUNE_PATH = os.environ.get("FSMI_TUNE_PATH") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning", "fsmi_conv.json")
_TUNE = None
_RECORD = None          # set of shape keys while tools/tune_conv.py records a forward


def _tune_key(ks, kd, cin, cout, B, D, H, W) -> str:
    return f"k{ks}_d{kd}_ci{cin}_co{cout}_b{B}_D{D}_h{H}_w{W}"


def _tuned(ks, kd, cin, cout, B, D, H, W, cfg, nsplit):
    global _TUNE
    key = _tune_key(ks, kd, cin, cout, B, D, H, W)
    if _RECORD is not None:           # a set (shape keys) or a dict (call counts, tools/conv_census.py)
        if isinstance(_RECORD, dict):
            _RECORD[key] = _RECORD.get(key, 0) + 1
        else:
            _RECORD.add(key)
    if cfg >= 0 and nsplit >= 0 or os.environ.get("FSMI_TUNE_DB", "1") == "0":
        return cfg, nsplit
    if _TUNE is None:
        _TUNE = {}
        if os.path.exists(_TUNE_PATH):
            with open(_TUNE_PATH) as f:
                _TUNE = json.load(f).get("entries", {})
    e = _TUNE.get(key)
    if e is not None:
        cfg, nsplit = (e["cfg"] if cfg < 0 else cfg), (e["nsplit"] if nsplit < 0 else nsplit)
    if _SPLIT_MAXPIX and kd == 1 and D == 1 and H * W <= _SPLIT_MAXPIX:
        nsplit = 1
    if _SPLIT_CAP and nsplit > _SPLIT_CAP and not (e is not None and e.get("insitu")):
        nsplit = _SPLIT_CAP          # entries chosen end to end (tools/insitu_tune.py) are kept as they are
    return cfg, nsplit


# A/B knob: no split-K for 2D maps of at most this many pixels (the 1/8 and 1/16 GRU levels run on
# a side stream beside gru04, so the chip is already busy and split-K only adds the reduce pass)
_SPLIT_MAXPIX = int(os.environ.get("FSMI_SPLIT_MAXPIX", "0"))
# Cap on the split-K factor of auto-chosen layers (0: none).  The table is timed one layer at a
# time on an idle chip; inside the 4-stream pipelined loop other streams' kernels fill the CUs that
# a deep split was chosen to fill, and the extra partial-sum traffic remains.  Measured end to end
# (cfg2, two runs each): cap 2 +1.3 %, cap 3 -1.2 %, cap 1 -12 %; cfg3 (4 pairs / GPU) neutral.
_SPLIT_CAP = int(os.environ.get("FSMI_SPLIT_CAP", "2"))
# (17, 1, 1) volume convs (Conv3dNormActReduced.conv2) on the depth-blocked tile (cfg 30); 0: the
# generic volume tiles from the tuning table (A/B)
_DEPTH_TILE = os.environ.get("FSMI_DEPTH_TILE", "1") != "0"


_SPLIT_WS = {}


def _split_workspace(dev, stream, floats: int):
    """Split-K partial-sum buffer, one per (device, stream); reuse is stream-ordered."""
    key = (dev, stream)
    ws = _SPLIT_WS.get(key)
    if ws is None or ws.numel() < floats:
        ws = torch.empty(max(floats, 1 << 22), device=dev, dtype=torch.float32)
        _SPLIT_WS[key] = ws
    return ws


def conv2d(segs, pk, bias: Tensor = None, act=None, alpha: float = 1.0, gamma: Tensor = None,
           res: Tensor = None, out: Tensor = None, co0: int = 0, cfg: int = -1, nsplit: int = -1) -> Tensor:
    """Halo-tiled split-precision conv (stride 1, 'same' zero padding, ``fsmi_conv2d_halo_x3``).

    ``segs``: list of NCHW tensors or ``(tensor, c_start, c_count)`` channel slices,
    concatenated along C without a copy.  ``pk``: a ``PackedConv``.  Writes
    ``out[:, co0:co0+cout]`` (allocated as (B, cout, H, W) when None) =
    ``res + gamma * alpha * act(conv + bias)``."""
    norm, (pp, chs, tots, keep), cin = _segments(segs)
    t0 = norm[0][0]
    B, _, H, W = t0.shape
    extra = [x for x in (bias, gamma, res) if x is not None]
    _check("conv2d", *[t for t, _, _ in norm], *extra)
    assert pk.mode == "halo" and cin == pk.cin, f"conv2d: {cin} input channels for a conv packed with {pk.cin}"
    if out is None:
        out = torch.empty((B, pk.cout, H, W), device=t0.device, dtype=torch.float32)
    assert out.is_contiguous() and out.shape[0] == B and out.shape[2:] == (H, W)
    if res is not None:
        assert res.is_contiguous() and res.shape[2:] == (H, W)
    if _CONV_FLOPS["on"]:
        _CONV_FLOPS["flops"] += 2 * cin * pk.cout * pk.k * pk.k * B * H * W
    stream = _stream(t0)
    # auto split-K is capped at 8; the workspace covers that for this output
    ws = _split_workspace(t0.device, stream, 8 * B * pk.cout * H * W)
    tcfg, nsplit = _tuned(pk.k, 1, cin, pk.cout, B, 1, H, W, cfg, nsplit)
    _lib.check(_lib.load().fsmi_conv2d_halo_x3(
        pp, chs, tots, len(norm), _p(pk.whi), _p(pk.wlo), _p(pk.scale_bias(bias)),
        _p(gamma) if gamma is not None else None, _p(res) if res is not None else None,
        res.shape[1] if res is not None else 0, _p(out), out.shape[1], co0, B, pk.cout, pk.k, H, W, ACT[act],
        float(alpha), tcfg, nsplit, _p(ws), ws.numel(), stream), "conv2d_halo_x3")
    _range_debug(f"conv2d k{pk.k} {cin}->{pk.cout}", norm, out, (co0, co0 + pk.cout))
    del keep
    return out


def dwconv2d(x: Tensor, w: Tensor, bias: Tensor = None) -> Tensor:
    """Depthwise conv, ``nn.Conv2d(C, C, KS, padding=KS//2, groups=C)`` (KS in 3/5/7)."""
    _check("dwconv2d", x, w, *([bias] if bias is not None else []))
    B, C, H, W = x.shape
    KS = w.shape[-1]
    assert w.shape == (C, 1, KS, KS), f"dwconv2d: weight {tuple(w.shape)} for {C} channels"
    x, w = _c(x), _c(w)
    out = torch.empty_like(x)
    _lib.check(_lib.load().fsmi_dwconv2d(_p(x), _p(w), _p(_c(bias)) if bias is not None else None, _p(out), B, C,
                                         KS, H, W, _stream(x)), "dwconv2d")
    return out


def edgenext_mlp(x: Tensor, res: Tensor, pk1: "PackedConv", bias1: Tensor, pk2: "PackedConv", bias2: Tensor,
                 gamma: Tensor = None, out: Tensor = None) -> Tensor:
    """EdgeNextConvEncoder's MLP tail in one kernel (core/submodule.py:583-590):
    ``res + gamma * pwconv2(gelu(pwconv1(x)))`` over channels at every pixel; ``pk1`` / ``pk2`` the
    PackedConv of the pwconv1 (E x C) / pwconv2 (C x E) Linear weights as 1x1 convs."""
    g = _c(gamma.detach().float()) if gamma is not None else None
    _check("edgenext_mlp", x, res, bias1, bias2, *([g] if g is not None else []))
    B, C, H, W = x.shape
    assert res.shape == x.shape, f"edgenext_mlp: res {tuple(res.shape)} vs x {tuple(x.shape)}"
    assert pk1.k == 1 and pk2.k == 1 and pk1.cin == C and pk2.cout == C and pk2.cin == pk1.cout, \
        f"edgenext_mlp: W1 {pk1.cout}x{pk1.cin}, W2 {pk2.cout}x{pk2.cin} for {C} channels"
    if out is not None:
        # the kernel writes dense NCHW fp32 at out's data pointer: a caller's buffer must be exactly
        # that, and an in-place update (out is res) must not go through a copy of res
        _check("edgenext_mlp", out)
        if tuple(out.shape) != tuple(x.shape) or not out.is_contiguous() or out.device != x.device:
            raise RuntimeError(f"edgenext_mlp: out must be a contiguous {tuple(x.shape)} fp32 tensor on {x.device}")
        if out.data_ptr() % 16:
            raise RuntimeError("edgenext_mlp: out must be 16-byte aligned")
        if out is res or out.data_ptr() == res.data_ptr():
            if not res.is_contiguous() or res.data_ptr() % 16:
                raise RuntimeError("edgenext_mlp: an in-place update (out is res) needs a contiguous, aligned res")
        elif _overlaps(out, res):
            raise RuntimeError("edgenext_mlp: out partially overlaps res")
        if _overlaps(out, x):
            raise RuntimeError("edgenext_mlp: out must not alias x (x is re-read after out is written)")
    x, res = _c(x), (res if out is not None and out.data_ptr() == res.data_ptr() else _c(res))
    out = torch.empty_like(x) if out is None else out
    sb1, sb2 = pk1.scale_bias(bias1), pk2.scale_bias(bias2)
    _lib.check(_lib.load().fsmi_edgenext_mlp(_p(x), _p(res), _p(out), _p(pk1.whi), _p(pk1.wlo), _p(sb1), _p(pk2.whi),
                                             _p(pk2.wlo), _p(sb2), _p(g) if g is not None else None, B, C,
                                             pk1.cout, H, W, _stream(x)), "edgenext_mlp")
    if _CONV_FLOPS["on"]:
        _CONV_FLOPS["flops"] += 2 * 2 * C * pk1.cout * B * H * W
    return out


def pool2x(x: Tensor) -> Tensor:
    """``F.avg_pool2d(x, 3, stride=2, padding=1)`` (count_include_pad: every window / 9)."""
    _check("pool2x", x)
    B, C, H, W = x.shape
    x = _c(x)
    out = torch.empty((B, C, (H - 1) // 2 + 1, (W - 1) // 2 + 1), device=x.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_pool2x(_p(x), _p(out), B, C, H, W, _stream(x)), "pool2x")
    return out


def conv2d_1in(x: Tensor, w: Tensor, bias: Tensor = None, relu: bool = False) -> Tensor:
    """``Conv2d(1, Cout, KS, padding=KS//2)`` (+ ReLU) -- the motion encoder's convd1."""
    _check("conv2d_1in", x, w, *([bias] if bias is not None else []))
    B, C, H, W = x.shape
    Cout, KS = w.shape[0], w.shape[-1]
    assert C == 1 and tuple(w.shape) == (Cout, 1, KS, KS), f"conv2d_1in: {tuple(x.shape)} x {tuple(w.shape)}"
    x, w = _c(x), _c(w)
    out = torch.empty((B, Cout, H, W), device=x.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_conv2d_1in(_p(x), _p(w), _p(_c(bias)) if bias is not None else None, _p(out), B,
                                           Cout, KS, H, W, 1 if relu else 0, _stream(x)), "conv2d_1in")
    return out


def conv3x3_cout1(x: Tensor, w: Tensor, bias: Tensor = None, res: Tensor = None, out: Tensor = None,
                  co0: int = 0) -> Tensor:
    """``Conv2d(Cin, 1, 3, padding=1)`` (+ bias, + ``res`` (B, 1, H, W)) in fp32 (``fsmi_conv3x3_cout1``):
    DispHead's last layer.  Writes channel ``co0`` of ``out`` (allocated as (B, 1, H, W) when None)."""
    _check("conv3x3_cout1", x, w, *[t for t in (bias, res) if t is not None])
    B, C, H, W = x.shape
    assert tuple(w.shape) == (1, C, 3, 3), f"conv3x3_cout1: weight {tuple(w.shape)} for {C} channels"
    x, w = _c(x), _c(w.detach().float())
    if out is None:
        out = torch.empty((B, 1, H, W), device=x.device, dtype=torch.float32)
    assert out.is_contiguous() and out.shape[0] == B and out.shape[2:] == (H, W) and 0 <= co0 < out.shape[1], \
        "conv3x3_cout1: out must be a contiguous (B, C, H, W) tensor with channel co0"
    if res is not None:
        assert res.shape[0] == B and res.shape[1] == 1 and res.shape[2:] == (H, W) and res.stride(2) == W and \
            res.stride(3) == 1, "conv3x3_cout1: res must be (B, 1, H, W) with dense planes"
    b = _c(bias.detach().float().reshape(-1)) if bias is not None else None    # device pointer: no sync under capture
    HW = H * W
    _lib.check(_lib.load().fsmi_conv3x3_cout1(
        _p(x), C, _p(w), _p(b) if b is not None else None, _p(res) if res is not None else None, res.stride(0) if res is not None else 0,
        out.data_ptr() + 4 * co0 * HW, out.stride(0), B, H, W, _stream(x)), "conv3x3_cout1")
    if _CONV_FLOPS["on"]:
        _CONV_FLOPS["flops"] += 2 * C * 9 * B * HW
    return out


def resize_bilinear(x: Tensor, size) -> Tensor:
    """``F.interpolate(x, size, mode="bilinear", align_corners=True)``."""
    _check("resize_bilinear", x)
    B, C, Hi, Wi = x.shape
    Ho, Wo = size
    x = _c(x)
    out = torch.empty((B, C, Ho, Wo), device=x.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_resize_bilinear(_p(x), _p(out), B, C, Hi, Wi, Ho, Wo, _stream(x)),
               "resize_bilinear")
    return out


# ---------------------------------------------------------------- disparity transformer

def dt_patch_embed(x: Tensor, w: Tensor, scale: Tensor, shift: Tensor) -> Tensor:
    """``conv_patch`` (core/foundation_stereo.py:85-88): depthwise Conv3d k4 s4 with bias + eval
    BatchNorm folded into per-channel ``scale`` / ``shift``; (B,C,D,H,W) -> (B,C,D/4,H/4,W/4)."""
    _check("dt_patch_embed", x, w, scale, shift)
    B, C, D, H, W = x.shape
    assert tuple(w.shape) == (C, 1, 4, 4, 4) and scale.numel() == C and shift.numel() == C
    if D % 4 or H % 4 or W % 4:
        raise RuntimeError(f"dt_patch_embed: D, H, W must be multiples of 4, got {(D, H, W)}")
    x, w, scale, shift = _c(x), _c(w), _c(scale), _c(shift)
    out = torch.empty((B, C, D // 4, H // 4, W // 4), device=x.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_dt_patch_embed(_p(x), _p(w), _p(scale), _p(shift), _p(out), B, C, D, H, W,
                                               _stream(x)), "dt_patch_embed")
    return out


def dt_layer_floats() -> int:
    return _lib.load().fsmi_dt_layer_floats()


def pack_dt_layers(layers) -> Tensor:
    """Per-layer parameters of FlashAttentionTransformerEncoderLayer modules in the kernel's
    order [Wq bq Wk bk Wv bv Wo bo ln1.w ln1.b W1 b1 W2 b2 ln2.w ln2.b]."""
    parts = []
    for m in layers:
        a = m.self_attn
        for t in (a.q_proj.weight, a.q_proj.bias, a.k_proj.weight, a.k_proj.bias, a.v_proj.weight, a.v_proj.bias,
                  a.out_proj.weight, a.out_proj.bias, m.norm1.weight, m.norm1.bias, m.linear1.weight,
                  m.linear1.bias, m.linear2.weight, m.linear2.bias, m.norm2.weight, m.norm2.bias):
            parts.append(t.detach().float().reshape(-1))
    p = torch.cat(parts).contiguous()
    if layers and p.numel() != len(layers) * dt_layer_floats():
        raise RuntimeError(f"pack_dt_layers: {p.numel()} floats, kernel expects {dt_layer_floats()} per layer "
                           "(built for d_model 28, 4 heads, FFN 28)")
    return p


def disparity_transformer(x: Tensor, params: Tensor, pe: Tensor, nheads: int, ffdim: int, nlayers: int,
                          eps: float = 1e-5) -> Tensor:
    """CostVolumeDisparityAttention.forward (core/submodule.py:506-528) on (B,C,L,H,W): tokens
    are the L disparities of each pixel; ``pe`` (L, C) is the positional table already sliced."""
    _check("disparity_transformer", x, params, pe)
    B, C, L, H, W = x.shape
    assert tuple(pe.shape) == (L, C)
    x, params, pe = _c(x), _c(params), _c(pe)
    out = torch.empty_like(x)
    _lib.check(_lib.load().fsmi_disparity_transformer(_p(x), _p(out), _p(params), _p(pe), B, C, L, H * W, nheads,
                                                      ffdim, nlayers, float(eps), _stream(x)),
               "disparity_transformer")
    return out


def upsample4_add_(vol: Tensor, t: Tensor) -> Tensor:
    """``vol += F.interpolate(t, scale_factor=4, mode="trilinear", align_corners=False)`` in place
    (core/foundation_stereo.py:119-120)."""
    _check("upsample4_add_", vol, t)
    B, C, D, H, W = t.shape
    if tuple(vol.shape) != (B, C, 4 * D, 4 * H, 4 * W):
        raise RuntimeError(f"upsample4_add_: volume {tuple(vol.shape)} is not 4x {tuple(t.shape)}")
    if not vol.is_contiguous() or vol.data_ptr() % 16:
        raise RuntimeError("upsample4_add_: the volume must be contiguous and 16-B aligned (in-place add)")
    t = _c(t)
    _lib.check(_lib.load().fsmi_upsample4_add(_p(t), _p(vol), B, C, D, H, W, _stream(vol)), "upsample4_add_")
    return vol


# ---------------------------------------------------------------- range guard

class RangeError(_lib.FsmiError):
    """A split-precision conv saw an activation its block exponent could not bring into fp16's
    range (more than 2^9 x the largest value of the block's first 32-channel chunk)."""


def range_overflowed(reset: bool = True) -> bool:
    """Whether any halo conv overflowed since the last reset (fsmi_range_status).  Asynchronous:
    synchronises the device first."""
    import ctypes
    torch.cuda.synchronize()
    flag = ctypes.c_int(0)
    _lib.check(_lib.load().fsmi_range_status(1 if reset else 0, ctypes.byref(flag)), "range_status")
    return bool(flag.value)


def check_range():
    """Raise RangeError if a halo conv overflowed since the last check (then resets the flag)."""
    if range_overflowed(reset=True):
        raise RangeError("split-precision conv: an activation exceeded fp16's range after the block "
                         "exponent (inputs spanning > 2^9 within one conv tile)")


def range_poison_(out: Tensor) -> Tensor:
    """NaN-fill ``out`` on its stream if the range flag is set (device-side; capturable)."""
    _check("range_poison", out)
    assert out.is_contiguous()
    _lib.check(_lib.load().fsmi_range_poison(_p(out), out.numel(), _stream(out)), "range_poison")
    return out


def reset_range_flag():
    """Clear the range flag without synchronising (kernels still in flight may set it again)."""
    import ctypes
    flag = ctypes.c_int(0)
    _lib.check(_lib.load().fsmi_range_status(1, ctypes.byref(flag)), "range_status")


def set_range_safe(safe: bool = True):
    """Safe range mode for every 2D split-precision conv launched or captured afterwards: a
    per-chunk block exponent with exact accumulator rescaling (cannot overflow; ~3 % slower)."""
    _lib.check(_lib.load().fsmi_set_range_safe(1 if safe else 0), "set_range_safe")


def range_safe() -> bool:
    import ctypes
    v = ctypes.c_int(0)
    _lib.check(_lib.load().fsmi_get_range_safe(ctypes.byref(v)), "get_range_safe")
    return bool(v.value)


# forwards re-run in safe mode after their range flag came back set (FoundationStereo.forward,
# ShardedStereo.step); read by tests and the bench
RANGE_RECOVERIES = [0]


def guarded(run):
    """Run ``run()`` (a whole forward, eager or a graph replay) and return its result, enforcing
    the range guard once per call: synchronise, read the flag; when it is set, switch to safe
    range mode (sticky: the activations that overflowed once will again) and run again.  A
    flag still set in safe mode raises RangeError (an inf / NaN input)."""
    reset_range_flag()
    out = run()
    if range_overflowed(reset=True):
        set_range_safe(True)
        RANGE_RECOVERIES[0] += 1
        out = run()
        check_range()
    return out


def conv_launch_counts(reset: bool = False) -> List[int]:
    """Halo / pointwise / depth conv launches per tile config since the last reset (64 counters,
    fsmi_conv_launch_counts): which tile the tuning table or the policy actually ran."""
    import ctypes
    buf = (ctypes.c_longlong * 64)()
    _lib.check(_lib.load().fsmi_conv_launch_counts(buf, 64, 1 if reset else 0), "conv_launch_counts")
    return list(buf)


# ---------------------------------------------------------------- timing

# algorithmic fp32 conv FLOPs (2*Cin*Cout*k*k*B*H*W) of the conv2d calls made since the last
# timer_reset() while timers are enabled -- the numerator of bench.py's conv roofline
_CONV_FLOPS = {"on": False, "flops": 0}

# the tensors of the last timed launch per replayable kernel: fsmi_timer_replay re-issues that
# launch with its raw pointers, so they stay allocated (not recycled by the caching allocator)
# until the next timer_reset / timer_enable, which also drop the recorded launch on the C side
_REPLAY_KEEP = {}


def _keep_for_replay(kernel: str, *tensors):
    if _CONV_FLOPS["on"] and not torch.cuda.is_current_stream_capturing():
        _REPLAY_KEEP[kernel] = tensors


def timer_enable(on: bool = True, in_capture: bool = False, timeline: bool = False):
    """Per-kernel timers on / off.  ``in_capture``: the geometry kernels' clocks are also baked into
    launches captured into a hipGraph (each replay rewrites them; query after replaying).
    ``timeline``: every instrumented kernel (convs, MLP, aux) is clocked in the capture as well
    (timer mode 3; ``timer_dump_captured``)."""
    mode = (3 if timeline else 2 if in_capture else 1) if on else 0
    _lib.check(_lib.load().fsmi_timer_enable(mode), "timer_enable")
    _CONV_FLOPS["on"] = bool(on)
    _REPLAY_KEEP.clear()


def timer_reset():
    _lib.check(_lib.load().fsmi_timer_reset(), "timer_reset")
    _CONV_FLOPS["flops"] = 0
    _REPLAY_KEEP.clear()


def conv_flops() -> int:
    return _CONV_FLOPS["flops"]


def timer_replay(kernel: str, reps: int = 20) -> float:
    """Average ms of ``reps`` back-to-back replays of the last timed launch of ``kernel``
    (lookup / comb), between two hipEvents on its stream.  The launch's tensors are held in
    ``_REPLAY_KEEP`` since it was recorded, so the replays write only memory they own."""
    if kernel not in _REPLAY_KEEP:
        raise RuntimeError(f"timer_replay: no timed launch of {kernel!r} since the last timer reset")
    import ctypes
    ms = ctypes.c_double(0.0)
    _lib.check(_lib.load().fsmi_timer_replay(_lib.KERNELS.index(kernel), int(reps), ctypes.byref(ms)),
               "timer_replay")
    return ms.value


def timer_query_clock(kernel: str, captured: bool = False):
    """(total_ms, launches) of ``kernel`` from the kernel's own clock (first block start to last wave
    end): the eager launches since the last reset, or (``captured``) the launches baked into graphs
    captured with ``timer_enable(True, in_capture=True)`` -- their last replay.  Instrumented: lookup,
    cost-volume build ("comb"), all-pairs correlation ("corr") and its normalisation ("norm"), volume
    pyramid ("volpyr")."""
    import ctypes
    tot = ctypes.c_double(0.0)
    cnt = ctypes.c_longlong(0)
    fn = _lib.load().fsmi_timer_query_clock_captured if captured else _lib.load().fsmi_timer_query_clock
    _lib.check(fn(_lib.KERNELS.index(kernel), ctypes.byref(tot), ctypes.byref(cnt)), "timer_query_clock")
    return tot.value, cnt.value


def timer_dump_captured():
    """[(kernel, stream handle, start tick, end tick, tag)] of every launch captured with clocks, in
    capture order (include/fsmi.h fsmi_timer_dump_captured; ticks of 10 ns)."""
    import ctypes
    lib = _lib.load()
    need = ctypes.c_longlong(0)
    _lib.check(lib.fsmi_timer_dump_captured(None, 0, ctypes.byref(need)), "timer_dump_captured")
    buf = ctypes.create_string_buffer(int(need.value))
    _lib.check(lib.fsmi_timer_dump_captured(buf, need.value, ctypes.byref(need)), "timer_dump_captured")
    out = []
    for line in buf.value.decode().splitlines():
        k, st, t0, t1, *tag = line.split(" ", 4)
        out.append((int(k), int(st, 16) if st.startswith("0x") else 0, int(t0), int(t1),
                    (tag[0] if tag else "").strip()))
    return out


def timer_captured_count():
    """Launches captured with clocks so far; no device work, so callable inside a capture."""
    import ctypes
    n = ctypes.c_longlong(0)
    _lib.check(_lib.load().fsmi_timer_captured_count(ctypes.byref(n)), "timer_captured_count")
    return n.value


def timer_release_captured():
    """Forget the clock records of captured launches and free their slots; only once every graph
    captured with ``in_capture=True`` is destroyed (include/fsmi.h)."""
    _lib.check(_lib.load().fsmi_timer_release_captured(), "timer_release_captured")


def timer_query(kernel: str):
    """(total_ms, launches) of ``kernel`` since the last reset (synchronises its events)."""
    import ctypes
    tot = ctypes.c_double(0.0)
    cnt = ctypes.c_longlong(0)
    _lib.check(_lib.load().fsmi_timer_query(_lib.KERNELS.index(kernel), ctypes.byref(tot), ctypes.byref(cnt)),
               "timer_query")
    return tot.value, cnt.value


# ---------------------------------------------------------------- backbone (csrc/backbone.hip)

def channel_layernorm(x: Tensor, weight: Tensor = None, bias: Tensor = None, eps: float = 1e-6, n: int = None,
                      out: Tensor = None, x_offset: int = 0) -> Tensor:
    """LayerNorm over channels of every token: x (B, C, Tx, ...) with the trailing dims flattened to the
    token axis; tokens [x_offset, x_offset + n) -> out (B, C, To) (default To = n, allocated).
    nn.LayerNorm of the reference's token-major (B, T, C) tensors (dinov2 layers/block.py:63,75) and
    LayerNorm2d / channels-last LayerNorm of NCHW maps."""
    _check("channel_layernorm", x, *[t for t in (weight, bias) if t is not None])
    B, C = x.shape[:2]
    x = _c(x)
    Tx = x[0, 0].numel()
    n = Tx - x_offset if n is None else n
    assert 0 < n and x_offset + n <= Tx, f"channel_layernorm: tokens [{x_offset}, {x_offset + n}) of {Tx}"
    if out is None:
        out = torch.empty((B, C, n), device=x.device, dtype=torch.float32)
    _check("channel_layernorm", out)
    assert out.is_contiguous() and out.shape[:2] == (B, C)
    To = out[0, 0].numel()
    assert To >= n
    w = _c(weight.detach().float()) if weight is not None else None
    b = _c(bias.detach().float()) if bias is not None else None
    _lib.check(_lib.load().fsmi_channel_layernorm(_p(x) + 4 * x_offset, _p(out), _p(w) if w is not None else None,
                                                  _p(b) if b is not None else None, B, C, Tx, To, n, float(eps),
                                                  _stream(x)), "channel_layernorm")
    return out


def vit_attention(qkv: Tensor, heads: int, T: int, scale: float, out: Tensor = None) -> Tensor:
    """Multi-head softmax(q k^T * scale) v (dinov2 layers/attention.py:69-79) on the channel-major qkv
    (B, 3*heads*64, Tp) of the qkv 1x1 conv; keys >= T masked -> (B, heads*64, Tp)."""
    _check("vit_attention", qkv)
    B, C3 = qkv.shape[:2]
    qkv = _c(qkv)
    Tp = qkv[0, 0].numel()
    hd = C3 // (3 * heads)
    assert C3 == 3 * heads * hd
    if out is None:
        out = torch.empty((B, heads * hd) + tuple(qkv.shape[2:]), device=qkv.device, dtype=torch.float32)
    _check("vit_attention", out)
    lib = _lib.load()
    nws = int(lib.fsmi_vit_attention_ws_floats(B, heads, int(T), Tp))
    ws = torch.empty(max(nws, 1), device=qkv.device, dtype=torch.float32)
    _lib.check(lib.fsmi_vit_attention(_p(qkv), _p(out), B, heads, hd, int(T), Tp, float(scale), _p(ws), nws,
                                      _stream(qkv)), "vit_attention")
    return out


def space_to_depth(x: Tensor, k: int) -> Tensor:
    """(B, C, H, W) -> (B, C*k*k, H/k, W/k), channel (c*k + ky)*k + kx: a stride == kernel conv's im2col."""
    _check("space_to_depth", x)
    B, C, H, W = x.shape
    x = _c(x)
    out = torch.empty((B, C * k * k, H // k, W // k), device=x.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_space_to_depth(_p(x), _p(out), B, C, H, W, k, _stream(x)), "space_to_depth")
    return out


def depth_to_space(x: Tensor, k: int) -> Tensor:
    """(B, k*k*C, H, W) with channel (ky*k + kx)*C + c -> (B, C, H*k, W*k)."""
    _check("depth_to_space", x)
    B, CK, H, W = x.shape
    assert CK % (k * k) == 0
    C = CK // (k * k)
    x = _c(x)
    out = torch.empty((B, C, H * k, W * k), device=x.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_depth_to_space(_p(x), _p(out), B, C, H, W, k, _stream(x)), "depth_to_space")
    return out


def vit_tokens(emb: Tensor, cls: Tensor, pos: Tensor, Tp: int) -> Tensor:
    """[patch embeddings; class token; 0 ...] + position embedding -> (B, C, Tp) (patches first)."""
    _check("vit_tokens", emb, cls, pos)
    B, C = emb.shape[:2]
    emb = _c(emb)
    N = emb[0, 0].numel()
    assert cls.numel() == C and tuple(pos.shape) == (C, Tp), f"vit_tokens: pos {tuple(pos.shape)} for ({C}, {Tp})"
    cls, pos = _c(cls), _c(pos)
    out = torch.empty((B, C, Tp), device=emb.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_vit_tokens(_p(emb), _p(cls), _p(pos), _p(out), B, C, N, Tp, _stream(emb)),
               "vit_tokens")
    return out


def resize_bicubic(x: Tensor, size) -> Tensor:
    """``F.interpolate(x, size, mode="bicubic", align_corners=False)`` (core/extractor.py:352)."""
    _check("resize_bicubic", x)
    B, C, Hi, Wi = x.shape
    Ho, Wo = size
    x = _c(x)
    out = torch.empty((B, C, Ho, Wo), device=x.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_resize_bicubic(_p(x), _p(out), B, C, Hi, Wi, Ho, Wo, _stream(x)), "resize_bicubic")
    return out


_IN_ACT = {None: 0, "none": 0, "relu": 1, "leaky": 6}


def instance_norm(x: Tensor, act=None, res: Tensor = None, act2=None, eps: float = 1e-5, out: Tensor = None) -> Tensor:
    """``act2(act(InstanceNorm2d(x)) + res)`` (no affine, biased variance) per (b, c) plane."""
    _check("instance_norm", x, *([res] if res is not None else []))
    x = _c(x)
    B, C = x.shape[:2]
    HW = x[0, 0].numel()
    if res is not None:
        res = _c(res)
        assert res.shape == x.shape
    out = torch.empty_like(x) if out is None else out
    _lib.check(_lib.load().fsmi_instance_norm(_p(x), _p(res) if res is not None else None, _p(out), B * C, HW,
                                              float(eps), _IN_ACT[act], _IN_ACT[act2], _stream(x)), "instance_norm")
    return out


_EW = {"add": 0, "relu": 1, "add_relu": 2, "mul": 3}


def elementwise(a: Tensor, b: Tensor = None, op: str = "add", broadcast: bool = False, out: Tensor = None) -> Tensor:
    """``a + b`` / ``relu(a)`` / ``relu(a + b)`` / ``a * b``; ``broadcast``: b holds one image, repeated
    over a's batch."""
    _check("elementwise", a, *([b] if b is not None else []))
    a = _c(a)
    bper = 0
    if b is not None:
        b = _c(b)
        if broadcast:
            bper = b.numel()
            assert a.numel() % bper == 0
        else:
            assert b.numel() == a.numel()
    out = torch.empty_like(a) if out is None else out
    _lib.check(_lib.load().fsmi_elementwise(_p(a), _p(b) if b is not None else None, _p(out), a.numel(), bper,
                                            _EW[op], _stream(a)), "elementwise")
    return out


def xca(qkv: Tensor, temperature: Tensor, heads: int) -> Tensor:
    """EdgeNeXt cross-covariance attention core on the channel-major qkv (B, 3C, H, W) -> (B, C, H, W)."""
    t = _c(temperature.detach().float().reshape(-1))
    _check("xca", qkv, t)
    B, C3 = qkv.shape[:2]
    C = C3 // 3
    qkv = _c(qkv)
    N = qkv[0, 0].numel()
    nws = _lib.load().fsmi_xca_workspace_floats(B, C, heads)
    ws = torch.empty(max(int(nws), 1), device=qkv.device, dtype=torch.float32)
    out = torch.empty((B, C) + tuple(qkv.shape[2:]), device=qkv.device, dtype=torch.float32)
    _lib.check(_lib.load().fsmi_xca(_p(qkv), _p(t), _p(ws), _p(out), B, C, heads, N, _stream(qkv)), "xca")
    return out


def dwconv2d_ex(x, w: Tensor, bias: Tensor = None, add=None, out=None) -> Tensor:
    """Depthwise KSxKS conv (KS 3/5/7/9, 'same') on channel slices: ``x`` / ``add`` / ``out`` are tensors
    or (tensor, c0, n) slices of contiguous NCHW maps; out = conv(x + add) + bias."""
    def sl(s):
        return (s, 0, s.shape[1]) if isinstance(s, torch.Tensor) else s
    xt, xc0, C = sl(x)
    _check("dwconv2d_ex", xt, w, *([bias] if bias is not None else []))
    B, Cx, H, W = xt.shape
    KS = w.shape[-1]
    assert w.shape == (C, 1, KS, KS) and xt.is_contiguous(), f"dwconv2d_ex: weight {tuple(w.shape)} for {C} channels"
    if add is not None:
        at, ac0, an = sl(add)
        assert an == C and at.is_contiguous() and at.shape[2:] == (H, W)
        _check("dwconv2d_ex", at)
    if out is None:
        out = (torch.empty((B, C, H, W), device=xt.device, dtype=torch.float32), 0, C)
    ot, oc0, on = sl(out)
    assert on == C and ot.is_contiguous() and ot.shape[2:] == (H, W)
    HW = H * W
    w = _c(w.detach().float())
    b = _c(bias.detach().float()) if bias is not None else None
    _lib.check(_lib.load().fsmi_dwconv2d_ex(
        _p(xt) + 4 * xc0 * HW, Cx, (_p(at) + 4 * ac0 * HW) if add is not None else None,
        at.shape[1] if add is not None else C, _p(w), _p(b) if b is not None else None, _p(ot) + 4 * oc0 * HW,
        ot.shape[1], B, C, KS, H, W, _stream(xt)), "dwconv2d_ex")
    return ot
