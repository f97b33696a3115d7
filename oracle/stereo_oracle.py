"""Functional fp32 CPU restatement of the FoundationStereo hot path.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Every function is written from the reference's math, not its code, and cites
the reference ``file:line`` it restates.  Parameters are looked up by their
reference ``state_dict`` name in a flat dict ``P`` so the oracle, the product
modules and the reference module tree share one set of weights.

Reference root: TongZhe2016/FoundationStereo (snapshot 2025-06-29).
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
Params = Dict[str, Tensor]

__all__ = [
    "groupwise_correlation", "build_gwc_volume", "build_concat_volume",
    "disparity_regression", "context_upsample", "allpairs_corr",
    "GeoEncoding", "geo_lookup_naive", "oracle_forward", "oracle_hierarchical", "input_pad", "StageTimer",
]

_BN_EPS = 1e-5
_IN_EPS = 1e-5
_LN_EPS = 1e-5


# ----------------------------------------------------------------------------
# a1/a2: cost volumes  (core/submodule.py:388-427)
# ----------------------------------------------------------------------------

def _l2n(x: Tensor, dim: int) -> Tensor:
    # F.normalize: x / max(||x||_2, 1e-12)   (core/submodule.py:395)
    return x / x.norm(dim=dim, keepdim=True).clamp_min(1e-12)


def groupwise_correlation(f1: Tensor, f2: Tensor, G: int) -> Tensor:
    """core/submodule.py:388-397: mean-free group dot of L2-normalised groups."""
    B, C, H, W = f1.shape
    assert C % G == 0, f"C:{C}, num_groups:{G}"
    a = _l2n(f1.float().view(B, G, C // G, H, W), 2)
    b = _l2n(f2.float().view(B, G, C // G, H, W), 2)
    return (a * b).sum(2)


def build_gwc_volume(fl: Tensor, fr: Tensor, D: int, G: int) -> Tensor:
    """core/submodule.py:399-412.  V[b,g,d,h,w] = <nL(w), nR(w-d)>_g for w>=d, else 0.

    Normalisation is per pixel, so normalising once and shifting is the same
    value as the reference's per-slice re-normalisation (SURVEY App.A item 1).
    """
    B, C, H, W = fl.shape
    assert C % G == 0, f"C:{C}, num_groups:{G}"
    a = _l2n(fl.float().view(B, G, C // G, H, W), 2)
    b = _l2n(fr.float().view(B, G, C // G, H, W), 2)
    vol = fl.new_zeros((B, G, D, H, W), dtype=torch.float32)
    for d in range(D):
        if d == 0:
            vol[:, :, 0] = (a * b).sum(2)
        else:
            vol[:, :, d, :, d:] = (a[..., d:] * b[..., :-d]).sum(2)
    return vol


def build_concat_volume(pl: Tensor, pr: Tensor, D: int) -> Tensor:
    """core/submodule.py:416-427: left copied for ALL w, right shifted and zero for w<d."""
    B, C, H, W = pl.shape
    vol = pl.new_zeros((B, 2 * C, D, H, W))
    vol[:, :C] = pl.unsqueeze(2)
    for d in range(D):
        if d == 0:
            vol[:, C:, 0] = pr
        else:
            vol[:, C:, d, :, d:] = pr[..., :-d]
    return vol


def disparity_regression(prob: Tensor, D: int) -> Tensor:
    """core/submodule.py:431-435: sum_d d * p_d (keepdim)."""
    assert prob.dim() == 4
    dv = torch.arange(D, dtype=prob.dtype).view(1, D, 1, 1)
    return (prob * dv).sum(1, keepdim=True)


def context_upsample(disp_low: Tensor, w: Tensor) -> Tensor:
    """core/submodule.py:456-468: convex 3x3 combination, nearest x4."""
    b, _, h, ww = disp_low.shape
    nb = F.unfold(disp_low, 3, 1, 1).view(b, 9, h, ww)
    nb = nb.repeat_interleave(4, dim=2).repeat_interleave(4, dim=3)   # == nearest x4
    return (nb * w).sum(1)


# ----------------------------------------------------------------------------
# a5/a6: geometry encoding + lookup  (core/geometry.py, core/utils/utils.py)
# ----------------------------------------------------------------------------

def allpairs_corr(f1: Tensor, f2: Tensor) -> Tensor:
    """core/geometry.py:68-77: corr[b,h,w1,w2] = <f1/|f1|, f2/|f2|> over all C."""
    a = _l2n(f1.float(), 1)
    b = _l2n(f2.float(), 1)
    return torch.einsum("bchx,bchy->bhxy", a, b)


def _pool_last(x: Tensor) -> Tensor:
    # avg_pool2d([1,2], stride [1,2]) over the last axis, floor  (core/geometry.py:35,39)
    n = x.shape[-1] // 2
    return (x[..., 0:2 * n:2] + x[..., 1:2 * n:2]) / 2


def _sample_1d(v: Tensor, x: Tensor) -> Tensor:
    """grid_sample(align_corners=True, zeros) along the last axis of ``v``.

    ``v``: (P, C, Lx); ``x``: (P, K) pixel coordinates -> (P, C, K).
    Restates core/utils/utils.py:44-55 including the [-1,1] round trip.
    """
    Lx = v.shape[-1]
    xn = 2 * x / (Lx - 1) - 1
    ix = ((xn + 1) / 2) * (Lx - 1)
    x0 = torch.floor(ix)
    w1 = ix - x0
    w0 = 1 - w1
    i0 = x0.long()
    i1 = i0 + 1
    P, C, _ = v.shape
    out = torch.zeros(P, C, x.shape[1], dtype=v.dtype)
    for idx, wt in ((i0, w0), (i1, w1)):
        ok = (idx >= 0) & (idx < Lx)
        g = torch.gather(v, 2, idx.clamp(0, Lx - 1).unsqueeze(1).expand(P, C, -1))
        out = out + g * (wt * ok).unsqueeze(1)
    return out


class GeoEncoding:
    """core/geometry.py:17-65 (Combined_Geo_Encoding_Volume) on the CPU."""

    def __init__(self, f1: Tensor, f2: Tensor, vol: Tensor, num_levels: int = 2, radius: int = 4):
        self.L = num_levels
        self.dx = torch.linspace(-radius, radius, 2 * radius + 1)          # core/foundation_stereo.py:179
        corr = allpairs_corr(f1, f2)                                        # (B,H,W1,W2)
        B, C, D, H, W = vol.shape
        self.shape = (B, H, W)
        g = vol.float().permute(0, 3, 4, 1, 2).reshape(B * H * W, C, D)    # core/geometry.py:29
        c = corr.reshape(B * H * W, 1, -1)
        self.geo = [g]
        self.cor = [c]
        for _ in range(num_levels - 1):
            g = _pool_last(g)
            self.geo.append(g)
        for _ in range(num_levels - 1):
            c = _pool_last(c)
            self.cor.append(c)

    def __call__(self, disp: Tensor, coords: Tensor) -> Tensor:
        B, H, W = self.shape
        P = B * H * W
        d = disp.reshape(P, 1).float()
        cx = coords.reshape(P, 1).float()
        outs = []
        for i in range(self.L):
            s = 2 ** i
            x_geo = self.dx.view(1, -1) + d / s                              # core/geometry.py:49
            x_cor = cx / s - d / s + self.dx.view(1, -1)                     # core/geometry.py:57
            gv = _sample_1d(self.geo[i], x_geo)                              # (P, Cv, K)
            cv = _sample_1d(self.cor[i], x_cor)                              # (P, 1, K)
            outs.append(gv.reshape(B, H, W, -1))
            outs.append(cv.reshape(B, H, W, -1))
        return torch.cat(outs, -1).permute(0, 3, 1, 2).contiguous()        # core/geometry.py:64-65


def geo_lookup_naive(vol: Tensor, corr: Tensor, disp: Tensor, L: int, r: int) -> Tensor:
    """Scalar-loop restatement of the lookup for tiny shapes (cross-checks GeoEncoding).

    vol (B,C,D,H,W) filtered volume, corr (B,H,W,W2) all-pairs corr, disp (B,1,H,W).
    """
    B, C, D, H, W = vol.shape
    W2 = corr.shape[-1]
    K = 2 * r + 1
    out = torch.zeros(B, L * K * (C + 1), H, W)
    geo = [vol.double()]
    cor = [corr.double()]
    for _ in range(L - 1):
        geo.append(_pool_last(geo[-1].permute(0, 1, 3, 4, 2)).permute(0, 1, 4, 2, 3))
        cor.append(_pool_last(cor[-1]))

    def lin(row, x):
        n = len(row)
        x0 = math.floor(x)
        f = x - x0
        v = 0.0
        if 0 <= x0 < n:
            v += row[x0] * (1 - f)
        if 0 <= x0 + 1 < n:
            v += row[x0 + 1] * f
        return v

    for b in range(B):
        for h in range(H):
            for w in range(W):
                dd = float(disp[b, 0, h, w])
                base = 0
                for i in range(L):
                    s = 2.0 ** i
                    for c in range(C):
                        row = geo[i][b, c, :, h, w].tolist()
                        for k in range(K):
                            out[b, base + c * K + k, h, w] = lin(row, dd / s + (k - r))
                    crow = cor[i][b, h, w].tolist()
                    for k in range(K):
                        out[b, base + C * K + k, h, w] = lin(crow, w / s - dd / s + (k - r))
                    base += K * (C + 1)
    return out


# ----------------------------------------------------------------------------
# Layer helpers keyed by reference state_dict names
# ----------------------------------------------------------------------------

def _conv(P: Params, name: str, x: Tensor, stride=1, padding=0, groups=1) -> Tensor:
    w = P[name + ".weight"]
    b = P.get(name + ".bias")
    fn = {3: F.conv1d, 4: F.conv2d, 5: F.conv3d}[w.dim()]
    return fn(x, w, b, stride, padding, 1, groups)


def _deconv(P: Params, name: str, x: Tensor, stride, padding) -> Tensor:
    w = P[name + ".weight"]
    b = P.get(name + ".bias")
    fn = F.conv_transpose3d if w.dim() == 5 else F.conv_transpose2d
    return fn(x, w, b, stride, padding)


def _bn(P: Params, name: str, x: Tensor) -> Tensor:
    return F.batch_norm(x, P[name + ".running_mean"], P[name + ".running_var"],
                        P[name + ".weight"], P[name + ".bias"], False, 0.0, _BN_EPS)


def _inorm(x: Tensor) -> Tensor:
    # nn.InstanceNorm{2,3}d defaults: affine=False, no running stats
    dims = tuple(range(2, x.dim()))
    mu = x.mean(dims, keepdim=True)
    var = x.var(dims, unbiased=False, keepdim=True)
    return (x - mu) / torch.sqrt(var + _IN_EPS)


def _lrelu(x: Tensor) -> Tensor:
    return F.leaky_relu(x, 0.01)  # nn.LeakyReLU() default slope (core/submodule.py:85)


def basic_conv(P, name, x, *, deconv=False, bn=True, relu=True, norm="batch", stride=1, padding=0):
    """core/submodule.py:51-86 (conv no-bias -> BN/IN -> LeakyReLU)."""
    if deconv:
        x = _deconv(P, name + ".conv", x, stride, padding)
    else:
        x = _conv(P, name + ".conv", x, stride, padding)
    if bn:
        x = _bn(P, name + ".bn", x) if norm == "batch" else _inorm(x)
    return _lrelu(x) if relu else x


def basic_conv_in(P, name, x, stride=1, padding=0):
    """core/submodule.py:320-346 (conv -> InstanceNorm -> LeakyReLU)."""
    return _lrelu(_inorm(_conv(P, name + ".conv", x, stride, padding)))


def apc(P, name, x):
    """Conv3dNormActReduced, core/submodule.py:89-114: (1,3,3)+BN+ReLU then (17,1,1)+BN+ReLU."""
    x = F.relu(_bn(P, name + ".conv1.1", _conv(P, name + ".conv1.0", x, 1, (0, 1, 1))))
    kd = P[name + ".conv2.0.weight"].shape[2]
    return F.relu(_bn(P, name + ".conv2.1", _conv(P, name + ".conv2.0", x, 1, (kd // 2, 0, 0))))


def resblock3d(P, name, x):
    """ResnetBasicBlock3D, core/submodule.py:159-195."""
    y = F.relu(_bn(P, name + ".bn1", _conv(P, name + ".conv1", x, 1, 1)))
    y = _bn(P, name + ".bn2", _conv(P, name + ".conv2", y, 1, 1))
    return F.relu(y + x)


def resblock2d(P, name, x, stride=1):
    """core/extractor.py:20-80 with norm_fn='batch' (convs carry bias)."""
    y = F.relu(_bn(P, name + ".norm1", _conv(P, name + ".conv1", x, stride, 1)))
    y = F.relu(_bn(P, name + ".norm2", _conv(P, name + ".conv2", y, 1, 1)))
    if (name + ".downsample.0.weight") in P:
        x = _bn(P, name + ".downsample.1", _conv(P, name + ".downsample.0", x, stride, 0))
    return F.relu(x + y)


def feature_att(P, name, cv, feat):
    """FeatureAtt, core/submodule.py:438-454: sigmoid(conv1x1(LReLU(BN(conv1x1 feat)))) * cv."""
    a = basic_conv(P, name + ".feat_att.0", feat)
    a = _conv(P, name + ".feat_att.1", a)
    return torch.sigmoid(a).unsqueeze(2) * cv


def _positional(d_model: int, max_len: int) -> Tensor:
    """PositionalEmbedding table, core/submodule.py:472-488."""
    pe = torch.zeros(max_len, d_model)
    pos = torch.arange(0, max_len).float().unsqueeze(1)
    div = (torch.arange(0, d_model, 2).float() * -(math.log(10000.0) / d_model)).exp()[None]
    pe[:, 0::2] = torch.sin(pos * div)
    pe[:, 1::2] = torch.cos(pos * div)
    return pe


def _linear(P, name, x):
    return F.linear(x, P[name + ".weight"], P.get(name + ".bias"))


def _layernorm(P, name, x):
    return F.layer_norm(x, (x.shape[-1],), P[name + ".weight"], P[name + ".bias"], _LN_EPS)


def disparity_transformer(P, name, cv, max_len, nhead=4):
    """CostVolumeDisparityAttention, core/submodule.py:198-257,506-528 (post-norm, eval)."""
    B, C, D, H, W = cv.shape
    x = cv.permute(0, 3, 4, 2, 1).reshape(B * H * W, D, C)
    if D > max_len:
        raise RuntimeError(f"x:{tuple(x.shape)}, pe:(1, {max_len}, {C})")
    x = x + _positional(C, max_len)[:D].unsqueeze(0)
    hd = C // nhead
    i = 0
    while (f"{name}.sa.{i}.norm1.weight") in P:
        p = f"{name}.sa.{i}"
        q = _linear(P, p + ".self_attn.q_proj", x).view(-1, D, nhead, hd).transpose(1, 2)
        k = _linear(P, p + ".self_attn.k_proj", x).view(-1, D, nhead, hd).transpose(1, 2)
        v = _linear(P, p + ".self_attn.v_proj", x).view(-1, D, nhead, hd).transpose(1, 2)
        att = torch.softmax((q @ k.transpose(-1, -2)) / math.sqrt(hd), -1) @ v  # flash_attn_func, non-causal
        att = _linear(P, p + ".self_attn.out_proj", att.transpose(1, 2).reshape(-1, D, C))
        x = _layernorm(P, p + ".norm1", x + att)
        ff = _linear(P, p + ".linear2", F.gelu(_linear(P, p + ".linear1", x)))
        x = _layernorm(P, p + ".norm2", x + ff)
        i += 1
    return x.reshape(B, H, W, D, C).permute(0, 4, 3, 1, 2)


def hourglass(P, name, x, feats, max_disp):
    """core/foundation_stereo.py:45-123."""
    n = name
    c1 = basic_conv(P, n + ".conv1.0", x, stride=2, padding=1)
    c1 = apc(P, n + ".conv1.1", c1)
    c1 = feature_att(P, n + ".feature_att_8", c1, feats[1])
    c2 = apc(P, n + ".conv2.1", basic_conv(P, n + ".conv2.0", c1, stride=2, padding=1))
    c2 = feature_att(P, n + ".feature_att_16", c2, feats[2])
    c3 = apc(P, n + ".conv3.1", basic_conv(P, n + ".conv3.0", c2, stride=2, padding=1))
    c3 = feature_att(P, n + ".feature_att_32", c3, feats[3])
    c3u = basic_conv(P, n + ".conv3_up", c3, deconv=True, stride=2, padding=1)
    c2 = torch.cat([c3u, c2], 1)
    c2 = basic_conv(P, n + ".agg_0.0", c2)
    c2 = apc(P, n + ".agg_0.2", apc(P, n + ".agg_0.1", c2))
    c2 = feature_att(P, n + ".feature_att_up_16", c2, feats[2])
    c2u = basic_conv(P, n + ".conv2_up", c2, deconv=True, stride=2, padding=1)
    c1 = torch.cat([c2u, c1], 1)
    c1 = basic_conv(P, n + ".agg_1.0", c1)
    c1 = apc(P, n + ".agg_1.2", apc(P, n + ".agg_1.1", c1))
    c1 = feature_att(P, n + ".feature_att_up_8", c1, feats[1])
    conv = basic_conv(P, n + ".conv1_up", c1, deconv=True, stride=2, padding=1)
    xp = _bn(P, n + ".conv_patch.1", _conv(P, n + ".conv_patch.0", x, 4, 0, groups=x.shape[1]))
    xp = disparity_transformer(P, n + ".atts.4", xp, max_disp // 16)
    xp = F.interpolate(xp, scale_factor=4, mode="trilinear", align_corners=False)
    conv = conv + xp
    return apc(P, n + ".conv_out.1", apc(P, n + ".conv_out.0", conv))


# ----------------------------------------------------------------------------
# Context path (stock PyTorch in the product; restated here for the E2E oracle)
# ----------------------------------------------------------------------------

def context_net(P, name, img, vit_feat, n_downsample=2):
    """ContextNetDino.forward, core/extractor.py:262-283 (norm_fn='batch')."""
    x = _conv(P, name + ".conv1", img, 1 + (n_downsample > 2), 3)
    x = F.relu(_bn(P, name + ".norm1", x))
    strides = {1: 1, 2: 1 + (n_downsample > 1), 3: 1 + (n_downsample > 0), 4: 2, 5: 2}
    for li in (1, 2, 3):
        x = resblock2d(P, f"{name}.layer{li}.0", x, strides[li])
        x = resblock2d(P, f"{name}.layer{li}.1", x, 1)
    x = torch.cat([x, vit_feat], 1)
    x = basic_conv(P, name + ".conv2", x, padding=1)

    def heads(prefix, t, res):
        outs = []
        j = 0
        while f"{name}.{prefix}.{j}.0.conv1.weight" in P or f"{name}.{prefix}.{j}.weight" in P:
            if res:
                y = resblock2d(P, f"{name}.{prefix}.{j}.0", t)
                outs.append(_conv(P, f"{name}.{prefix}.{j}.1", y, 1, 1))
            else:
                outs.append(_conv(P, f"{name}.{prefix}.{j}", t, 1, 1))
            j += 1
        return outs

    o4 = heads("outputs04", x, True)
    y = x
    for li in (4,):
        y = resblock2d(P, f"{name}.layer{li}.0", y, 2)
        y = resblock2d(P, f"{name}.layer{li}.1", y, 1)
    o8 = heads("outputs08", y, True)
    z = resblock2d(P, f"{name}.layer5.0", y, 2)
    z = resblock2d(P, f"{name}.layer5.1", z, 1)
    o16 = heads("outputs16", z, False)
    return o4, o8, o16


def channel_att(P, name, x):
    """ChannelAttentionEnhancement, core/submodule.py:532-547."""
    def fc(t):
        return _conv(P, name + ".fc.2", F.relu(_conv(P, name + ".fc.0", t)))
    return torch.sigmoid(fc(x.mean((2, 3), keepdim=True)) + fc(x.amax((2, 3), keepdim=True)))


def spatial_att(P, name, x):
    """SpatialAttentionExtractor, core/submodule.py:549-561."""
    t = torch.cat([x.mean(1, keepdim=True), x.amax(1, keepdim=True)], 1)
    return torch.sigmoid(_conv(P, name + ".samconv", t, 1, 3))


# ----------------------------------------------------------------------------
# a7: refinement update block  (core/update.py)
# ----------------------------------------------------------------------------

def _pool2x(x):
    return F.avg_pool2d(x, 3, stride=2, padding=1)          # core/update.py:72-73


def _interp(x, dest):
    return F.interpolate(x, dest.shape[2:], mode="bilinear", align_corners=True)   # :78-80


def raft_gru(P, name, h, x, hx, k):
    """RaftConvGRU, core/update.py:83-95."""
    z = torch.sigmoid(_conv(P, name + ".convz", hx, 1, k // 2))
    r = torch.sigmoid(_conv(P, name + ".convr", hx, 1, k // 2))
    q = torch.tanh(_conv(P, name + ".convq", torch.cat([r * h, x], 1), 1, k // 2))
    return (1 - z) * h + z * q


def selective_gru(P, name, att, h, *xs):
    """SelectiveConvGRU, core/update.py:98-119."""
    x = F.relu(_conv(P, name + ".conv0.0", torch.cat(xs, 1), 1, 1))
    hx = F.relu(_conv(P, name + ".conv1.0", torch.cat([x, h], 1), 1, 1))
    return raft_gru(P, name + ".small_gru", h, x, hx, 1) * att + raft_gru(P, name + ".large_gru", h, x, hx, 3) * (1 - att)


def edgenext_block(P, name, x):
    """EdgeNextConvEncoder(norm=None), core/submodule.py:565-591."""
    C = x.shape[1]
    y = _conv(P, name + ".dwconv", x, 1, P[name + ".dwconv.weight"].shape[-1] // 2, groups=C)
    y = y.permute(0, 2, 3, 1)
    y = _linear(P, name + ".pwconv2", F.gelu(_linear(P, name + ".pwconv1", y)))
    y = P[name + ".gamma"] * y
    return x + y.permute(0, 3, 1, 2)


def update_block(P, name, net, inp, corr, disp, att, n_gru_layers=3):
    """BasicSelectiveMultiUpdateBlock.forward, core/update.py:141-159 (3 GRU levels)."""
    net = list(net)
    net[2] = selective_gru(P, name + ".gru16", att[2], net[2], inp[2], _pool2x(net[1]))
    net[1] = selective_gru(P, name + ".gru08", att[1], net[1], inp[1], _pool2x(net[0]), _interp(net[2], net[1]))
    e = name + ".encoder"                                                    # core/update.py:62-70
    cor = F.relu(_conv(P, e + ".convc1", corr))
    cor = F.relu(_conv(P, e + ".convc2", cor, 1, 1))
    dsp = F.relu(_conv(P, e + ".convd1", disp, 1, 3))
    dsp = F.relu(_conv(P, e + ".convd2", dsp, 1, 1))
    mot = torch.cat([F.relu(_conv(P, e + ".conv", torch.cat([cor, dsp], 1), 1, 1)), disp], 1)
    mot = torch.cat([inp[0], mot], 1)
    net[0] = selective_gru(P, name + ".gru04", att[0], net[0], mot, _interp(net[1], net[0]))
    hd = name + ".disp_head.conv"                                            # core/update.py:20-32
    y = F.relu(_conv(P, hd + ".0", net[0], 1, 1))
    y = edgenext_block(P, hd + ".2", y)
    y = edgenext_block(P, hd + ".3", y)
    delta = _conv(P, hd + ".4", y, 1, 1)
    m = F.relu(_conv(P, name + ".mask.0", net[0], 1, 1))
    m = F.relu(_conv(P, name + ".mask.2", m, 1, 1))
    return net, 0.25 * m, delta


# ----------------------------------------------------------------------------
# Full forward (minus backbone)
# ----------------------------------------------------------------------------

class StageTimer:
    """Wall-clock accumulator for the per-stage CPU-baseline split."""

    def __init__(self):
        import time
        self._t = time.perf_counter
        self.stages: Dict[str, float] = {}
        self._last = None
        self._name = None

    def mark(self, name=None):
        now = self._t()
        if self._name is not None:
            self.stages[self._name] = self.stages.get(self._name, 0.0) + now - self._last
        self._name, self._last = name, now


def oracle_forward(P: Params, args, image1: Tensor, image2: Tensor,
                   feats_left: Sequence[Tensor], feats_right: Sequence[Tensor], vit_feat: Tensor,
                   iters: int = 12, init_disp: Tensor = None, timer: StageTimer = None,
                   return_aux: bool = False):
    """FoundationStereo.forward(test_mode=True), core/foundation_stereo.py:194-254.

    The backbone output (``feats_left/right``, ``vit_feat``) is an input: the
    synthetic source replaces ``self.feature``.
    """
    T = timer or StageTimer()
    max_disp = args["max_disp"]
    D4 = max_disp // 4
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    im1 = ((image1 / 255.0) - mean) / std                                    # :37-42
    aux = {}

    T.mark("context")
    s = basic_conv_in(P, "stem_2.0", im1, stride=2, padding=1)              # :146-150,205
    s = F.relu(_inorm(_conv(P, "stem_2.1", s, 1, 1)))
    stem_2x = s

    T.mark("build")
    fl0, fr0 = feats_left[0].float(), feats_right[0].float()
    gwc = build_gwc_volume(fl0, fr0, D4, 8)                                  # :207
    pl = _conv(P, "proj_cmb", fl0)
    pr = _conv(P, "proj_cmb", fr0)
    comb = torch.cat([gwc, build_concat_volume(pl, pr, D4)], 1)              # :208-212

    T.mark("filter")
    v = _conv(P, "corr_stem.0", comb)                                        # :164-169
    v = basic_conv(P, "corr_stem.1", v, padding=1)
    v = resblock3d(P, "corr_stem.2", v)
    v = resblock3d(P, "corr_stem.3", v)
    v = feature_att(P, "corr_feature_att", v, fl0)                           # :214
    v = hourglass(P, "cost_agg", v, feats_left, max_disp)                    # :215
    logit = basic_conv(P, "classifier.0", v, padding=1)                      # :172-176
    logit = resblock3d(P, "classifier.1", logit)
    logit = _conv(P, "classifier.2", logit, 1, 3).squeeze(1)
    prob = torch.softmax(logit, 1)                                           # :218
    if init_disp is None:
        init_disp = disparity_regression(prob, D4)                          # :220
    aux["init_disp"] = init_disp

    T.mark("context")
    cl = context_net(P, "cnet", im1, vit_feat, args.get("n_downsample", 2))  # :222
    net = [torch.tanh(cl[i][0]) for i in range(3)]
    inp = [F.relu(cl[i][1]) for i in range(3)]
    inp = [channel_att(P, "cam", x) * x for x in inp]
    att = [spatial_att(P, "sam", x) for x in inp]

    T.mark("geo_init")
    geo = GeoEncoding(fl0, fr0, v, args["corr_levels"], args["corr_radius"])  # :229
    B, _, H, W = fl0.shape
    coords = torch.arange(W, dtype=torch.float).view(1, 1, W, 1).repeat(B, H, 1, 1)
    disp = init_disp.float()
    mask = None
    for itr in range(iters):
        T.mark("lookup")
        gf = geo(disp, coords)                                               # :238
        if itr == 0:
            aux["geo_feat0"] = gf
        T.mark("gru")
        net, mask, delta = update_block(P, "update_block", net, inp, gf, disp, att)   # :240
        disp = disp + delta.float()                                          # :242
    T.mark("upsample")
    x = _lrelu(_deconv(P, "spx_2_gru.conv1.conv", mask, 2, 1))              # :183-191
    if x.shape != stem_2x.shape:
        x = F.interpolate(x, size=stem_2x.shape[-2:], mode="bilinear")
    x = _lrelu(_conv(P, "spx_2_gru.conv2.conv", torch.cat([x, stem_2x], 1), 1, 1))
    spx = torch.softmax(_deconv(P, "spx_gru.0", x, 2, 1), 1)
    up = context_upsample(disp * 4.0, spx).unsqueeze(1)
    T.mark(None)
    aux["disp_low"] = disp
    return (up, aux) if return_aux else up


def input_pad(ht: int, wd: int, divis_by: int = 32):
    """InputPadder(dims, mode='sintel', force_square=False)._pad, core/utils/utils.py:19-31:
    [left, right, top, bottom] replicate padding up to the next multiple of ``divis_by``."""
    pad_ht = (((ht // divis_by) + 1) * divis_by - ht) % divis_by
    pad_wd = (((wd // divis_by) + 1) * divis_by - wd) % divis_by
    return [pad_wd // 2, pad_wd - pad_wd // 2, pad_ht // 2, pad_ht - pad_ht // 2]


def _unpad(x: Tensor, pad) -> Tensor:
    """InputPadder.unpad, core/utils/utils.py:37-41."""
    ht, wd = x.shape[-2:]
    return x[..., pad[2]:ht - pad[3], pad[0]:wd - pad[1]]


def oracle_hierarchical(P: Params, args, image1: Tensor, image2: Tensor, features, iters: int = 12,
                        small_ratio: float = 0.5, timer: StageTimer = None, return_aux: bool = False):
    """FoundationStereo.run_hierachical(test_mode=True), core/foundation_stereo.py:257-274.

    ``features(B, H, W)`` -> ``(feats_left, feats_right, vit_feat)`` is the backbone stand-in at a
    padded pass resolution (the reference calls ``self.feature`` inside each ``forward``).  Kept
    as in the reference: bilinear x``small_ratio`` downscale (align_corners False), the coarse
    pass at the /32-padded small size, unpad, bilinear upsample (align_corners True) scaled by
    1/small_ratio and clipped at 0, the ``+= _pad[0]`` on the padded init (``:270``, the
    reference adds the LEFT pad to the disparity value), x0.25 bilinear downscale of it as the
    1/4-resolution ``init_disp``, then the fine pass -- whose classifier + soft-argmin are still
    computed and discarded (``:218-220``)."""
    B, _, H, W = image1.shape
    s1 = F.interpolate(image1, scale_factor=small_ratio, align_corners=False, mode="bilinear")
    s2 = F.interpolate(image2, scale_factor=small_ratio, align_corners=False, mode="bilinear")
    pad = input_pad(*s1.shape[-2:])
    s1, s2 = (F.pad(x, pad, mode="replicate") for x in (s1, s2))
    fl, fr, vf = features(B, *s1.shape[-2:])
    d_small = oracle_forward(P, args, s1, s2, fl, fr, vf, iters=iters, timer=timer)
    d_small = _unpad(d_small.float(), pad)
    up = F.interpolate(d_small, size=(H, W), mode="bilinear", align_corners=True) * 1 / small_ratio
    up = up.clip(0, None)
    pad = input_pad(H, W)
    image1, image2, up = (F.pad(x, pad, mode="replicate") for x in (image1, image2, up))
    up = up + pad[0]
    init_disp = F.interpolate(up, scale_factor=0.25, mode="bilinear", align_corners=True) * 0.25
    fl, fr, vf = features(B, *image1.shape[-2:])
    disp = oracle_forward(P, args, image1, image2, fl, fr, vf, iters=iters, init_disp=init_disp, timer=timer)
    disp = _unpad(disp.float(), pad)
    if return_aux:
        return disp, {"disp_small": d_small, "init_disp": init_disp}
    return disp
