"""GPU parity of the backbone on the HIP kernels.

* kernels vs fp64 torch: channel LayerNorm, multi-head attention (masked padding, both block shapes),
  space-to-depth / depth-to-space, bicubic resize, InstanceNorm (+ act, + residual), elementwise,
  cross-covariance attention, depthwise k3..k9 on channel slices with a fused add;
* DepthAnythingFeature (ViT-S, ViT-L) vs the REFERENCE goldens (tools/make_goldens.py backbone) and
  vs the CPU oracle at a larger size;
* Feature (EdgeNeXt-S + DepthAnythingV2 + fusion) vs the reference golden and the oracle;
* FoundationStereo with the real backbone end to end vs the oracle (< 1e-3 px);
* the product backbone path never falls back to torch.nn convs / SDPA (patched to raise).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import oracle
from foundationstereo_amd import backbone as bb, ops, synth
from oracle import backbone_oracle as bo
from tests.helpers import load_golden, t

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from foundationstereo_amd import _lib
    return _lib.load()


def _rand(shape, seed, std=1.0):
    return t(synth.normal(synth.name_seed(f"bbt{seed}"), shape, std))


def _err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max()), float(b.abs().max())


def _close(a, b, rel=2e-5, abs_=1e-5, what=""):
    e, m = _err(a, b)
    assert e <= abs_ + rel * m, f"{what}: max |diff| {e:.3g} vs max |ref| {m:.3g}"
    return e


# ---------------------------------------------------------------- kernels

@pytest.mark.parametrize("C,T,n,off", [(384, 256, 256, 0), (1024, 1984, 1921, 0), (48, 700, 699, 0), (384, 192, 1, 150)])
def test_channel_layernorm(C, T, n, off):
    x = _rand((2, C, T), 1, 3.0) + 0.5
    w, b = _rand((C,), 2, 0.3) + 1, _rand((C,), 3, 0.1)
    out = ops.channel_layernorm(x.to(DEV), w.to(DEV), b.to(DEV), 1e-6, n=n, x_offset=off)
    ref = F.layer_norm(x.double()[:, :, off:off + n].transpose(1, 2), (C,), w.double(), b.double(), 1e-6).transpose(1, 2)
    _close(out, ref, what="layernorm")


def _sdpa_ref(qkv, heads, T, scale):
    B, C3, Tp = qkv.shape
    hd = C3 // (3 * heads)
    q, k, v = qkv.double().view(B, 3, heads, hd, Tp).unbind(1)          # (B, heads, hd, Tp)
    s = torch.einsum("bhdi,bhdj->bhij", q, k[..., :T]) * scale
    p = torch.softmax(s, -1)
    return torch.einsum("bhij,bhdj->bhdi", p, v[..., :T]).reshape(B, heads * hd, Tp)


# key ranges per (image, head, query tile) (fsmi_vit_attention_ws_floats > 0): 1 (64, 192), 2 (1x16 heads
# 1984, 4x16 704), 3 (2x6 heads 1984: ViT-S at cfg2), 6 (1x6 heads 1984)
@pytest.mark.parametrize("B,heads,T,Tp", [(2, 6, 21, 64), (2, 6, 150, 192), (1, 16, 1921, 1984), (4, 16, 700, 704),
                                          (2, 6, 1921, 1984), (1, 6, 1900, 1984)])
def test_vit_attention(B, heads, T, Tp):
    qkv = _rand((B, 3 * heads * 64, Tp), 4, 1.5)
    out = ops.vit_attention(qkv.to(DEV), heads, T, 0.125)
    _close(out, _sdpa_ref(qkv, heads, T, 0.125), rel=3e-6, abs_=3e-6, what="attention")


def test_vit_attention_peaked_scores():
    """Large logits (a near one-hot softmax) and small ones in the same rows."""
    qkv = _rand((1, 3 * 4 * 64, 128), 5, 1.0)
    qkv[:, :256] *= 6.0
    out = ops.vit_attention(qkv.to(DEV), 4, 100, 0.125)
    _close(out, _sdpa_ref(qkv, 4, 100, 0.125), rel=3e-6, abs_=3e-6, what="attention")


@pytest.mark.parametrize("k,C,H,W", [(14, 3, 56, 70), (4, 3, 64, 96), (2, 48, 16, 24)])
def test_space_to_depth(k, C, H, W):
    x = _rand((2, C, H, W), 6)
    out = ops.space_to_depth(x.to(DEV), k).cpu()
    ref = F.unfold(x, k, stride=k).view(2, C * k * k, H // k, W // k)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("k,C", [(4, 48), (2, 96)])
def test_deconv_as_depth_to_space(k, C):
    """ConvTranspose2d(k, stride k) = 1x1 conv with k*k*C outputs + depth-to-space."""
    x = _rand((2, 40, 5, 6), 7)
    dc = torch.nn.ConvTranspose2d(40, C, k, stride=k).eval()
    with torch.no_grad():
        dc.weight.copy_(_rand(tuple(dc.weight.shape), 8, 0.2))
        dc.bias.copy_(_rand((C,), 9, 0.1))
        ref = dc(x)
    dcd = dc.to(DEV)
    pk, b = bb._deconv_pack(dcd)
    with torch.no_grad():
        out = ops.depth_to_space(ops.conv2d([x.to(DEV)], pk, bias=b), k)
    _close(out, ref, what="deconv k=s")


@pytest.mark.parametrize("Hi,Wi,Ho,Wo", [(64, 96, 112, 112), (480, 640, 560, 672), (50, 30, 33, 71)])
def test_resize_bicubic(Hi, Wi, Ho, Wo):
    x = _rand((2, 3, Hi, Wi), 10, 2.0)
    out = ops.resize_bicubic(x.to(DEV), (Ho, Wo))
    # the reference runs it in fp32 (source coordinates from the fp32 in/out scale, one fma rounding):
    # agree with that to rounding; against the fp64 interpolation, be no further than the reference's
    # own fp32 result is (its fp32 source coordinate is off by up to an ulp of a few hundred pixels,
    # which on this noise moves outputs by up to ~5e-5 relative)
    ref32 = F.interpolate(x, size=(Ho, Wo), mode="bicubic", align_corners=False)
    _close(out, ref32, rel=5e-6, abs_=1e-6, what="bicubic vs fp32")
    ref = F.interpolate(x.double(), size=(Ho, Wo), mode="bicubic", align_corners=False)
    e32, _ = _err(ref32, ref)
    e, m = _err(out, ref)
    assert e <= 1.1 * e32 + 2e-6 * m, f"bicubic vs fp64: {e:.3g}, the reference's fp32 path {e32:.3g}"


@pytest.mark.parametrize("act,res,act2", [(None, False, None), ("leaky", False, None), ("relu", True, "relu"),
                                          (None, True, "relu")])
def test_instance_norm(act, res, act2):
    x = _rand((2, 24, 17, 33), 11, 2.0) + 1.0
    r = _rand((2, 24, 17, 33), 12)
    out = ops.instance_norm(x.to(DEV), act=act, res=r.to(DEV) if res else None, act2=act2)
    acts = {None: lambda v: v, "relu": F.relu, "leaky": lambda v: F.leaky_relu(v, 0.01)}
    ref = acts[act](F.instance_norm(x.double(), eps=1e-5))
    if res:
        ref = acts[act2](ref + r.double())
    _close(out, ref, what="instance norm")


def test_elementwise():
    a, b = _rand((2, 5, 7, 9), 13), _rand((1, 5, 7, 9), 14)
    ad, bd = a.to(DEV), b.to(DEV)
    assert torch.equal(ops.elementwise(ad, op="relu").cpu(), F.relu(a))
    assert torch.equal(ops.elementwise(ad, bd, "add", broadcast=True).cpu(), a + b)
    assert torch.equal(ops.elementwise(ad, ad, "add_relu").cpu(), F.relu(a + a))


@pytest.mark.parametrize("C,heads,N", [(96, 8, 4800), (304, 8, 300), (160, 8, 1200)])
def test_xca(C, heads, N):
    qkv = _rand((2, 3 * C, N), 15)
    temp = _rand((heads, 1, 1), 16, 0.5) + 1.0
    out = ops.xca(qkv.to(DEV), temp.to(DEV), heads)
    B, ch = 2, C // heads
    q, k, v = qkv.double().view(B, 3, heads, ch, N).unbind(1)
    q = q / q.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    k = k / k.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    a = torch.softmax(q @ k.transpose(-2, -1) * temp.double(), -1)
    _close(out, (a @ v).reshape(B, C, N), rel=3e-6, abs_=3e-6, what="xca")


@pytest.mark.parametrize("KS", [3, 5, 7, 9])
def test_dwconv_slices(KS):
    x = _rand((2, 40, 19, 70), 17)
    y = _rand((2, 30, 19, 70), 18)
    w, b = _rand((12, 1, KS, KS), 19, 0.3), _rand((12,), 20, 0.1)
    out = torch.zeros((2, 50, 19, 70), device=DEV)
    ops.dwconv2d_ex((x.to(DEV), 5, 12), w.to(DEV), b.to(DEV), add=(y.to(DEV), 17, 12), out=(out, 30, 12))
    ref = F.conv2d(x[:, 5:17].double() + y[:, 17:29].double(), w.double(), b.double(), padding=KS // 2, groups=12)
    _close(out[:, 30:42], ref, what="dwconv")
    assert float(out[:, :30].abs().max()) == 0.0 and float(out[:, 42:].abs().max()) == 0.0


# ---------------------------------------------------------------- modules

def _init(m, seed=4321):
    synth.init_module_(m, seed=seed)
    return m.eval().to(DEV)


def _P(m):
    return {k: v.detach().float().cpu() for k, v in m.state_dict().items()}


@pytest.mark.parametrize("name,enc,shape", [("dav2_vits", "vits", (2, 3, 56, 70)), ("dav2_vitl", "vitl", (1, 3, 28, 42))])
def test_depth_anything_vs_reference_golden(name, enc, shape):
    g = load_golden(name)
    m = _init(bb.DepthAnythingFeature(enc))
    x = t(synth.normal(synth.name_seed(name + "_x"), shape)).to(DEV)
    with torch.no_grad():
        out = m(x)
    for k in ("out", "path_1", "path_2", "path_3", "path_4"):
        _close(out[k], t(g[k]), rel=5e-5, abs_=1e-5, what=f"{name} {k}")
    # disp = (1 / depth) / max(1 / depth) (dpt.py:137-141): the smallest ReLU'd depth sets the scale of every
    # pixel, so a 1e-6 absolute error on a depth of ~1e-2 is ~1e-4 relative everywhere -- compared at 1e-3
    _close(out["disp"], t(g["disp"]), rel=1e-3, abs_=1e-5, what=f"{name} disp")
    for i, (tok, cls) in enumerate(out["features"]):
        _close(tok, t(g[f"feat{i}"]), rel=5e-5, abs_=1e-5, what=f"{name} feat{i}")
        _close(cls, t(g[f"cls{i}"]), rel=5e-5, abs_=1e-5, what=f"{name} cls{i}")


def test_depth_anything_vits_vs_oracle_cfg2_size():
    """The cfg2 backbone input (640x480 resized to 672x560: 48x40 patches, 1921 tokens), both images."""
    m = _init(bb.DepthAnythingFeature("vits"))
    x = t(synth.normal(synth.name_seed("dav2_cfg2"), (2, 3, 560, 672)))
    with torch.no_grad():
        out = m(x.to(DEV), with_disp=False, with_features=False)
        ref = bo.depth_anything_feature(_P(m), "", x, "vits")
    for k in ("out", "path_1", "path_4"):
        _close(out[k], ref[k], rel=1e-4, abs_=1e-5, what=f"cfg2 {k}")


def test_feature_vs_reference_golden():
    g = load_golden("feature_vits")
    m = _init(bb.Feature(synth.make_args(vit_size="vits")))
    x = t(synth.normal(synth.name_seed("feature_vits_x"), (2, 3, 64, 96))).to(DEV)
    with torch.no_grad():
        feats, vit_feat = m(x)
    for i, f in enumerate(feats):
        _close(f, t(g[f"x{4 << i}"]), rel=1e-4, abs_=1e-5, what=f"x{4 << i}")
    _close(vit_feat, t(g["vit_feat"]), rel=5e-5, abs_=1e-5, what="vit_feat")


@pytest.mark.parametrize("vit,H,W", [("vits", 128, 160), ("vitl", 96, 128)])
def test_feature_vs_oracle(vit, H, W):
    m = _init(bb.Feature(synth.make_args(vit_size=vit)))
    x = t(synth.normal(synth.name_seed(f"feat_{vit}"), (2, 3, H, W)))
    with torch.no_grad():
        feats, vit_feat = m(x.to(DEV))
        rf, rv = bo.feature_forward(_P(m), "", x, vit)
    for i, (a, b) in enumerate(zip(feats, rf)):
        _close(a, b, rel=1e-4, abs_=1e-5, what=f"{vit} x{4 << i}")
    _close(vit_feat, rv, rel=1e-4, abs_=1e-5, what=f"{vit} vit_feat")


def test_backbone_runs_no_torch_conv_or_sdpa(monkeypatch):
    """Every conv / attention / norm / resize of the backbone path is a HIP kernel: torch's are patched
    to raise (after a first call has prepared the weights: packing, the interpolated position tables)."""
    m = _init(bb.Feature(synth.make_args(vit_size="vits")))
    x = t(synth.normal(synth.name_seed("feature_vits_x"), (2, 3, 64, 96))).to(DEV)
    with torch.no_grad():
        m(x)

    def boom(*a, **k):
        raise AssertionError("torch conv / attention on the backbone path")
    for name in ("conv2d", "conv_transpose2d", "scaled_dot_product_attention", "layer_norm", "instance_norm",
                 "interpolate"):
        monkeypatch.setattr(F, name, boom)
    with torch.no_grad():
        m(x)


def test_e2e_with_real_backbone_vs_oracle():
    """FoundationStereo with the real Feature vs the oracle fed by the oracle backbone (< 1e-3 px)."""
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    H, W = 64, 96
    args = synth.make_args(max_disp=32, corr_levels=2, vit_size="vits")
    args["backbone"] = "real"
    m = FoundationStereo(args).eval()
    synth.init_module_(m, seed=1234)
    m = m.to(DEV)
    left, right = synth.stereo_images(1, H, W)
    with torch.no_grad():
        d = m(t(left).to(DEV), t(right).to(DEV), iters=4, test_mode=True)
        P = {k: v.detach().float().cpu() for k, v in m.state_dict().items()}
        mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
        std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
        ims = torch.cat([t(left), t(right)], 0)
        feats, vit = bo.feature_forward(P, "feature.", (ims / 255.0 - mean) / std, "vits")
        ref = oracle.oracle_forward(P, args, t(left), t(right), [f[:1] for f in feats], [f[1:] for f in feats],
                                    vit[:1], iters=4)
    e, _ = _err(d, ref)
    assert e < 1e-3, f"|dd| {e:.3g} px"
