"""GPU parity: the HIP hot path (through the C ABI) vs the CPU oracle and the reference goldens.

Tolerances (fp32 everywhere; the north-star bar is |dd| < 1e-3 px end to end):
* per-op kernels vs oracle / golden: abs 1e-5 (different fp32 summation order only);
* all-pairs correlation (K = C products, normalised operands): abs 2e-6 + 2e-6*|x|;
* end-to-end disparity vs oracle and vs the reference golden: max |dd| < 1e-3 px.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import oracle
from foundationstereo_amd import synth
from tests.helpers import load_golden, model_keys, oracle_params, t

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def g(a):
    return t(a).to(DEV)


@pytest.fixture(scope="module")
def ops_mod():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from foundationstereo_amd import _lib, ops
    _lib.load()
    return ops


@pytest.fixture(scope="module")
def gold():
    return load_golden("ops_small")


def record(name, value):
    """Append a measured parity figure to $FSMI_PARITY_LOG (JSON lines) when set."""
    import json
    import os
    path = os.environ.get("FSMI_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"test": name, "max_abs_diff_px": value}) + "\n")


def close(a, b, atol=1e-5, rtol=0.0):
    a = a.detach().float().cpu().numpy() if isinstance(a, torch.Tensor) else a
    b = b.detach().float().cpu().numpy() if isinstance(b, torch.Tensor) else b
    np.testing.assert_allclose(a, b, atol=atol, rtol=rtol)


# ------------------------------------------------------------------ a1 / a2

@pytest.mark.parametrize("tag", ["a", "b"])
def test_gwc_golden(ops_mod, gold, tag):
    B, C, G, H, W, D = (int(v) for v in gold[f"gwc_{tag}_meta"])
    out = ops_mod.gwc_volume(g(gold[f"gwc_{tag}_fl"]), g(gold[f"gwc_{tag}_fr"]), D, G)
    close(out, gold[f"gwc_{tag}_out"])
    assert torch.all(out[:, :, 1:, :, 0] == 0)


@pytest.mark.parametrize("shape", [(1, 128, 8, 5, 40, 48), (2, 224, 8, 3, 24, 30), (1, 32, 8, 2, 11, 7)])
def test_gwc_vs_oracle(ops_mod, shape):
    B, C, G, H, W, D = shape
    fl = synth.normal(11, (B, C, H, W))
    fr = synth.normal(12, (B, C, H, W))
    close(ops_mod.gwc_volume(g(fl), g(fr), D, G), oracle.build_gwc_volume(t(fl), t(fr), D, G))


def test_concat_golden(ops_mod, gold):
    B, C, H, W, D = (int(v) for v in gold["concat_meta"])
    out = ops_mod.concat_volume(g(gold["concat_pl"]), g(gold["concat_pr"]), D)
    assert np.array_equal(out.cpu().numpy(), gold["concat_out"])


@pytest.mark.parametrize("vit,W", [("vits", 40), ("vitl", 24), ("vits", 13)])
def test_comb_volume_stem_vs_oracle(ops_mod, vit, W):
    """Fused gwc+concat+corr_stem[0] == Conv3d_1x1(cat(gwc, concat(proj(fl), proj(fr))))."""
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    args = synth.make_args(max_disp=64, corr_levels=2, vit_size=vit)
    m = FoundationStereo(args)
    synth.init_module_(m, seed=5)
    m = m.to(DEV).eval()
    C = m.feature.d_out[0]
    B, H, D = 2, 3, 16
    fl, fr = synth.normal(21, (B, C, H, W)), synth.normal(22, (B, C, H, W))
    args["max_disp"] = 4 * D
    with torch.no_grad():
        out = m.build_stem_volume(g(fl), g(fr))
        P = {k: v.cpu() for k, v in m.state_dict().items()}
        comb = torch.cat([oracle.build_gwc_volume(t(fl), t(fr), D, 8),
                          oracle.build_concat_volume(oracle.stereo_oracle._conv(P, "proj_cmb", t(fl)),
                                                     oracle.stereo_oracle._conv(P, "proj_cmb", t(fr)), D)], 1)
        ref = oracle.stereo_oracle._conv(P, "corr_stem.0", comb)
        wg, wa, ba, wb, bb = m._stem_weights()
        A, Bm = ops_mod.pointwise_proj(g(fl), wa, ba), ops_mod.pointwise_proj(g(fr), wb, bb)
        two_pass = ops_mod.comb_volume_stem(g(fl), g(fr), A, Bm, wg, D, two_pass=True)
        m.fused_volume = False
        unfused = m.build_stem_volume(g(fl), g(fr))
    close(out, ref, atol=2e-5)
    close(two_pass, ref, atol=2e-5)
    close(unfused, ref, atol=2e-5)


@pytest.mark.parametrize("vit,W,D,tile", [("vits", 100, 80, "16,16"), ("vits", 100, 80, "8,12"), ("vitl", 52, 24, "4,6"),
                                          ("vits", 37, 20, "16,4"), ("vitl", 160, 48, ""), ("vits", 13, 8, "")])
def test_build_stem_tiles(ops_mod, vit, W, D, tile, monkeypatch):
    """Single-pass build over tile shapes (ragged column / disparity tiles, several chunks, W % 4 != 0)
    == the oracle's Conv3d_1x1(cat(gwc, concat(proj(fl), proj(fr)))) (core/foundation_stereo.py:207-213,165)."""
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    monkeypatch.setenv("FSMI_BUILD_TILE", tile)
    args = synth.make_args(max_disp=4 * D, corr_levels=2, vit_size=vit)
    m = FoundationStereo(args)
    synth.init_module_(m, seed=6)
    m = m.to(DEV).eval()
    C = m.feature.d_out[0]
    B, H = 1, 2
    fl, fr = synth.normal(31, (B, C, H, W)), synth.normal(32, (B, C, H, W))
    with torch.no_grad():
        out = m.build_stem_volume(g(fl), g(fr))
        P = {k: v.cpu() for k, v in m.state_dict().items()}
        comb = torch.cat([oracle.build_gwc_volume(t(fl), t(fr), D, 8),
                          oracle.build_concat_volume(oracle.stereo_oracle._conv(P, "proj_cmb", t(fl)),
                                                     oracle.stereo_oracle._conv(P, "proj_cmb", t(fr)), D)], 1)
        ref = oracle.stereo_oracle._conv(P, "corr_stem.0", comb)
    close(out, ref, atol=2e-5)


@pytest.mark.parametrize("vit,B,H", [("vits", 1, 135), ("vitl", 2, 150)])
def test_build_stem_multiround(ops_mod, vit, B, H):
    """More tiles than one round of the 256 CUs: the build's 80-KB image (two blocks per CU, the
    groups staged in four phases instead of one or two) == the oracle's
    Conv3d_1x1(cat(gwc, concat(proj(fl), proj(fr))))."""
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    W, D = 160, 48
    args = synth.make_args(max_disp=4 * D, corr_levels=2, vit_size=vit)
    m = FoundationStereo(args)
    synth.init_module_(m, seed=7)
    m = m.to(DEV).eval()
    C = m.feature.d_out[0]
    fl, fr = synth.normal(41, (B, C, H, W)), synth.normal(42, (B, C, H, W))
    with torch.no_grad():
        out = m.build_stem_volume(g(fl), g(fr))
        P = {k: v.cpu() for k, v in m.state_dict().items()}
        comb = torch.cat([oracle.build_gwc_volume(t(fl), t(fr), D, 8),
                          oracle.build_concat_volume(oracle.stereo_oracle._conv(P, "proj_cmb", t(fl)),
                                                     oracle.stereo_oracle._conv(P, "proj_cmb", t(fr)), D)], 1)
        ref = oracle.stereo_oracle._conv(P, "corr_stem.0", comb)
    close(out, ref, atol=2e-5)


@pytest.mark.parametrize("KS,shape", [(7, (1, 14, 12, 16, 40)), (7, (2, 5, 5, 9, 33)), (3, (1, 14, 8, 8, 64))])
def test_conv3d_direct_vs_torch(ops_mod, KS, shape):
    """Classifier head Conv3d(Cin, 1, KS, padding=KS//2) vs the fp32 torch CPU conv (ragged tiles included)."""
    x = synth.normal(81, shape)
    w = synth.normal(82, (1, shape[1], KS, KS, KS), 0.05)
    b = synth.normal(83, (1,), 0.1)
    ref = torch.nn.functional.conv3d(t(x).double(), t(w).double(), t(b).double(), padding=KS // 2)
    # fp32 sums of Cin*KS^3 (up to 4802) products vs an fp64 reference
    close(ops_mod.conv3d_direct(g(x), g(w), g(b)), ref, atol=2e-5, rtol=1e-5)


@pytest.mark.parametrize("HW", [(19, 45), (12, 40)])
@pytest.mark.parametrize("nsplit", [1, 2])
@pytest.mark.parametrize("cfg", [-1, 0, 1, 2, 3, 4, 5, 8, 9, 11, 19, 20, 21, 23])
@pytest.mark.parametrize("k,cout,act", [(3, 37, "relu"), (1, 70, "gelu"), (3, 136, None), (1, 129, "relu")])
def test_conv2d_halo_vs_torch(ops_mod, cfg, k, cout, act, nsplit, HW):
    """Halo-tiled split-precision conv (cfg 0/1 weights via LDS, 2-5, 8, 9 in registers, 16+c the
    K-group variants: two wave groups per block on alternate chunks): 2 segments (16 channels + a 29-channel slice -> 2 channel
    chunks, ragged last chunk), ragged row/column tiles (19x45; 12x40 takes the float4 split-K
    reduce), ragged couts, output slice, every epilogue term, with and without split-K; vs fp64
    torch.  Same 2e-5 abs + 1e-5 rel tolerance as the im2col kernels."""
    import torch.nn.functional as F
    B, (H, W) = 2, HW
    a_ = synth.normal(191, (B, 16, H, W))
    c_ = synth.normal(192, (B, 40, H, W))
    w = synth.normal(193, (cout, 45, k, k), 0.2)
    bias = synth.normal(194, (cout,), 0.1)
    gamma = synth.uniform(195, (cout,), 0.5, 1.5)
    res = synth.normal(196, (B, cout, H, W))
    segs, x = [g(a_), (g(c_), 5, 29)], torch.cat([t(a_), t(c_[:, 5:34])], 1)
    out = torch.zeros(B, cout + 3, H, W, device=DEV)
    ops_mod.conv2d(segs, ops_mod.PackedConv(g(w), mode="halo"), bias=g(bias), act=act, alpha=0.75,
                   gamma=g(gamma), res=g(res), out=out, co0=2, cfg=cfg, nsplit=nsplit)
    y = F.conv2d(x.double(), t(w).double(), t(bias).double(), padding=k // 2)
    y = {"relu": F.relu, "gelu": F.gelu, None: lambda v: v}[act](y)
    ref = t(res).double() + t(gamma).double().view(1, -1, 1, 1) * 0.75 * y
    close(out[:, 2:2 + cout], ref, atol=2e-5, rtol=1e-5)
    assert float(out[:, :2].abs().max()) == 0 and float(out[:, 2 + cout:].abs().max()) == 0


@pytest.mark.parametrize("HW", [(12, 40), (16, 64)])
@pytest.mark.parametrize("nsplit", [1, 2, 3])
@pytest.mark.parametrize("cfg", [24, 25, 26, 27, 28, 29])
@pytest.mark.parametrize("cout,act,wide", [(70, "gelu", False), (129, "relu", True), (256, None, True)])
def test_conv2d_pw_vs_torch(ops_mod, cfg, cout, act, wide, nsplit, HW):
    """Pointwise LDS-DMA tiles (conv_pw.hip, cfg 24-26; 27-29 split once per block): 2 or 3 segments (16 channels, optionally
    160 more, a 29-channel slice: 2 or 7 chunks through the 3/4-deep ring, ragged last chunk), pixel
    tiles past the plane end (480 px), ragged couts, output slice, every epilogue term, split-K;
    vs fp64 torch, same tolerance as the halo tiles."""
    import torch.nn.functional as F
    B, (H, W) = 2, HW
    a_ = synth.normal(291, (B, 16, H, W))
    c_ = synth.normal(292, (B, 40, H, W))
    e_ = synth.normal(297, (B, 160, H, W)) if wide else None
    cin = 45 + (160 if wide else 0)
    w = synth.normal(293, (cout, cin, 1, 1), 0.2)
    bias = synth.normal(294, (cout,), 0.1)
    gamma = synth.uniform(295, (cout,), 0.5, 1.5)
    res = synth.normal(296, (B, cout, H, W))
    segs = [g(a_)] + ([g(e_)] if wide else []) + [(g(c_), 5, 29)]      # inner segments: multiples of 8
    x = torch.cat([t(a_)] + ([t(e_)] if wide else []) + [t(c_[:, 5:34])], 1)
    out = torch.zeros(B, cout + 3, H, W, device=DEV)
    ops_mod.conv2d(segs, ops_mod.PackedConv(g(w), mode="halo"), bias=g(bias), act=act, alpha=0.75,
                   gamma=g(gamma), res=g(res), out=out, co0=2, cfg=cfg, nsplit=nsplit)
    y = F.conv2d(x.double(), t(w).double(), t(bias).double())
    y = {"relu": F.relu, "gelu": F.gelu, None: lambda v: v}[act](y)
    ref = t(res).double() + t(gamma).double().view(1, -1, 1, 1) * 0.75 * y
    close(out[:, 2:2 + cout], ref, atol=2e-5, rtol=1e-5)
    assert float(out[:, :2].abs().max()) == 0 and float(out[:, 2 + cout:].abs().max()) == 0


@pytest.mark.parametrize("cfg", [-1, 2, 3, 5, 6, 7])
@pytest.mark.parametrize("cin,cout,D,H,W,B", [(56, 28, 6, 9, 37, 1), (112, 56, 3, 8, 20, 2), (168, 112, 2, 4, 10, 1)])
def test_conv3d_up2_vs_torch(ops_mod, cin, cout, D, H, W, B, cfg):
    """ConvTranspose3d(k=4, s=2, p=1) + folded eval BatchNorm + LeakyReLU (the hourglass *_up,
    core/foundation_stereo.py:62-68) as 8 phase convs on the 2x2x2 halo tiles vs fp64 torch: ragged
    row / column / cout tiles, multi-chunk Cin, batch 2."""
    import torch.nn.functional as F
    gen = torch.Generator().manual_seed(cin + cout + D)
    x = torch.randn(B, cin, D, H, W, generator=gen)
    w = torch.randn(cin, cout, 4, 4, 4, generator=gen) * 0.05
    sc = torch.rand(cout, generator=gen) + 0.5
    sh = torch.randn(cout, generator=gen) * 0.1
    packs = ops_mod.pack_deconv_phases(g(w), g(sc))
    out = ops_mod.conv3d_up2(g(x), packs, bias=g(sh), act="leaky", cfg=cfg)
    ref = F.conv_transpose3d(x.double(), w.double(), stride=2, padding=1) * sc.double().view(1, -1, 1, 1, 1) \
        + sh.double().view(1, -1, 1, 1, 1)
    ref = F.leaky_relu(ref, 0.01)
    assert out.shape == ref.shape
    close(out, ref, atol=2e-5, rtol=1e-5)


@pytest.mark.parametrize("cfg", [-1, 2, 3, 5, 6, 7])
@pytest.mark.parametrize("cin,cout,H,W,B,act", [(32, 32, 60, 80, 1, "leaky"), (64, 9, 24, 37, 2, None),
                                                (40, 70, 9, 33, 1, "relu"), (64, 130, 5, 65, 1, None)])
def test_conv2d_up2_vs_torch(ops_mod, cin, cout, H, W, B, act, cfg):
    """ConvTranspose2d(k=4, s=2, p=1) (+ bias / folded scale, activation) as 4 phase convs on the 2x2
    halo tiles vs fp64 torch: the spx pair's shapes (32 -> 32 + LeakyReLU, 64 -> 9 + bias;
    core/foundation_stereo.py:183-191), ragged rows / columns / couts / channel chunks, batch 2."""
    import torch.nn.functional as F
    gen = torch.Generator().manual_seed(cin * 7 + cout + H)
    x = torch.randn(B, cin, H, W, generator=gen)
    w = torch.randn(cin, cout, 4, 4, generator=gen) * 0.05
    sc = torch.rand(cout, generator=gen) + 0.5
    sh = torch.randn(cout, generator=gen) * 0.1
    packs = ops_mod.pack_deconv2d_phases(g(w), g(sc))
    out = ops_mod.conv2d_up2(g(x), packs, bias=g(sh), act=act, cfg=cfg)
    ref = F.conv_transpose2d(x.double(), w.double(), stride=2, padding=1) * sc.double().view(1, -1, 1, 1) \
        + sh.double().view(1, -1, 1, 1)
    ref = {"leaky": lambda v: F.leaky_relu(v, 0.01), "relu": F.relu, None: lambda v: v}[act](ref)
    assert out.shape == ref.shape
    close(out, ref, atol=2e-5, rtol=1e-5)


def test_spx_deconvs_on_hip(ops_mod, monkeypatch):
    """upsample_disp's ConvTranspose2d pair (spx_2_gru.conv1, spx_gru) runs on the phase tiles, never
    through torch (MIOpen), and equals the torch modules (fp64) on the same input."""
    import torch.nn.functional as F
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    args = synth.make_args(max_disp=32, corr_levels=2, vit_size="vits")
    m = FoundationStereo(args).eval()
    synth.init_module_(m, seed=77)
    m = m.to(DEV)
    B, H4, W4 = 1, 16, 24
    disp = g(synth.uniform(78, (B, 1, H4, W4), 0.0, 8.0))
    mask = g(synth.normal(79, (B, 32, H4, W4)))
    stem = g(synth.normal(80, (B, 32, 2 * H4, 2 * W4)))
    m64 = m.double()
    with torch.no_grad():
        x1 = F.leaky_relu(m64.spx_2_gru.conv1.conv(mask.double()), 0.01)
        x2 = m64.spx_2_gru.conv2(torch.cat((x1, stem.double()), 1))
        lg = m64.spx_gru(x2)
        ref = oracle.context_upsample(disp.double().cpu() * 4.0, torch.softmax(lg.cpu(), 1))
    m = m.float()

    def refuse(*a, **k):
        raise AssertionError("conv_transpose2d reached torch")
    monkeypatch.setattr(F, "conv_transpose2d", refuse)
    monkeypatch.setattr(torch, "conv_transpose2d", refuse)
    with torch.no_grad():
        out = m.upsample_disp(disp, mask, stem)
    close(out.squeeze(1), ref, atol=2e-4, rtol=1e-5)


@pytest.mark.parametrize("cfg,nsplit", [(-1, -1), (4, 1), (5, 1), (7, 1), (10, 1), (10, 3), (4, 2)])
@pytest.mark.parametrize("cin,cout,D,H,W,B", [(28, 56, 12, 19, 70, 1), (56, 112, 7, 10, 40, 2),
                                              (112, 168, 6, 15, 20, 1), (40, 37, 5, 9, 65, 1)])
def test_conv3d_s2_vs_torch(ops_mod, cin, cout, D, H, W, B, cfg, nsplit):
    """Conv3d(k=3, s=2, p=1) + folded BN + LeakyReLU (the hourglass conv1/2/3 downsampling,
    core/foundation_stereo.py:50-58) on the stride-2 halo tiles vs fp64 torch: even and odd input
    sizes (output (n-1)//2+1), ragged row / column / cout tiles and channel chunks, batch 2,
    split-K, every stride-2 tile; 2e-5 abs + 1e-5 rel as the stride-1 volume convs."""
    import torch.nn.functional as F
    gen = torch.Generator().manual_seed(cin + cout + D + H)
    x = torch.randn(B, cin, D, H, W, generator=gen)
    w = torch.randn(cout, cin, 3, 3, 3, generator=gen) * 0.05
    bias = torch.randn(cout, generator=gen) * 0.1
    out = ops_mod.conv3d(g(x), ops_mod.PackedConv(g(w), mode="halo"), bias=g(bias), act="leaky", stride=2,
                         cfg=cfg, nsplit=nsplit)
    ref = F.leaky_relu(F.conv3d(x.double(), w.double(), bias.double(), stride=2, padding=1), 0.01)
    assert out.shape == ref.shape
    close(out, ref, atol=2e-5, rtol=1e-5)
    assert not ops_mod.range_overflowed(reset=True)


@pytest.mark.parametrize("k,cin,cout,H,W,res", [(3, 64, 96, 120, 160, False), (1, 64, 96, 120, 160, True),
                                                 (3, 96, 128, 31, 45, False), (1, 128, 128, 15, 20, True)])
def test_conv2d_s2_vs_torch(ops_mod, k, cin, cout, H, W, res):
    """The context net's stride-2 convs (core/extractor.py:20-80: 3x3 s2 p1 and the 1x1 s2
    projection finishing a block as relu(conv + b + y)) as depth-1 volumes on the stride-2 tiles,
    odd sizes included, vs fp64 torch."""
    import torch.nn.functional as F
    gen = torch.Generator().manual_seed(k + cin + H)
    x = torch.randn(2, cin, H, W, generator=gen)
    w = torch.randn(cout, cin, k, k, generator=gen) * 0.05
    bias = torch.randn(cout, generator=gen) * 0.1
    ref = F.conv2d(x.double(), w.double(), bias.double(), stride=2, padding=k // 2)
    y = torch.randn(ref.shape, generator=gen) if res else None
    ref = F.relu(ref + y.double()) if res else F.relu(ref)
    out = ops_mod.conv3d(g(x).unsqueeze(2), ops_mod.PackedConv(g(w), mode="halo"), bias=g(bias), act="relu",
                         res=g(y).unsqueeze(2) if res else None, res_pre=res, stride=2).squeeze(2)
    close(out, ref, atol=2e-5, rtol=1e-5)


def test_context_resblock_s2_vs_torch(ops_mod):
    """ResidualBlock(stride 2, batch norm) fast path (every conv on the halo kernel, the projection
    fused with the block's final relu(x + y)) vs the same module in fp64 on the CPU."""
    import copy
    from foundationstereo_amd.extractor import ResidualBlock
    m = ResidualBlock(64, 96, "batch", stride=2).eval()
    synth.init_module_(m, seed=91)
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(1, 64, 60, 81, generator=gen)
    with torch.no_grad():
        ref = copy.deepcopy(m).double()(x.double())
        out = m.to(DEV)(x.to(DEV))
    close(out, ref, atol=5e-5, rtol=1e-5)


@pytest.mark.parametrize("nsplit", [1, 2])
@pytest.mark.parametrize("kern,stride,cfg", [((17, 1, 1), 1, -1), ((17, 1, 1), 1, 7), ((3, 3, 3), 2, 10),
                                             ((1, 3, 3), 1, 5)])
def test_conv3d_feature_gate_vs_torch(ops_mod, kern, stride, cfg, nsplit):
    """FeatureAtt (core/submodule.py:438-454) folded into the producing conv's epilogue:
    relu(conv(x) + b) * sigmoid(gate) broadcast over depth, gate (B, Cout, Ho, Wo), with and
    without split-K (the reduce pass applies it), vs fp64 torch."""
    import torch.nn.functional as F
    gen = torch.Generator().manual_seed(7 + kern[0] + stride)
    B, cin, cout, D, H, W = 2, 56, 56, 12, 9, 37
    x = torch.randn(B, cin, D, H, W, generator=gen)
    w = torch.randn(cout, cin, *kern, generator=gen) * 0.05
    bias = torch.randn(cout, generator=gen) * 0.1
    pad = tuple(k // 2 for k in kern)
    y = F.conv3d(x.double(), w.double(), bias.double(), stride=stride, padding=pad)
    gate = torch.randn(B, cout, y.shape[3], y.shape[4], generator=gen) * 3
    ref = F.relu(y) * torch.sigmoid(gate.double()).unsqueeze(2)
    out = ops_mod.conv3d(g(x), ops_mod.PackedConv(g(w), mode="halo"), bias=g(bias), act="relu", stride=stride,
                         fatt=g(gate), cfg=cfg, nsplit=nsplit)
    close(out, ref, atol=2e-5, rtol=1e-5)


def test_hourglass_gated_vs_unfused(ops_mod):
    """hourglass with every FeatureAtt folded into its producing conv and the stride-2 convs on
    HIP vs the same module with both off (FeatureAtt as sigmoid * cv in ATen, stride-2 on
    MIOpen), fp32 on the same weights."""
    from foundationstereo_amd import submodule as sub
    from foundationstereo_amd.foundation_stereo import hourglass
    C, fd = 8, [48, 64, 192, 160]
    m = hourglass({"max_disp": 64}, C, fd).eval()
    synth.init_module_(m, seed=77)
    m = m.to(DEV)
    B, D, H, W = 1, 16, 24, 32
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(B, C, D, H, W, generator=gen).to(DEV)
    feats = [torch.randn(B, fd[i], H // 2 ** i, W // 2 ** i, generator=gen).to(DEV) for i in range(4)]
    with torch.no_grad():
        a = m(x, feats)
        old = sub.FATT_FUSE, sub.S2_3D
        try:
            sub.FATT_FUSE, sub.S2_3D = False, False
            b = m(x, feats)
        finally:
            sub.FATT_FUSE, sub.S2_3D = old
    close(a, b.double(), atol=5e-5, rtol=5e-5)


@pytest.mark.parametrize("scale", [3e5, 1e3, 1e-4, 1e-7])
@pytest.mark.parametrize("cfg", [24, 25, 26, 27, 28, 29])
def test_conv2d_pw_range(ops_mod, scale, cfg):
    """Pointwise tiles keep ~22 bits across input scales (block exponent from the first chunk)."""
    import torch.nn.functional as F
    B, H, W, cin, cout = 1, 16, 40, 96, 130
    x = synth.normal(391, (B, cin, H, W)) * scale
    w = synth.normal(392, (cout, cin, 1, 1), 0.2)
    ops_mod.range_overflowed(reset=True)
    ref = F.conv2d(t(x).double(), t(w).double())
    for nsplit in (1, 2):
        out = ops_mod.conv2d([g(x)], ops_mod.PackedConv(g(w), mode="halo"), cfg=cfg, nsplit=nsplit)
        assert bool(torch.isfinite(out).all())
        d = (out.double().cpu() - ref).abs() / ref.abs().max()
        err = float(d.max())
        if err >= 3e-6:
            # diagnostics for an intermittent failure: where, how many, and whether the same call
            # reproduces it right away (same inputs, same stream)
            idx = int(d.argmax())
            again = ops_mod.conv2d([g(x)], ops_mod.PackedConv(g(w), mode="halo"), cfg=cfg, nsplit=nsplit)
            err2 = float(((again.double().cpu() - ref).abs() / ref.abs().max()).max())
            bad = int((d >= 3e-6).sum())
            raise AssertionError(f"nsplit {nsplit}: err {err:.3e} at (co {(idx // (H * W)) % cout}, px {idx % (H * W)}), "
                                 f"{bad} bad elements; immediate re-run err {err2:.3e}")
    assert not ops_mod.range_overflowed(reset=True)


@pytest.mark.parametrize("scale", [3e5, 1e3, 1e-4, 1e-7])
@pytest.mark.parametrize("cfg", [-1, 1, 3, 4, 9])
@pytest.mark.parametrize("k", [1, 3])
def test_conv2d_halo_range(ops_mod, scale, cfg, k):
    """Range-safe split (conv_halo.h, chunk_exp): activations far outside fp16's range -- |x| up to
    ~1e6 (> 65504: fp16 hi halves would overflow) and down to ~1e-7 (hi and lo subnormal) -- with
    one input segment 1e-4x the other inside the same 32-channel chunk.  Error relative to the
    output's magnitude stays at the 22-bit split level (vs fp64 torch), with and without split-K."""
    import torch.nn.functional as F
    B, H, W = 1, 12, 40
    a_ = synth.normal(291, (B, 16, H, W)) * scale
    c_ = synth.normal(292, (B, 40, H, W)) * (scale * 1e-4)
    w = synth.normal(293, (64, 45, k, k), 0.2)
    segs, x = [g(a_), (g(c_), 5, 29)], torch.cat([t(a_), t(c_[:, 5:34])], 1)
    ref = F.conv2d(x.double(), t(w).double(), padding=k // 2)
    for nsplit in (1, 2):
        out = ops_mod.conv2d(segs, ops_mod.PackedConv(g(w), mode="halo"), cfg=cfg, nsplit=nsplit)
        assert bool(torch.isfinite(out).all())
        err = float((out.double().cpu() - ref).abs().max() / ref.abs().max())
        assert err < 3e-6, (nsplit, err)


def test_conv2d_halo_range_flag(ops_mod):
    """A value more than 2^9 x the largest of its block's first 32-channel chunk cannot be brought
    into fp16 by the block exponent: the conv raises the range flag (ops.check_range ->
    RangeError) instead of silently returning inf; in-range calls leave it clear."""
    B, H, W = 1, 8, 32
    small = synth.normal(381, (B, 32, H, W)) * 1e-3          # chunk 0
    big = synth.normal(382, (B, 32, H, W)) * 1e4             # chunk 1: 1e7 x chunk 0
    w = synth.normal(383, (16, 64, 3, 3), 0.2)
    pk = ops_mod.PackedConv(g(w), mode="halo")
    ops_mod.range_overflowed(reset=True)
    ops_mod.conv2d([g(big), g(small)], pk, nsplit=1)        # large chunk first: fine
    ops_mod.check_range()
    ops_mod.conv2d([g(small), g(big)], pk, nsplit=1)
    with pytest.raises(ops_mod.RangeError):
        ops_mod.check_range()
    assert not ops_mod.range_overflowed()                   # check_range reset it


@pytest.mark.parametrize("k", [1, 3])
def test_conv2d_halo_cout_scales(ops_mod, k):
    """Output channels whose weights differ by up to 1e12 in scale (BatchNorm folding spreads
    gamma / sqrt(var) over decades): each row packs with its own exponent (wscale[co]), so every
    output channel keeps the split's ~22 bits relative to its own magnitude (vs fp64 torch)."""
    import torch.nn.functional as F
    B, H, W, cin, cout = 1, 12, 40, 45, 64
    x = synth.normal(391, (B, cin, H, W))
    w = synth.normal(393, (cout, cin, k, k), 0.2) * (10.0 ** np.linspace(-6, 6, cout)).reshape(-1, 1, 1, 1)
    w = w.astype(np.float32)
    out = ops_mod.conv2d([g(x)], ops_mod.PackedConv(g(w), mode="halo"), nsplit=1).double().cpu()
    ref = F.conv2d(t(x).double(), t(w).double(), padding=k // 2)
    rel = ((out - ref).abs().amax((0, 2, 3)) / ref.abs().amax((0, 2, 3))).max()
    assert float(rel) < 3e-6, float(rel)


@pytest.mark.parametrize("scale", [1e5, 1e-6])
@pytest.mark.parametrize("cfg", [-1, 6, 8, 9])
def test_conv3d_halo_range(ops_mod, scale, cfg):
    """The same range guarantee on NCDHW volumes (3^3 conv, chunks span kd planes)."""
    import torch.nn.functional as F
    x = synth.normal(591, (1, 28, 5, 9, 37)) * scale
    w = synth.normal(592, (28, 28, 3, 3, 3), 0.15)
    out = ops_mod.conv3d(g(x), ops_mod.PackedConv(g(w), mode="halo"), cfg=cfg)
    ref = F.conv3d(t(x).double(), t(w).double(), padding=1)
    assert bool(torch.isfinite(out).all())
    err = float((out.double().cpu() - ref).abs().max() / ref.abs().max())
    assert err < 3e-6, err


@pytest.mark.parametrize("cfg", [-1, 5, 6, 7, 8, 9, 21, 23])
@pytest.mark.parametrize("kern,cin,cout,D,act,res", [((3, 3, 3), 28, 28, 7, "leaky", None),
                                                     ((1, 3, 3), 28, 28, 5, "relu", None),
                                                     ((17, 1, 1), 28, 28, 20, "relu", None),
                                                     ((1, 1, 1), 56, 28, 6, None, "post"),
                                                     ((3, 3, 3), 28, 28, 4, "relu", "pre"),
                                                     ((3, 3, 3), 40, 37, 3, None, None)])
def test_conv3d_halo_vs_torch(ops_mod, kern, cin, cout, D, act, res, cfg):
    """Stride-1 Conv3d on the halo kernel (sum over kd of 2D planes): 3^3, axial (1,3,3) and
    (17,1,1), 1^3 with a residual, the ResNet tail act(conv + res), ragged channels / tiles,
    auto split-K, every tile incl. the 128x8 / 256x4 register tiles (cfg 8 / 9: legal on volumes
    since the kernel's lambdas are force-inlined); vs fp64 torch.  2e-5 abs + 1e-5 rel
    as the 2D halo conv."""
    import torch.nn.functional as F
    B, H, W = 1, 9, 37
    x = synth.normal(501, (B, cin, D, H, W))
    w = synth.normal(502, (cout, cin) + kern, 0.15)
    bias = synth.normal(503, (cout,), 0.1)
    r = synth.normal(504, (B, cout, D, H, W)) if res else None
    pk = ops_mod.PackedConv(g(w), mode="halo")
    out = ops_mod.conv3d(g(x), pk, bias=g(bias), act=act, res=g(r) if res else None, res_pre=res == "pre", cfg=cfg)
    y = F.conv3d(t(x).double(), t(w).double(), t(bias).double(), padding=tuple(k // 2 for k in kern))
    if res == "pre":
        y = y + t(r).double()
    y = {"relu": F.relu, "leaky": lambda v: F.leaky_relu(v, 0.01), None: lambda v: v}[act](y)
    if res == "post":
        y = y + t(r).double()
    close(out, y, atol=2e-5, rtol=1e-5)


def test_filter3d_blocks_vs_torch(ops_mod):
    """BasicConv(3D) / ResnetBasicBlock3D / Conv3dNormActReduced fast paths (BatchNorm folded into
    the packed weights) vs the same modules in fp64 on the CPU (torch path)."""
    import copy
    from foundationstereo_amd.submodule import BasicConv, Conv3dNormActReduced, ResnetBasicBlock3D
    mods = [BasicConv(28, 28, is_3d=True, kernel_size=3, padding=1, stride=1),
            ResnetBasicBlock3D(28, 28, kernel_size=3, stride=1, padding=1),
            Conv3dNormActReduced(28, 28, kernel_size=3, kernel_disp=17)]
    x = synth.normal(511, (1, 28, 18, 10, 33))
    for i, m in enumerate(mods):
        synth.init_module_(m, seed=520 + i)
        m.eval()
        ref = copy.deepcopy(m).double()
        with torch.no_grad():
            out = m.to(DEV)(g(x))
            want = ref(t(x).double())
        close(out, want, atol=3e-5, rtol=1e-5)


def test_context_blocks_vs_torch(ops_mod):
    """Context-net fast paths (BN folded into halo convs): ResidualBlock with and without a
    strided projection, the 2D BasicConv with LeakyReLU, and the ContextNetDino output heads,
    vs the same modules in fp64 on the CPU."""
    import copy
    from foundationstereo_amd.extractor import ResidualBlock
    from foundationstereo_amd.submodule import BasicConv
    cases = [(ResidualBlock(64, 64, "batch", stride=1), (1, 64, 24, 40)),
             (ResidualBlock(64, 96, "batch", stride=2), (1, 64, 24, 40)),
             (BasicConv(136, 128, kernel_size=3, padding=1), (1, 136, 17, 33))]
    for i, (m, shape) in enumerate(cases):
        synth.init_module_(m, seed=530 + i)
        m.eval()
        ref = copy.deepcopy(m).double()
        x = synth.normal(540 + i, shape)
        with torch.no_grad():
            out = m.to(DEV)(g(x))
            want = ref(t(x).double())
        close(out, want, atol=3e-5, rtol=1e-5)


@pytest.mark.parametrize("KS,shape", [(7, (2, 5, 19, 70)), (7, (1, 3, 120, 160)), (3, (1, 4, 17, 9)),
                                      (5, (1, 2, 33, 65)), (7, (2, 3, 37, 100)), (5, (1, 2, 9, 4))])
def test_dwconv2d_vs_torch(ops_mod, KS, shape):
    """Depthwise conv (EdgeNeXt dwconv) vs the fp64 torch conv; ragged tiles, 1e-5 abs (49-term fp32 sums);
    W % 4 == 0 shapes take the float4 staging (incl. ragged rows / a partial last column tile)."""
    C = shape[1]
    x = synth.normal(201, shape)
    w = synth.normal(202, (C, 1, KS, KS), 0.2)
    b = synth.normal(203, (C,), 0.1)
    ref = torch.nn.functional.conv2d(t(x).double(), t(w).double(), t(b).double(), padding=KS // 2, groups=C)
    close(ops_mod.dwconv2d(g(x), g(w), g(b)), ref, atol=1e-5)


@pytest.mark.parametrize("B,H,W,gscale", [(1, 120, 160, 1e-6), (2, 7, 13, 0.7), (1, 1, 1, 1.0), (3, 9, 64, 0.3)])
def test_edgenext_mlp_vs_fp64(ops_mod, B, H, W, gscale):
    """The fused EdgeNeXt MLP (pwconv1 -> GELU -> pwconv2 -> gamma -> + input, core/submodule.py:583-590)
    vs the fp64 torch composition: cfg2's shape with the reference's 1e-6 layer-scale init, ragged
    pixel tiles (91, 1, 576 px per image) with a gamma large enough that the MLP dominates, batch > 1;
    in place (out = res) as well."""
    from foundationstereo_amd import update
    from foundationstereo_amd.submodule import EdgeNextConvEncoder
    C = 128
    enc = EdgeNextConvEncoder(C, expan_ratio=4, kernel_size=7, norm=None)
    synth.init_module_(enc, seed=211)
    with torch.no_grad():
        enc.gamma.copy_(torch.from_numpy(synth.uniform(212, (C,), 0.5, 1.5)) * gscale)
    enc = enc.to(DEV).eval()
    x = synth.normal(213, (B, C, H, W), 1.5)
    y = synth.normal(214, (B, C, H, W))
    with torch.no_grad():
        pk1, b1 = update._packed(enc.pwconv1)
        pk2, b2 = update._packed(enc.pwconv2)
        out = ops_mod.edgenext_mlp(g(x), g(y), pk1, b1, pk2, b2, gamma=enc.gamma)
        yy = g(y)
        ops_mod.edgenext_mlp(g(x), yy, pk1, b1, pk2, b2, gamma=enc.gamma, out=yy)
    P = {k: v.detach().cpu().double() for k, v in enc.state_dict().items()}
    h = torch.nn.functional.gelu(torch.einsum("ec,bchw->behw", P["pwconv1.weight"], t(x).double())
                                 + P["pwconv1.bias"].view(1, -1, 1, 1))
    m = torch.einsum("ce,behw->bchw", P["pwconv2.weight"], h) + P["pwconv2.bias"].view(1, -1, 1, 1)
    ref = t(y).double() + P["gamma"].view(1, -1, 1, 1) * m
    tol = 2e-5 * max(1.0, float(m.abs().max()) * gscale)
    close(out, ref, atol=tol, rtol=1e-5)
    close(yy, out, atol=0, rtol=0)


def test_edgenext_mlp_rejects_bad_out(ops_mod):
    """``out`` is validated, not silently written past: wrong shape, non-contiguous, aliasing x, a
    partial overlap with res, and an in-place update on a non-contiguous res all raise."""
    from foundationstereo_amd import update
    from foundationstereo_amd.submodule import EdgeNextConvEncoder
    C, B, H, W = 128, 1, 4, 8
    enc = EdgeNextConvEncoder(C, expan_ratio=4, kernel_size=7, norm=None)
    synth.init_module_(enc, seed=215)
    enc = enc.to(DEV).eval()
    x, y = g(synth.normal(216, (B, C, H, W))), g(synth.normal(217, (B, C, H, W)))
    with torch.no_grad():
        pk1, b1 = update._packed(enc.pwconv1)
        pk2, b2 = update._packed(enc.pwconv2)
        run = lambda xx, rr, oo: ops_mod.edgenext_mlp(xx, rr, pk1, b1, pk2, b2, gamma=enc.gamma, out=oo)  # noqa: E731
        with pytest.raises(RuntimeError, match="contiguous"):
            run(x, y, torch.empty((B, C, H, W + 1), device=DEV))
        with pytest.raises(RuntimeError, match="contiguous"):
            run(x, y, torch.empty((B, C, W, H), device=DEV).transpose(2, 3))
        with pytest.raises(RuntimeError, match="alias x"):
            run(x, y, x)
        big = torch.empty((B, C + 1, H, W), device=DEV)
        big[:, :C] = y
        with pytest.raises(RuntimeError, match="overlaps res"):
            run(x, big[:, :C], big[:, 1:])
        yt = y.transpose(2, 3).contiguous().transpose(2, 3)
        with pytest.raises(RuntimeError, match="contiguous"):
            run(x, yt, yt)


@pytest.mark.parametrize("shape", [(1, 128, 60, 80), (2, 3, 7, 9), (1, 2, 1, 1), (1, 4, 30, 40)])
def test_pool2x_vs_torch(ops_mod, shape):
    """pool2x (avg 3x3, stride 2, pad 1, count_include_pad) vs the torch CPU fp32 op."""
    x = synth.normal(207, shape)
    ref = torch.nn.functional.avg_pool2d(t(x), 3, stride=2, padding=1)
    close(ops_mod.pool2x(g(x)), ref, atol=2e-6)


@pytest.mark.parametrize("KS,B,cout,HW,relu", [(7, 1, 64, (120, 160), True), (7, 2, 13, (19, 70), False),
                                              (3, 1, 9, (17, 9), True), (5, 1, 8, (33, 65), False)])
def test_conv2d_1in_vs_torch(ops_mod, KS, B, cout, HW, relu):
    """Single-input-channel conv (+ReLU) -- the motion encoder's convd1 -- vs the fp64 torch conv;
    ragged pixel tiles and output-channel groups, 1e-5 abs (49-term fp32 sums)."""
    x = synth.normal(204, (B, 1) + HW, 10.0)            # disparity-like magnitudes
    w = synth.normal(205, (cout, 1, KS, KS), 0.2)
    b = synth.normal(206, (cout,), 0.1)
    ref = torch.nn.functional.conv2d(t(x).double(), t(w).double(), t(b).double(), padding=KS // 2)
    if relu:
        ref = ref.clamp_min(0)
    close(ops_mod.conv2d_1in(g(x), g(w), g(b), relu=relu), ref, atol=2e-5 * 10)


@pytest.mark.parametrize("src,dst", [((30, 40), (60, 80)), ((60, 80), (120, 160)), ((7, 5), (13, 11)),
                                     ((1, 6), (3, 6))])
def test_resize_bilinear_vs_torch(ops_mod, src, dst):
    """interp() (align_corners=True bilinear) vs the torch CPU fp32 op."""
    x = synth.normal(211, (2, 3) + src)
    ref = torch.nn.functional.interpolate(t(x), dst, mode="bilinear", align_corners=True)
    close(ops_mod.resize_bilinear(g(x), dst), ref, atol=2e-6)


# ------------------------------------------------------------------ a4 / a9

def test_regression_golden(ops_mod, gold):
    close(ops_mod.disparity_regression(g(gold["reg_prob"]), 16), gold["reg_out"])
    close(ops_mod.softmax_regression(g(gold["reg_logits"])), gold["reg_out"], atol=2e-5)


def test_upsample_golden(ops_mod, gold):
    close(ops_mod.context_upsample(g(gold["up_disp"]), g(gold["up_w"])), gold["up_out"])


def test_softmax_upsample_vs_oracle(ops_mod):
    d = synth.normal(31, (2, 1, 6, 10), 7.0)
    lg = synth.normal(32, (2, 9, 24, 40), 2.0)
    ref = oracle.context_upsample(t(d) * 4.0, torch.softmax(t(lg), 1))
    close(ops_mod.softmax_context_upsample(g(d), g(lg), 4.0), ref, atol=2e-5)


# ------------------------------------------------------------------ a5 / a6

@pytest.mark.parametrize("L", [2, 4])
def test_geo_encoding_golden(ops_mod, gold, L):
    from foundationstereo_amd.geometry import Combined_Geo_Encoding_Volume
    p = f"geo{L}_"
    dx = torch.linspace(-4, 4, 9).reshape(1, 1, 9, 1)
    ge = Combined_Geo_Encoding_Volume(g(gold[p + "f1"]), g(gold[p + "f2"]), g(gold[p + "vol"]), num_levels=L, dx=dx)
    for i in range(L):
        close(ge.init_corr_pyramid[i].reshape(-1), gold[p + f"corrpyr{i}"].reshape(-1), atol=4e-6)
    close(ge.geo_volume_pyramid[1].permute(0, 3, 4, 1, 2).reshape(-1), gold[p + "volpyr1"].reshape(-1), atol=1e-6)
    out = ge(g(gold[p + "disp"]))
    close(out, gold[p + "out"], atol=1e-5)


@pytest.mark.parametrize("C,H,W", [(128, 3, 160), (224, 2, 96), (32, 2, 24), (64, 1, 70)])
def test_allpairs_corr_vs_oracle(ops_mod, C, H, W):
    f1, f2 = synth.normal(41, (2, C, H, W)), synth.normal(42, (2, C, H, W))
    lv = ops_mod.allpairs_corr(g(f1), g(f2), 4)
    lv1 = ops_mod.allpairs_corr(g(f1), g(f2), 4, two_pass=False)
    ref = oracle.allpairs_corr(t(f1), t(f2))
    for i in range(4):
        close(lv[i], ref, atol=3e-6)
        close(lv1[i], ref, atol=3e-6)
        ref = oracle.stereo_oracle._pool_last(ref)


@pytest.mark.parametrize("D,L", [(48, 4), (20, 4), (17, 2), (80, 3)])
def test_volume_pyramid_vs_oracle(ops_mod, D, L):
    v = synth.normal(51, (2, 5, D, 3, 20))
    lv = ops_mod.volume_pyramid(g(v), L)
    ref = t(v).permute(0, 1, 3, 4, 2)
    for i in range(1, L):
        ref = oracle.stereo_oracle._pool_last(ref)
        assert torch.equal(lv[i].cpu(), ref.permute(0, 1, 4, 2, 3).contiguous())


@pytest.mark.parametrize("L,D,W", [(2, 48, 160), (4, 48, 160), (4, 80, 96), (2, 16, 40)])
def test_lookup_vs_oracle(ops_mod, L, D, W):
    """Includes disparities below 0, beyond D and exact integers (border / floor cases)."""
    from foundationstereo_amd.geometry import Combined_Geo_Encoding_Volume
    B, C, Cv, H = 1, 64, 28, 4
    f1, f2 = synth.normal(61, (B, C, H, W)), synth.normal(62, (B, C, H, W))
    vol = synth.normal(63, (B, Cv, D, H, W))
    disp = synth.uniform(64, (B, 1, H, W), -8.0, D + 8.0)
    disp[0, 0, 0, :6] = [0.0, 1.0, D - 1.0, D, -1.0, 2.5]
    ge = Combined_Geo_Encoding_Volume(g(f1), g(f2), g(vol), num_levels=L, dx=torch.linspace(-4, 4, 9))
    out = ge(g(disp))
    ref = oracle.GeoEncoding(t(f1), t(f2), t(vol), L, 4)
    coords = torch.arange(W, dtype=torch.float).view(1, 1, W, 1).repeat(B, H, 1, 1)
    close(out, ref(t(disp), coords), atol=1e-5)


@pytest.mark.parametrize("B,H,W,D,L", [(2, 3, 37, 48, 4), (3, 5, 64, 24, 2)])
def test_lookup_batched_ragged(ops_mod, B, H, W, D, L):
    """Batch > 1 with a pixel count that is not a multiple of 64 (tail lanes, a tile per image) and
    image 0 at integer disparities everywhere: the round trip puts taps of many lanes at a window
    pair other than the centre one (the lookup's general tap path), image 1 at fractional ones (its
    window path); the last image spans the clamped range ends."""
    from foundationstereo_amd.geometry import Combined_Geo_Encoding_Volume
    C, Cv = 32, 28
    f1, f2 = synth.normal(65, (B, C, H, W)), synth.normal(66, (B, C, H, W))
    vol = synth.normal(67, (B, Cv, D, H, W))
    disp = synth.uniform(68, (B, 1, H, W), -6.0, D + 6.0)
    disp[0] = np.round(disp[0])
    disp[-1, 0, 0, :] = np.linspace(-12.0, D + 12.0, W)
    ge = Combined_Geo_Encoding_Volume(g(f1), g(f2), g(vol), num_levels=L, dx=torch.linspace(-4, 4, 9))
    out = ge(g(disp))
    ref = oracle.GeoEncoding(t(f1), t(f2), t(vol), L, 4)
    coords = torch.arange(W, dtype=torch.float).view(1, 1, W, 1).repeat(B, H, 1, 1)
    close(out, ref(t(disp), coords), atol=1e-5)


@pytest.mark.parametrize("kind", ["arange", "shifted", "random"])
def test_lookup_coords_vs_oracle(ops_mod, kind):
    """The reference's ``coords`` argument (core/geometry.py:43,57) honoured, not assumed: the
    arange(W) the reference passes (same result as coords=None), a shifted / fractional grid and
    arbitrary per-pixel columns (beyond the image too), each against the oracle's restatement of
    ``__call__`` with the same coords; also through torch.ops.fsmi.geo_lookup."""
    from foundationstereo_amd import torch_ops
    from foundationstereo_amd.geometry import Combined_Geo_Encoding_Volume
    B, C, Cv, H, W, D, L = 2, 32, 28, 3, 40, 32, 4
    f1, f2 = synth.normal(71, (B, C, H, W)), synth.normal(72, (B, C, H, W))
    vol = synth.normal(73, (B, Cv, D, H, W))
    disp = synth.uniform(74, (B, 1, H, W), -4.0, D + 4.0)
    coords = torch.arange(W, dtype=torch.float).view(1, 1, W, 1).repeat(B, H, 1, 1)
    if kind == "shifted":
        coords = coords + 2.75
    elif kind == "random":
        coords = t(synth.uniform(75, (B, H, W, 1), -6.0, W + 6.0))
    ge = Combined_Geo_Encoding_Volume(g(f1), g(f2), g(vol), num_levels=L, dx=torch.linspace(-4, 4, 9))
    out = ge(g(disp), g(coords))
    ref = oracle.GeoEncoding(t(f1), t(f2), t(vol), L, 4)(t(disp), coords)
    close(out, ref, atol=1e-5)
    if kind == "arange":
        assert torch.equal(out, ge(g(disp)))
    else:
        assert float((out - ge(g(disp))).abs().max()) > 1e-3     # coords really moved the corr taps
    if torch_ops.available():
        op = torch.ops.fsmi.geo_lookup(ge.geo_volume_pyramid, ge.init_corr_pyramid, g(disp), 4, g(coords))
        assert torch.equal(op, out)


@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
def test_bilinear_sampler_returns_img_dtype(ops_mod, gold, dtype):
    """core/utils/utils.py:50-51: the grid is cast to img.dtype and grid_sample returns img.dtype."""
    from foundationstereo_amd.utils import bilinear_sampler
    img = g(gold["bs_img"]).to(dtype)
    out = bilinear_sampler(img, g(gold["bs_coords"]))
    assert out.dtype == dtype
    close(out.float(), gold["bs_out"], atol=1e-5 if dtype == torch.float32 else 2e-2)


def test_bilinear_sampler_golden(ops_mod, gold):
    from foundationstereo_amd.utils import bilinear_sampler
    close(bilinear_sampler(g(gold["bs_img"]), g(gold["bs_coords"])), gold["bs_out"])


# ------------------------------------------------------------------ a7

def test_gru_gates_vs_torch(ops_mod):
    B, Hd, Cx, H, W = 2, 16, 24, 5, 7
    zr_s, zr_l = (g(synth.normal(s, (B, 2 * Hd, H, W), 2.0)) for s in (71, 72))
    h, x = g(synth.normal(73, (B, Hd, H, W))), g(synth.normal(74, (B, Cx, H, W)))
    qs_in, ql_in = ops_mod.gru_reset(zr_s, zr_l, h, x)
    close(qs_in, torch.cat([torch.sigmoid(zr_s[:, Hd:]) * h, x], 1), atol=1e-6)
    close(ql_in, torch.cat([torch.sigmoid(zr_l[:, Hd:]) * h, x], 1), atol=1e-6)
    q_s, q_l = (g(synth.normal(s, (B, Hd, H, W), 2.0)) for s in (75, 76))
    att = g(synth.uniform(77, (B, 1, H, W)))
    out = ops_mod.gru_blend(zr_s, zr_l, q_s, q_l, h, att)
    zs, zl = torch.sigmoid(zr_s[:, :Hd]), torch.sigmoid(zr_l[:, :Hd])
    ref = ((1 - zs) * h + zs * torch.tanh(q_s)) * att + ((1 - zl) * h + zl * torch.tanh(q_l)) * (1 - att)
    close(out, ref, atol=1e-6)


@pytest.mark.parametrize("HW", [(24, 40), (13, 21)])
def test_selective_gru_fused_vs_oracle(ops_mod, HW):
    """SelectiveConvGRU with the gates in the conv epilogues (zr -> z, r*h; convq -> blend) vs the
    oracle's unfused restatement (core/update.py:83-119).  Small maps take split-K, so both reduce
    kernels (float4 at 24x40, scalar at 13x21) run the gate epilogues too."""
    from foundationstereo_amd.update import SelectiveConvGRU
    H, W = HW
    B, Hd, Ci = 2, 32, 48
    mod = SelectiveConvGRU(Hd, Ci + 16)
    synth.init_module_(mod, seed=401)
    mod = mod.to(DEV).eval()
    h = synth.normal(402, (B, Hd, H, W))
    x1, x2 = synth.normal(403, (B, Ci, H, W)), synth.normal(404, (B, 16, H, W))
    att = synth.uniform(405, (B, 1, H, W), 0.0, 1.0)
    with torch.no_grad():
        out = mod(g(att), g(h), g(x1), g(x2))
    P = {"m." + k: v.cpu() for k, v in mod.state_dict().items()}
    ref = oracle.stereo_oracle.selective_gru(P, "m", t(att), t(h), t(x1), t(x2))
    close(out, ref, atol=2e-5)


@pytest.mark.parametrize("B,C,H,W", [(1, 128, 120, 160), (2, 128, 13, 70), (1, 40, 5, 3)])
def test_conv3x3_cout1_vs_torch(ops_mod, B, C, H, W):
    """DispHead's last conv (Cin -> 1, 3x3) on its fp32 kernel, + res, written into a channel slice."""
    x = g(synth.normal(synth.name_seed(f"c1x{B}{C}{H}"), (B, C, H, W)))
    w = g(synth.normal(synth.name_seed(f"c1w{B}{C}{H}"), (1, C, 3, 3), 0.05))
    bias = g(synth.normal(7, (1,), 0.3))
    res = g(synth.normal(synth.name_seed(f"c1r{B}{C}{H}"), (B, 1, H, W), 20.0))
    out = torch.full((B, 5, H, W), 7.0, device=DEV)
    ops_mod.conv3x3_cout1(x, w, bias, res=res, out=out, co0=3)
    ref = F.conv2d(x.double(), w.double(), bias.double(), padding=1) + res.double()
    close(out[:, 3:4], ref, atol=2e-5 + 1e-6 * float(ref.abs().max()))
    assert bool((out[:, :3] == 7.0).all()) and bool((out[:, 4:] == 7.0).all())
    close(ops_mod.conv3x3_cout1(x, w), F.conv2d(x.double(), w.double(), padding=1), atol=2e-5)


def test_update_step_golden(ops_mod):
    gd = load_golden("update_step")
    from foundationstereo_amd.update import BasicSelectiveMultiUpdateBlock
    args = synth.make_args(max_disp=64, corr_levels=2)
    blk = BasicSelectiveMultiUpdateBlock(args, 128, volume_dim=28)
    synth.init_module_(blk, seed=77)
    blk = blk.to(DEV).eval()
    with torch.no_grad():
        net, mask, delta = blk([g(gd[f"net{i}"]) for i in range(3)], [g(gd[f"inp{i}"]) for i in range(3)],
                               g(gd["corr"]), g(gd["disp"]), [g(gd[f"att{i}"]) for i in range(3)])
    for i in range(3):
        close(net[i], gd[f"onet{i}"], atol=5e-5)
    close(mask, gd["mask"], atol=5e-5)
    close(delta, gd["delta"], atol=5e-5)


# ------------------------------------------------------------------ end to end

def _product(args, H, W, shift, seed=1234):
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    m = FoundationStereo(args).eval()
    synth.init_module_(m, seed=seed)
    m = m.to(DEV)
    fl, fr, vf = synth.backbone_features(1, H, W, args.vit_size, shift_px=shift)
    m.feature.set_features([g(a) for a in fl], [g(a) for a in fr], g(vf))
    left, right = synth.stereo_images(1, H, W)
    return m, (fl, fr, vf), (left, right)


@pytest.mark.parametrize("name", ["e2e_tiny", "e2e_cfg1_L2", "e2e_cfg1_L4"])
def test_e2e_vs_reference_golden(ops_mod, name):
    gd = load_golden(name)
    H, W, md, iters, L, shift = (int(v) for v in gd["meta"])
    args = synth.make_args(max_disp=md, corr_levels=L, vit_size="vits")
    m, _, (left, right) = _product(args, H, W, shift)
    with torch.no_grad():
        out = m(g(left), g(right), iters=iters, test_mode=True)
    d = float(np.abs(out.cpu().numpy() - gd["disp"]).max())
    record(f"e2e_vs_reference_golden[{name}]", d)
    assert d < 1e-3, f"max |dd| vs reference = {d} px"


@pytest.mark.parametrize("H,W,md,iters,L,vit", [(480, 640, 192, 2, 4, "vits"), (256, 320, 64, 4, 2, "vitl"),
                                               (480, 640, 192, 32, 4, "vits")])
def test_e2e_vs_oracle(ops_mod, H, W, md, iters, L, vit):
    """cfg2 geometry (640x480, D192, L=4) at reduced and at the full 32 iterations (the bench
    workload, north-star bar 1e-3 px); the oracle runs on the host CPU."""
    args = synth.make_args(max_disp=md, corr_levels=L, vit_size=vit)
    m, (fl, fr, vf), (left, right) = _product(args, H, W, 8)
    with torch.no_grad():
        out = m(g(left), g(right), iters=iters, test_mode=True).cpu()
        P = {k: v.cpu() for k, v in m.state_dict().items()}
        ref = oracle.oracle_forward(P, args, t(left), t(right), [t(a) for a in fl], [t(a) for a in fr], t(vf),
                                    iters=iters)
    d = float((out - ref).abs().max())
    record(f"e2e_vs_oracle[{H}x{W},D{md},iters{iters},L{L},{vit}]", d)
    assert d < 1e-3, f"max |dd| vs oracle = {d} px"


def test_batch_invariance(ops_mod):
    """Pairs are independent: B=2 == two B=1 runs (the basis of batch sharding)."""
    args = synth.make_args(max_disp=32, corr_levels=2, vit_size="vits")
    H, W = 64, 96
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    m = FoundationStereo(args).eval()
    synth.init_module_(m, seed=3)
    m = m.to(DEV)
    fl, fr, vf = synth.backbone_features(2, H, W, "vits", shift_px=2)
    left, right = synth.stereo_images(2, H, W)
    with torch.no_grad():
        m.feature.set_features([g(a) for a in fl], [g(a) for a in fr], g(vf))
        both = m(g(left), g(right), iters=3, test_mode=True)
        singles = []
        for i in range(2):
            m.feature.set_features([g(a[i:i + 1]) for a in fl], [g(a[i:i + 1]) for a in fr], g(vf[i:i + 1]))
            singles.append(m(g(left[i:i + 1]), g(right[i:i + 1]), iters=3, test_mode=True))
    close(both, torch.cat(singles, 0), atol=1e-4)


def test_graph_replay_matches_eager(ops_mod):
    """The bench's hipGraph replay (ShardedStereo.capture) == the eager forward, and a replay
    picks up new contents of the captured input batch.  1e-5 px: MIOpen / hipBLASLt may pick a
    different (equally valid) algorithm under capture, i.e. another fp32 summation order."""
    from foundationstereo_amd import dist as fdist
    args = synth.make_args(max_disp=32, corr_levels=2, vit_size="vits")
    H, W = 64, 96
    m, _, (left, right) = _product(args, H, W, 2)
    batch = torch.stack([g(left), g(right)], 1).contiguous()
    runner = fdist.ShardedStereo(lambda lf, rt: m(lf, rt, iters=3, test_mode=True), 0, 1)
    with torch.no_grad():
        eager = runner.step(batch, (1, H, W)).clone()
        runner.capture(batch)
        replay = runner.step(batch, (1, H, W)).clone()
        close(replay, eager, atol=1e-5)
        batch[:, 0].mul_(0.5)                                  # new left image, same storage
        eager2 = m(batch[:, 0], batch[:, 1], iters=3, test_mode=True)
        replay2 = runner.step(batch, (1, H, W))
    close(replay2, eager2, atol=1e-5)
    assert float((replay2 - replay).abs().max()) > 0


def test_timer_clock_and_replay(ops_mod):
    """bench.py's roofline timing hooks: with timing on, a build launch records an in-kernel clock
    span and a replay closure; replays rewrite identical outputs and report a positive duration."""
    gen = torch.Generator().manual_seed(5)
    C, Cs, H, W, D = 64, 28, 6, 40, 12
    fl, fr = (torch.randn(1, C, H, W, generator=gen).to(DEV) for _ in range(2))
    A, Bm = (torch.randn(1, Cs, H, W, generator=gen).to(DEV) for _ in range(2))
    Wg = (torch.randn(Cs, 8, generator=gen) * 0.3).to(DEV)
    ops_mod.timer_enable(True)
    try:
        ops_mod.timer_reset()
        out = ops_mod.comb_volume_stem(fl, fr, A, Bm, Wg, D)
        ref = out.clone()
        ms, n = ops_mod.timer_query_clock("comb")
        assert n == 1 and ms > 0
        avg = ops_mod.timer_replay("comb", 3)
        torch.cuda.synchronize()
        assert avg > 0 and torch.equal(out, ref)
    finally:
        ops_mod.timer_enable(False)
