"""Loop-invariant context segment of SelectiveConvGRU.conv0 (update.SelectiveConvGRU.context_pre).

conv0(cat(inp, rest)) = W0[:, :Ci] * inp + b0 + W0[:, Ci:] * rest: the first term is computed once per
forward and the loop's conv0 convolves only ``rest`` with the halo kernel's act 7 epilogue
(ReLU(conv + bias + res), the residual added BEFORE the activation).  Checked here:

* act 7 on every 2D tile family (LDS / register / pipelined / K-group / pointwise) and both split-K
  reduce kernels vs fp64 torch (tolerance of the other halo conv tests: 2e-5 abs + 1e-5 rel);
* SelectiveConvGRU with ``pre`` vs the oracle's restatement (core/update.py:98-119), with a large
  disparity-like last channel in the motion segment (the segment reordering for the block exponent);
* the product forward with context_pre (FSMI_CTX_PRE) and DispHead's Cout=1 kernel (FSMI_COUT1) on vs
  off.
"""
import pytest
import torch
import torch.nn.functional as F

import oracle
from foundationstereo_amd import synth
from tests.helpers import t

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def ops_mod():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from foundationstereo_amd import _lib, ops
    _lib.load()
    return ops


def g(a):
    return t(a).to(DEV)


def _check(out, ref, what):
    out, ref = out.detach().double().cpu(), ref.detach().double().cpu()
    err = float((out - ref).abs().max())
    tol = 2e-5 + 1e-5 * float(ref.abs().max())
    assert err <= tol, f"{what}: max |diff| {err:.3g} > {tol:.3g}"


# (KS, cfg, nsplit, H, W): LDS tiles 0 / 1, register tiles 3 / 5 / 9 / 11, pipelined 32 + c, K groups 16 + c,
# pointwise 24 / 26 (1x1); split-K 2 / 3 through the float4 reduce (H*W % 4 == 0) and the scalar one
CASES = [(3, 0, 1, 20, 40), (3, 1, 1, 20, 40), (3, 3, 1, 20, 40), (3, 5, 1, 13, 21), (3, 9, 1, 20, 40),
         (3, 11, 1, 30, 40), (3, 40, 1, 30, 40), (3, 43, 1, 30, 40), (3, 35, 1, 13, 21), (3, 19, 1, 20, 40),
         (3, 3, 2, 20, 40), (3, 3, 3, 13, 21), (1, 4, 1, 20, 40), (1, 24, 1, 20, 40), (1, 26, 2, 20, 40),
         (3, -1, -1, 60, 80)]


@pytest.mark.parametrize("KS,cfg,nsplit,H,W", CASES)
def test_conv_act7_vs_torch(ops_mod, KS, cfg, nsplit, H, W):
    B, C1, C2, Co = 2, 96, 64, 160
    x1 = g(synth.normal(synth.name_seed(f"a7x1_{KS}_{cfg}"), (B, C1, H, W)))
    x2 = g(synth.normal(synth.name_seed(f"a7x2_{KS}_{cfg}"), (B, C2, H, W), 3.0))
    w = g(synth.normal(synth.name_seed(f"a7w_{KS}_{cfg}"), (Co, C1 + C2, KS, KS), 0.05))
    pre = g(synth.normal(synth.name_seed(f"a7p_{KS}_{cfg}"), (B, Co, H, W), 2.0))
    pk = ops_mod.PackedConv(w, mode="halo")
    out = ops_mod.conv2d([x1, x2], pk, act="relu_pre", res=pre, cfg=cfg, nsplit=nsplit)
    ref = F.relu(F.conv2d(torch.cat([x1, x2], 1).double(), w.double(), padding=KS // 2) + pre.double())
    _check(out, ref, f"act 7 k{KS} cfg {cfg} split {nsplit}")


def test_conv_act7_needs_res(ops_mod):
    x = g(synth.normal(5, (1, 32, 8, 32)))
    pk = ops_mod.PackedConv(g(synth.normal(6, (32, 32, 3, 3), 0.1)), mode="halo")
    with pytest.raises(RuntimeError, match="act 7"):
        ops_mod.conv2d([x], pk, act="relu_pre")


@pytest.mark.parametrize("HW,disp", [((24, 40), 1.0), ((30, 40), 150.0)])
def test_selective_gru_with_pre_vs_oracle(ops_mod, HW, disp):
    """gru04's shape class: x = (inp, motion features with the disparity as last channel, interp)."""
    from foundationstereo_amd.update import SelectiveConvGRU
    H, W = HW
    B, Hd, Ci = 1, 32, 32
    mod = SelectiveConvGRU(Hd, 3 * Ci)
    synth.init_module_(mod, seed=411)
    mod = mod.to(DEV).eval()
    h = synth.normal(412, (B, Hd, H, W))
    inp = synth.normal(413, (B, Ci, H, W)).clip(0, None)
    mot = synth.normal(414, (B, Ci, H, W)).clip(0, None)
    mot[:, -1] = disp * synth.uniform(415, (B, H, W), 0.2, 1.0)
    up = synth.normal(416, (B, Ci, H, W)).clip(-1, 1)
    att = synth.uniform(417, (B, 1, H, W), 0.0, 1.0)
    with torch.no_grad():
        pre = mod.context_pre(g(inp))
        out = mod(g(att), g(h), g(inp), g(mot), g(up), pre=pre)
        plain = mod(g(att), g(h), g(inp), g(mot), g(up))
    P = {"m." + k: v.cpu() for k, v in mod.state_dict().items()}
    ref = oracle.stereo_oracle.selective_gru(P, "m", t(att), t(h), t(inp), t(mot), t(up))
    _check(out, ref, "SelectiveConvGRU with context_pre")
    _check(plain, ref, "SelectiveConvGRU")


@pytest.mark.parametrize("knob", ["CTX_PRE", "COUT1"])
def test_forward_pre_on_off(ops_mod, monkeypatch, knob):
    """The product forward (pipelined loop) with the conv0 context part hoisted (CTX_PRE) / the fp32
    Cout=1 head conv (COUT1) vs without: equal to fp32 reordering (and within the oracle's bar in the
    end-to-end tests)."""
    from foundationstereo_amd import update
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    args = synth.make_args(max_disp=64, corr_levels=2, vit_size="vits")
    H, W = 96, 128
    m = FoundationStereo(args).eval()
    synth.init_module_(m, seed=1234)
    m = m.to(DEV)
    fl, fr, vf = synth.backbone_features(1, H, W, args.vit_size, shift_px=4)
    m.feature.set_features([g(a) for a in fl], [g(a) for a in fr], g(vf))
    left, right = synth.stereo_images(1, H, W)
    outs = {}
    for on in (True, False):
        monkeypatch.setattr(update, knob, on)
        with torch.no_grad():
            outs[on] = m(g(left), g(right), iters=6, test_mode=True).cpu()
    d = float((outs[True] - outs[False]).abs().max())
    assert d < 1e-4, f"|dd| {knob} on vs off {d:.3g} px"

