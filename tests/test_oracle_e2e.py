"""Pin the oracle's end-to-end forward and single update step to reference goldens."""
import numpy as np
import pytest
import torch

import oracle
from foundationstereo_amd import synth
from tests.helpers import load_golden, model_keys, oracle_params, t

torch.set_num_threads(min(8, torch.get_num_threads()))


def _run_oracle(name):
    g = load_golden(name)
    H, W, md, iters, L, shift = (int(v) for v in g["meta"])
    args = synth.make_args(max_disp=md, corr_levels=L, vit_size="vits")
    P = oracle_params(model_keys(args), seed=1234)
    fl, fr, vf = synth.backbone_features(1, H, W, "vits", shift_px=shift)
    left, right = synth.stereo_images(1, H, W)
    with torch.no_grad():
        out, aux = oracle.oracle_forward(P, args, t(left), t(right), [t(x) for x in fl], [t(x) for x in fr], t(vf),
                                         iters=iters, return_aux=True)
    return g, out, aux


@pytest.mark.parametrize("name", ["e2e_tiny", "e2e_cfg1_L2", "e2e_cfg1_L4"])
def test_oracle_e2e_matches_reference(name):
    g, out, aux = _run_oracle(name)
    np.testing.assert_allclose(aux["init_disp"].numpy(), g["init_disp"], atol=1e-4, rtol=0)
    geo0 = aux["geo_feat0"]
    assert abs(float(geo0.double().sum()) - float(g["geo0_sum"])) <= 1e-6 * float(g["geo0_abs"]) + 1e-3
    np.testing.assert_allclose(geo0[0, :, 3, :].numpy(), g["geo0_row"], atol=1e-4, rtol=0)
    d = np.abs(out.numpy() - g["disp"]).max()
    assert d < 1e-3, f"max |dd| = {d} px"


def test_oracle_update_step_matches_reference():
    g = load_golden("update_step")
    args = synth.make_args(max_disp=64, corr_levels=2)
    from foundationstereo_amd.update import BasicSelectiveMultiUpdateBlock
    keys = [(k, tuple(v.shape)) for k, v in BasicSelectiveMultiUpdateBlock(args, 128, 28).state_dict().items()]
    P = {("update_block." + k): v for k, v in oracle_params(keys, seed=77).items()}
    net = [t(g[f"net{i}"]) for i in range(3)]
    inp = [t(g[f"inp{i}"]) for i in range(3)]
    att = [t(g[f"att{i}"]) for i in range(3)]
    with torch.no_grad():
        onet, mask, delta = oracle.stereo_oracle.update_block(P, "update_block", net, inp, t(g["corr"]),
                                                              t(g["disp"]), att)
    for i in range(3):
        np.testing.assert_allclose(onet[i].numpy(), g[f"onet{i}"], atol=2e-5, rtol=0)
    np.testing.assert_allclose(mask.numpy(), g["mask"], atol=2e-5, rtol=0)
    np.testing.assert_allclose(delta.numpy(), g["delta"], atol=2e-5, rtol=0)


def synth_features(vit, shift):
    """Backbone stand-in at a pass's padded size (the product's unpreset SyntheticFeature)."""
    def features(B, H, W):
        fl, fr, vf = synth.backbone_features(B, H, W, vit, shift_px=shift)
        return [t(x) for x in fl], [t(x) for x in fr], t(vf)
    return features


def test_oracle_hierarchical_matches_reference():
    """run_hierachical (core/foundation_stereo.py:257-274) incl. the ``+= _pad[0]`` quirk (_pad[0] = 10
    at 200x300) vs the reference golden: the coarse pass's padded output and the final disparity."""
    g = load_golden("hiera_small")
    H, W, md, iters, L, shift = (int(v) for v in g["meta"])
    args = synth.make_args(max_disp=md, corr_levels=L, vit_size="vits")
    P = oracle_params(model_keys(args), seed=1234)
    left, right = synth.stereo_images(1, H, W)
    assert oracle.input_pad(H, W)[0] == 10
    with torch.no_grad():
        out, aux = oracle.oracle_hierarchical(P, args, t(left), t(right), synth_features("vits", shift), iters=iters,
                                              return_aux=True)
    assert out.shape == (1, 1, H, W)
    pad = oracle.input_pad(H // 2, W // 2)
    np.testing.assert_allclose(oracle.stereo_oracle._unpad(t(g["disp_small_padded"]), pad).numpy(),
                               aux["disp_small"].numpy(), atol=1e-3, rtol=0)
    d = np.abs(out.numpy() - g["disp"]).max()
    assert d < 1e-3, f"max |dd| = {d} px"
