"""Pin the CPU oracle against golden vectors generated from the reference.

The goldens were produced by ``tools/make_goldens.py`` importing the
reference modules in the build container.  These tests run on
the CPU only and are the oracle's pin.
"""
import numpy as np
import pytest
import torch

import oracle
from tests.helpers import load_golden, t

torch.set_num_threads(min(8, torch.get_num_threads()))


@pytest.fixture(scope="module")
def ops():
    return load_golden("ops_small")


@pytest.mark.parametrize("tag", ["a", "b"])
def test_gwc_volume(ops, tag):
    B, C, G, H, W, D = ops[f"gwc_{tag}_meta"]
    out = oracle.build_gwc_volume(t(ops[f"gwc_{tag}_fl"]), t(ops[f"gwc_{tag}_fr"]), int(D), int(G))
    np.testing.assert_allclose(out.numpy(), ops[f"gwc_{tag}_out"], atol=2e-6, rtol=0)
    # zero region w < d (core/submodule.py:405-410)
    for d in range(1, int(D)):
        assert np.all(out.numpy()[:, :, d, :, :d] == 0)


def test_gwc_group_assert():
    with pytest.raises(AssertionError):
        oracle.build_gwc_volume(torch.zeros(1, 30, 2, 8), torch.zeros(1, 30, 2, 8), 4, 8)


def test_concat_volume(ops):
    B, C, H, W, D = ops["concat_meta"]
    out = oracle.build_concat_volume(t(ops["concat_pl"]), t(ops["concat_pr"]), int(D))
    np.testing.assert_array_equal(out.numpy(), ops["concat_out"])


def test_disparity_regression(ops):
    out = oracle.disparity_regression(t(ops["reg_prob"]), 16)
    np.testing.assert_allclose(out.numpy(), ops["reg_out"], atol=2e-6, rtol=0)


def test_context_upsample(ops):
    out = oracle.context_upsample(t(ops["up_disp"]), t(ops["up_w"]))
    np.testing.assert_allclose(out.numpy(), ops["up_out"], atol=2e-6, rtol=0)


@pytest.mark.parametrize("L", [2, 4])
def test_geo_encoding(ops, L):
    p = f"geo{L}_"
    f1, f2, vol, disp = (t(ops[p + k]) for k in ("f1", "f2", "vol", "disp"))
    np.testing.assert_allclose(oracle.allpairs_corr(f1, f2).numpy(),
                               ops[p + "corr"].reshape(oracle.allpairs_corr(f1, f2).shape), atol=2e-6)
    ge = oracle.GeoEncoding(f1, f2, vol, L, 4)
    for i in range(L):
        np.testing.assert_allclose(ge.cor[i].numpy().ravel(), ops[p + f"corrpyr{i}"].ravel(), atol=2e-6)
    np.testing.assert_allclose(ge.geo[1].numpy().ravel(), ops[p + "volpyr1"].ravel(), atol=2e-6)
    B, _, H, W = disp.shape
    coords = torch.arange(W, dtype=torch.float).view(1, 1, W, 1).repeat(B, H, 1, 1)
    out = ge(disp, coords)
    assert out.shape == ops[p + "out"].shape
    np.testing.assert_allclose(out.numpy(), ops[p + "out"], atol=5e-6, rtol=0)


def test_geo_lookup_naive_matches(ops):
    """The scalar restatement (fp64) agrees with the vectorised oracle."""
    p = "geo2_"
    f1, f2, vol, disp = (t(ops[p + k]) for k in ("f1", "f2", "vol", "disp"))
    vol = vol[:1, :3, :, :2]
    disp = disp[:1, :, :2]
    f1, f2 = f1[:1, :, :2], f2[:1, :, :2]
    corr = oracle.allpairs_corr(f1, f2)
    naive = oracle.geo_lookup_naive(vol, corr, disp, 2, 4)
    ge = oracle.GeoEncoding(f1, f2, vol, 2, 4)
    W = disp.shape[-1]
    coords = torch.arange(W, dtype=torch.float).view(1, 1, W, 1).repeat(1, 2, 1, 1)
    np.testing.assert_allclose(ge(disp, coords).numpy(), naive.numpy(), atol=5e-6)


def test_bilinear_sampler(ops):
    img, coords = ops["bs_img"], ops["bs_coords"]
    P, C, _, Lx = img.shape
    x = t(coords[..., 0]).reshape(P, -1)
    out = oracle.stereo_oracle._sample_1d(t(img).reshape(P, C, Lx), x)
    np.testing.assert_allclose(out.numpy(), ops["bs_out"].reshape(P, C, -1), atol=2e-6)
