"""torch.ops.fsmi (csrc/torch_ops.cpp, TORCH_LIBRARY over the C ABI).

CPU: the prebuilt operator library loads, registers every schema, and has no CPU kernel.
GPU: each operator returns bit-identical results to the ctypes front end (``ops``) -- both call
the same HIP kernels on the current stream -- and to the oracle within the per-op tolerance.
"""
import numpy as np
import pytest
import torch

import oracle
from foundationstereo_amd import torch_ops


def test_operator_library_registers_every_op():
    torch_ops.load()
    for name in torch_ops.OPS:
        schema = str(getattr(torch.ops.fsmi, name).default._schema)
        assert schema.startswith(f"fsmi::{name}("), schema


def test_operators_have_no_cpu_kernel():
    torch_ops.load()
    x = torch.zeros(1, 8, 2, 8)
    with pytest.raises(NotImplementedError):
        torch.ops.fsmi.gwc_volume(x, x, 4, 2)
    from foundationstereo_amd import submodule
    with pytest.raises(RuntimeError, match="ROCm"):        # the reference-API wrapper says why
        submodule.build_gwc_volume(x, x, 4, 2)


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch_ops.load()
    return torch.device("cuda:0")


def _same(a, b):
    assert a.shape == b.shape and torch.equal(a, b)


@pytest.mark.gpu
def test_volume_ops_match_ctypes_and_oracle():
    dev = _gpu()
    from foundationstereo_amd import ops
    gen = torch.Generator().manual_seed(7)
    fl, fr = (torch.randn(2, 64, 9, 40, generator=gen) for _ in range(2))
    D, G = 12, 8
    a = torch.ops.fsmi.gwc_volume(fl.to(dev), fr.to(dev), D, G)
    _same(a, ops.gwc_volume(fl.to(dev), fr.to(dev), D, G))
    np.testing.assert_allclose(a.cpu().numpy(), oracle.build_gwc_volume(fl, fr, D, G).numpy(), atol=1e-5)
    c = torch.ops.fsmi.concat_volume(fl.to(dev), fr.to(dev), D)
    _same(c, ops.concat_volume(fl.to(dev), fr.to(dev), D))
    np.testing.assert_allclose(c.cpu().numpy(), oracle.build_concat_volume(fl, fr, D).numpy(), atol=0)


@pytest.mark.gpu
def test_geometry_ops_match_ctypes():
    dev = _gpu()
    from foundationstereo_amd import ops
    gen = torch.Generator().manual_seed(8)
    B, C, H, W, Cv, D, L, r = 1, 32, 6, 48, 8, 24, 3, 4
    fl, fr = (torch.randn(B, C, H, W, generator=gen).to(dev) for _ in range(2))
    vol = torch.randn(B, Cv, D, H, W, generator=gen).to(dev)
    disp = (torch.rand(B, 1, H, W, generator=gen) * D).to(dev)
    corr_t = torch.ops.fsmi.allpairs_corr(fl, fr, L)
    corr_c = ops.allpairs_corr(fl, fr, L)
    for x, y in zip(corr_t, corr_c):
        _same(x, y)
    vp_t = torch.ops.fsmi.volume_pyramid(vol, L)
    vp_c = ops.volume_pyramid(vol, L)
    for x, y in zip(vp_t, vp_c):
        _same(x, y)
    _same(torch.ops.fsmi.geo_lookup(vp_t, corr_t, disp, r), ops.geo_lookup(vp_c, corr_c, disp, r))
    img = torch.randn(5, 3, 1, 17, generator=gen).to(dev)
    x = (torch.rand(5, 9, generator=gen) * 20 - 2).to(dev)
    _same(torch.ops.fsmi.bilinear_sampler_1d(img, x), ops.bilinear_sampler_1d(img, x))


@pytest.mark.gpu
def test_head_ops_match_ctypes():
    dev = _gpu()
    from foundationstereo_amd import ops
    gen = torch.Generator().manual_seed(9)
    logits = torch.randn(2, 16, 5, 7, generator=gen).to(dev)
    prob = torch.softmax(logits, 1)
    _same(torch.ops.fsmi.disparity_regression(prob, 16), ops.disparity_regression(prob, 16))
    _same(torch.ops.fsmi.softmax_regression(logits), ops.softmax_regression(logits))
    d = torch.randn(2, 1, 5, 7, generator=gen).to(dev)
    w = torch.randn(2, 9, 20, 28, generator=gen).to(dev)
    _same(torch.ops.fsmi.context_upsample(d, torch.softmax(w, 1)), ops.context_upsample(d, torch.softmax(w, 1)))
    _same(torch.ops.fsmi.softmax_context_upsample(d, w, 4.0), ops.softmax_context_upsample(d, w, 4.0))
    with pytest.raises(RuntimeError, match="num_groups"):
        torch.ops.fsmi.gwc_volume(torch.zeros(1, 30, 2, 8, device=dev), torch.zeros(1, 30, 2, 8, device=dev), 4, 8)
