"""GPU parity of the call order an unmodified reference forward makes after ``patch_reference``.

``reference_order.forward_reference_order`` restates ``core/foundation_stereo.py:183-191,194-254``
statement for statement over this package's modules: the unfused volume build
(``build_gwc_volume`` + ``proj_cmb`` + ``build_concat_volume`` + ``cat``), ``corr_stem`` /
``corr_feature_att`` / ``classifier`` as plain module calls (MIOpen for ``corr_stem[0]``, ``proj_cmb``
and ``Conv3d(14, 1, 7)``), the context after the volume path, one ``update_block`` call per iteration
and the reference's ``upsample_disp``.  Held to the reference goldens, to the oracle at the bench
geometry, and to the fused ``FoundationStereo.forward`` -- all at the north-star bar, 1e-3 px.
"""
import numpy as np
import pytest
import torch

import oracle
from foundationstereo_amd import ops, synth
from tests.helpers import load_golden, t

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def g(a):
    return t(a).to(DEV)


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from foundationstereo_amd import _lib
    return _lib.load()


def record(name, value):
    import json
    import os
    path = os.environ.get("FSMI_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"test": name, "max_abs_diff_px": value}) + "\n")


def _product(args, H, W, shift, seed=1234):
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    m = FoundationStereo(args).eval()
    synth.init_module_(m, seed=seed)
    m = m.to(DEV)
    fl, fr, vf = synth.backbone_features(1, H, W, args.vit_size, shift_px=shift)
    m.feature.set_features([g(a) for a in fl], [g(a) for a in fr], g(vf))
    left, right = synth.stereo_images(1, H, W)
    return m, (fl, fr, vf), (g(left), g(right))


@pytest.mark.parametrize("name", ["e2e_tiny", "e2e_cfg1_L2", "e2e_cfg1_L4"])
def test_reference_order_vs_golden(lib, name):
    from tests.reference_order import forward_reference_order
    gd = load_golden(name)
    H, W, md, iters, L, shift = (int(v) for v in gd["meta"])
    args = synth.make_args(max_disp=md, corr_levels=L, vit_size="vits")
    m, _, (left, right) = _product(args, H, W, shift)
    ops.range_overflowed(reset=True)
    with torch.no_grad():
        out = forward_reference_order(m, left, right, iters=iters, test_mode=True)
        ops.check_range()
        fused = m(left, right, iters=iters, test_mode=True)
    d = float(np.abs(out.cpu().numpy() - gd["disp"]).max())
    d_fused = float((out - fused).abs().max())
    record(f"reference_order_vs_golden[{name}]", d)
    record(f"reference_order_vs_fused[{name}]", d_fused)
    assert tuple(out.shape) == tuple(gd["disp"].shape)
    assert d < 1e-3 and d_fused < 1e-3, (d, d_fused)


def test_reference_order_train_mode_outputs(lib):
    """test_mode=False: (init_disp, one upsampled prediction per iteration), like the reference."""
    from tests.reference_order import forward_reference_order
    gd = load_golden("e2e_tiny")
    H, W, md, iters, L, shift = (int(v) for v in gd["meta"])
    args = synth.make_args(max_disp=md, corr_levels=L, vit_size="vits")
    m, _, (left, right) = _product(args, H, W, shift)
    with torch.no_grad():
        init_disp, preds = forward_reference_order(m, left, right, iters=iters, test_mode=False)
    assert tuple(init_disp.shape) == (1, 1, H // 4, W // 4) and len(preds) == iters
    assert float(np.abs(preds[-1].cpu().numpy() - gd["disp"]).max()) < 1e-3


@pytest.mark.timeout(600)
def test_reference_order_vs_oracle_cfg2(lib):
    """The bench geometry (640x480, D192, L=4) at 2 iterations vs the CPU oracle."""
    from tests.reference_order import forward_reference_order
    H, W, md, iters, L = 480, 640, 192, 2, 4
    args = synth.make_args(max_disp=md, corr_levels=L, vit_size="vits")
    m, (fl, fr, vf), (left, right) = _product(args, H, W, 8)
    with torch.no_grad():
        out = forward_reference_order(m, left, right, iters=iters, test_mode=True).cpu()
        P = {k: v.cpu() for k, v in m.state_dict().items()}
        ref = oracle.oracle_forward(P, args, left.cpu(), right.cpu(), [t(a) for a in fl], [t(a) for a in fr],
                                    t(vf), iters=iters)
    d = float((out - ref).abs().max())
    record("reference_order_vs_oracle[cfg2,iters2]", d)
    assert d < 1e-3, d
