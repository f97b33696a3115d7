"""CPU-only checks of the host side: module-tree / state_dict compatibility,
the C-ABI library's exported surface, host logic and loud failure on CPU."""
import re
import os

import numpy as np
import pytest
import torch

from foundationstereo_amd import synth
from tests.helpers import reference_keys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("vit", ["vits", "vitl"])
def test_state_dict_matches_reference(vit):
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    args = synth.make_args(max_disp=192, corr_levels=4, vit_size=vit)
    mine = {k: tuple(v.shape) for k, v in FoundationStereo(args).state_dict().items()}
    ref = dict(reference_keys(vit))
    assert set(mine) == set(ref), (sorted(set(mine) - set(ref))[:10], sorted(set(ref) - set(mine))[:10])
    for k in ref:
        assert mine[k] == ref[k], k


def test_state_dict_order_matches_reference():
    """Key order matters where the reference shares a module under two names (norm3 / downsample.1)."""
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    args = synth.make_args(max_disp=192, corr_levels=4, vit_size="vits")
    mine = list(FoundationStereo(args).state_dict().keys())
    ref = [k for k, _ in reference_keys("vits")]
    assert mine == ref


def _header_symbols():
    txt = open(os.path.join(REPO, "include", "fsmi.h")).read()
    return sorted(set(re.findall(r"\b(fsmi_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_header_symbols():
    from foundationstereo_amd import _lib
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)
    assert lib.fsmi_arch() == b"gfx950"
    assert lib.fsmi_version() >= 100


def test_fast_library_same_abi(monkeypatch):
    """libfsmi_fast.so (FSMI_PRECISION=fast: one fp16 MFMA product per conv MAC) is a separate build of
    the same C ABI, selected by _lib.library_path(); an unknown precision is refused."""
    import ctypes
    from foundationstereo_amd import _lib, build
    monkeypatch.delenv("FSMI_LIB", raising=False)
    monkeypatch.setenv("FSMI_PRECISION", "fast")
    assert _lib.library_path() == build.LIB_FAST
    if not os.path.exists(build.LIB_FAST):
        pytest.skip("fast library not built")
    lib = ctypes.CDLL(build.LIB_FAST)
    for s in _header_symbols():
        assert hasattr(lib, s), s
    monkeypatch.setenv("FSMI_PRECISION", "parity")
    assert _lib.library_path() == build.LIB
    monkeypatch.setenv("FSMI_PRECISION", "bf16")
    with pytest.raises(_lib.FsmiError, match="FSMI_PRECISION"):
        _lib.precision()


def test_library_rejects_bad_args_without_gpu():
    """Argument validation happens before any HIP call, so it is testable on the CPU."""
    from foundationstereo_amd import _lib
    lib = _lib.load()
    rc = lib.fsmi_gwc_volume(1, 1, 1, 1, 30, 8, 4, 2, 8, None)
    assert rc == 1001 and b"num_groups" in lib.fsmi_last_error()
    rc = lib.fsmi_geo_lookup(None, None, None, None, 2, 4, 1, 28, 8, 2, 8, 8, None)
    assert rc == 1001


def test_ops_refuse_cpu_tensors():
    from foundationstereo_amd import ops
    x = torch.zeros(1, 16, 2, 8)
    with pytest.raises(RuntimeError, match="ROCm"):
        ops.gwc_volume(x, x, 4, 8)
    with pytest.raises(RuntimeError, match="ROCm"):
        ops.softmax_regression(torch.zeros(1, 4, 2, 2))


def test_gwc_assertion_mirrors_reference():
    from foundationstereo_amd import submodule
    x = torch.zeros(1, 30, 2, 8)
    with pytest.raises((AssertionError, RuntimeError)):
        submodule.build_gwc_volume(x, x, 4, 8)


@pytest.mark.parametrize("hw", [(240, 320), (375, 1242), (256, 320), (1, 31)])
def test_input_padder(hw):
    from foundationstereo_amd.utils import InputPadder
    x = torch.arange(hw[0] * hw[1], dtype=torch.float32).reshape(1, 1, *hw)
    p = InputPadder(x.shape, divis_by=32)
    (y,) = p.pad(x)
    assert y.shape[-2] % 32 == 0 and y.shape[-1] % 32 == 0
    assert torch.equal(p.unpad(y), x)
    pad_ht = (((hw[0] // 32) + 1) * 32 - hw[0]) % 32   # core/utils/utils.py:26
    pad_wd = (((hw[1] // 32) + 1) * 32 - hw[1]) % 32
    assert p._pad == [pad_wd // 2, pad_wd - pad_wd // 2, pad_ht // 2, pad_ht - pad_ht // 2]


def test_args_access_modes():
    a = synth.make_args(max_disp=64)
    assert a.max_disp == a["max_disp"] == a.get("max_disp") == 64
    assert a.get("low_memory") is False


def test_synth_is_deterministic():
    a = synth.normal(synth.name_seed("x"), (4, 5))
    b = synth.normal(synth.name_seed("x"), (4, 5))
    assert np.array_equal(a, b)
    assert abs(float(synth.normal(7, (100000,)).std()) - 1.0) < 0.02


def test_conv_tuning_db_wellformed():
    """tuning/fsmi_conv.json (tools/tune_conv.py) parses, and every entry names a valid tile
    config / split factor for a well-formed shape key."""
    import json
    import re
    from foundationstereo_amd import ops
    with open(ops._TUNE_PATH) as f:
        db = json.load(f)
    assert db["entries"], "empty tuning table"
    for key, e in db["entries"].items():
        if key.startswith("k3s2_"):        # stride-2 3x3x3 volume convs: their own tiles 4 / 5 / 7 / 10
            ks, stride, kd, cin, cout, B, D, H, W = (int(v) for v in re.findall(r"\d+", key))
            assert key == ops._tune_key(f"{ks}s{stride}", kd, cin, cout, B, D, H, W) and kd == 3
            assert e["cfg"] in (4, 5, 7, 10) and 1 <= e["nsplit"] <= 8, (key, e)
            continue
        ks, kd, cin, cout, B, D, H, W = (int(v) for v in re.findall(r"\d+", key))
        assert key == ops._tune_key(ks, kd, cin, cout, B, D, H, W)
        assert ks in (1, 3) and kd % 2 == 1 and min(cin, cout, B, D, H, W) > 0
        # plain tiles 0..9 (all legal on volumes too), the K-group variants 16 + 3/4/5/7, the
        # pointwise tiles 24..26 (2D 1x1 layers only), the depth-blocked (17, 1, 1) tile 30, or the
        # pipelined-staging register tiles 32 + (2..9) (conv_halo_x3.hip: volumes fall back to the
        # plain tile)
        # (11 / 43: the 2D-only 256 x 5-row tile and its pipelined variant)
        assert (0 <= e["cfg"] <= 9 or e["cfg"] in (19, 20, 21, 23)
                or (24 <= e["cfg"] <= 29 and ks == 1 and kd == 1 and D == 1)
                or (e["cfg"] == 30 and kd == 17 and ks == 1)
                or 34 <= e["cfg"] <= 41 or (e["cfg"] in (11, 43) and kd == 1 and D == 1)) \
            and 1 <= e["nsplit"] <= 8, (key, e)


def test_gelu_erf_coefficients_accuracy():
    """The branch-free erf of the GELU epilogues (csrc/conv_halo.h erf_nb), its coefficients read
    from the header and evaluated as the device does (fmaf Horner in float32, select at |z| = 1):
    within 3 ulp of math.erf over [-6, 6] (tools/fit_erf.py fits them)."""
    import math
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "foundationstereo_amd", "csrc", "conv_halo.h")).read()
    body = src[src.index("float erf_nb(float z)"):src.index("__device__ __forceinline__ float gelu_erf_h")]
    num = r"(-?\d\.\d+e[+-]\d+)f"
    p = [float(re.search(r"float p = " + num, body).group(1))] + \
        [float(v) for v in re.findall(r"p = fmaf\(p, t, " + num + r"\)", body)]
    r = [float(re.search(r"float r = " + num, body).group(1))] + \
        [float(v) for v in re.findall(r"r = fmaf\(r, az, " + num + r"\)", body)]
    assert len(p) == 7 and len(r) == 11
    f32 = np.float32

    def horner(c, x):
        acc = np.full_like(x, f32(c[0]))
        for ci in c[1:]:
            acc = (acc.astype(np.float64) * x + f32(ci)).astype(f32)
        return acc

    z = np.linspace(-6, 6, 400001).astype(f32)
    t = (z * z).astype(f32)
    small = (z.astype(np.float64) * horner(p, t)).astype(f32)
    az = np.minimum(np.abs(z), f32(4))
    e = np.exp2(-(t * f32(1.4426950408889634)).astype(f32).astype(np.float64)).astype(f32)
    big = np.copysign((1.0 - e.astype(np.float64) * horner(r, az)).astype(f32), z)
    got = np.where(np.abs(z) < 1, small, big).astype(np.float64)
    ref = np.array([math.erf(float(v)) for v in z])
    ulp = np.spacing(np.abs(ref).astype(f32)).astype(np.float64)
    assert (np.abs(got - ref) / ulp).max() < 3.0
