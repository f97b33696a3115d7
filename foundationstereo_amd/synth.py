"""Deterministic synthetic inputs and weights.

There is no network, so neither the pretrained checkpoint nor the timm /
DINOv2 backbone weights exist here.  Every number the
benchmarks, the parity tests and the golden generator feed the hot path
therefore comes from one portable counter-hash PRNG defined here:

* ``splitmix64`` over a per-tensor counter, seeded by an FNV-1a hash of the
  tensor's name, so a tensor's values do not depend on module construction
  order or on torch's RNG state;
* uniform values use the top 24 bits (exact in fp32);
* "normal" values are Irwin-Hall sums of four uniforms (pure arithmetic, no
  libm transcendental, so bit-identical on every host).

The synthetic backbone replaces ``FoundationStereo.feature``
(``core/foundation_stereo.py:143,201-204``): it returns feature maps with the
channel counts of ``Feature.d_out`` (``core/extractor.py:346``) at strides
4/8/16/32 plus ``vit_feat`` at stride 4 (``core/extractor.py:356-357``).
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Sequence, Tuple

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

# DepthAnythingFeature.model_configs[...]['features'] (core/extractor.py:287-291)
VIT_FEATURES = {"vits": 64, "vitb": 128, "vitl": 256}


def name_seed(name: str, base: int = 0) -> int:
    """64-bit FNV-1a of ``name`` mixed with ``base``."""
    h = 0xCBF29CE484222325
    for b in name.encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return (h ^ (base * 0x9E3779B97F4A7C15)) & 0xFFFFFFFFFFFFFFFF


def _splitmix(seed: int, n: int, stream: int = 0) -> np.ndarray:
    idx = np.arange(n, dtype=np.uint64) + np.uint64(stream) * np.uint64(n)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (idx + np.uint64(1)) * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed: int, shape: Sequence[int], lo: float = 0.0, hi: float = 1.0) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    u = (_splitmix(seed, n) >> np.uint64(40)).astype(np.float64) * (1.0 / (1 << 24))
    return (lo + (hi - lo) * u).astype(np.float32).reshape(shape)


def normal(seed: int, shape: Sequence[int], std: float = 1.0) -> np.ndarray:
    """Approximately N(0, std^2): Irwin-Hall(4), rescaled to unit variance."""
    n = int(np.prod(shape)) if len(shape) else 1
    acc = np.zeros(n, dtype=np.float64)
    for s in range(4):
        acc += (_splitmix(seed, n, stream=s) >> np.uint64(40)).astype(np.float64) * (1.0 / (1 << 24))
    z = (acc - 2.0) * math.sqrt(3.0)
    return (z * std).astype(np.float32).reshape(shape)


# ----------------------------------------------------------------------------
# Model configuration
# ----------------------------------------------------------------------------

class StereoArgs(dict):
    """Args object with attribute, item and ``.get`` access.

    The reference reads its config three ways: ``args.max_disp`` (attribute),
    ``cfg['max_disp']`` (``core/foundation_stereo.py:83``) and
    ``args.get('low_memory')`` (``:197``); OmegaConf and the SimpleNamespace
    wrapper of ``scripts/train.py:45-64`` both support all three.
    """

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def make_args(max_disp: int = 192, corr_levels: int = 2, corr_radius: int = 4,
              vit_size: str = "vits", n_gru_layers: int = 3,
              hidden_dims: Sequence[int] = (128, 128, 128), n_downsample: int = 2,
              mixed_precision: bool = False, low_memory: bool = False) -> StereoArgs:
    return StereoArgs(max_disp=max_disp, corr_levels=corr_levels, corr_radius=corr_radius,
                      vit_size=vit_size, n_gru_layers=n_gru_layers,
                      hidden_dims=list(hidden_dims), n_downsample=n_downsample,
                      mixed_precision=mixed_precision, low_memory=low_memory)


def feature_dims(vit_size: str) -> Tuple[List[int], int]:
    """``Feature.d_out`` and ``vit_feat`` channels (core/extractor.py:330-346)."""
    vit_dim = VIT_FEATURES[vit_size] // 2
    chans = [48, 96, 160, 304]
    return [chans[0] * 2 + vit_dim, chans[1] * 2, chans[2] * 2, chans[3]], vit_dim


# ----------------------------------------------------------------------------
# Synthetic inputs
# ----------------------------------------------------------------------------

def stereo_images(B: int, H: int, W: int, seed: int = 0x5EED) -> Tuple[np.ndarray, np.ndarray]:
    """Uniform [0,255) RGB pairs, seed = 0x5EED + pair index."""
    left = np.stack([uniform(name_seed("left", seed + i), (3, H, W), 0.0, 255.0) for i in range(B)])
    right = np.stack([uniform(name_seed("right", seed + i), (3, H, W), 0.0, 255.0) for i in range(B)])
    return left, right


def backbone_features(B: int, H: int, W: int, vit_size: str = "vits", seed: int = 0x5EED,
                      shift_px: int = 0) -> Tuple[List[np.ndarray], List[np.ndarray], np.ndarray]:
    """Synthetic stand-in for ``self.feature(cat[L, R])`` (core/foundation_stereo.py:201-204).

    Returns ``(features_left, features_right, vit_feat)``.  The right 1/4-scale
    map is the left one shifted by ``shift_px`` (at 1/4 resolution) blended with
    fresh noise, so the cost volume has a true matching peak; the coarser maps
    are independent noise.
    """
    d_out, vit_dim = feature_dims(vit_size)
    fl, fr = [], []
    for lvl, c in enumerate(d_out):
        s = 4 * (2 ** lvl)
        h, w = H // s, W // s
        left = np.stack([normal(name_seed(f"featL{lvl}", seed + i), (c, h, w)) for i in range(B)])
        noise = np.stack([normal(name_seed(f"featR{lvl}", seed + i), (c, h, w)) for i in range(B)])
        if lvl == 0 and shift_px > 0:
            shifted = np.zeros_like(left)
            shifted[..., : w - shift_px] = left[..., shift_px:]
            right = (0.8 * shifted + 0.6 * noise).astype(np.float32)
        else:
            right = noise
        fl.append(left)
        fr.append(right)
    vit = np.stack([normal(name_seed("vit", seed + i), (vit_dim, H // 4, W // 4)) for i in range(B)])
    return fl, fr, vit


# ----------------------------------------------------------------------------
# Deterministic weights
# ----------------------------------------------------------------------------

def _fan_in(shape: Sequence[int]) -> int:
    if len(shape) < 2:
        return max(int(shape[0]) if shape else 1, 1)
    return int(np.prod(shape[1:]))


def init_state(shapes: Iterable[Tuple[str, Tuple[int, ...]]], seed: int = 1234) -> Dict[str, np.ndarray]:
    """Hash-initialised values for every ``(name, shape)`` of a state_dict.

    Rules keyed on the parameter name, so they apply identically to the
    reference module tree and to this package's (their keys match):
    conv/linear weights U(-sqrt(3/fan_in), +); biases U(-0.1, 0.1); norm
    weights 1+U(-0.1,0.1); norm biases U(-0.1,0.1); BN running mean
    U(-0.1,0.1) and var 1+U(0,0.2); EdgeNeXt ``gamma`` U(0.1,0.5) so the
    residual branch is exercised (the reference inits it to 1e-6,
    ``core/submodule.py:576``).
    """
    out: Dict[str, np.ndarray] = {}
    weight_shapes = {}
    shapes = list(shapes)
    for name, shape in shapes:
        if name.endswith(".weight"):
            weight_shapes[name[: -len(".weight")]] = tuple(shape)
    for name, shape in shapes:
        shape = tuple(int(s) for s in shape)
        s = name_seed(name, seed)
        leaf = name.rsplit(".", 1)[-1]
        if leaf == "num_batches_tracked":
            out[name] = np.zeros(shape, dtype=np.int64)
        elif leaf == "running_mean":
            out[name] = uniform(s, shape, -0.1, 0.1)
        elif leaf == "running_var":
            out[name] = uniform(s, shape, 1.0, 1.2)
        elif leaf == "gamma":
            out[name] = uniform(s, shape, 0.1, 0.5)
        elif leaf == "weight" and len(shape) == 1:
            out[name] = uniform(s, shape, 0.9, 1.1)
        elif leaf == "weight":
            b = math.sqrt(3.0 / _fan_in(shape))
            out[name] = uniform(s, shape, -b, b)
        elif leaf == "bias":
            out[name] = uniform(s, shape, -0.1, 0.1)
        else:
            out[name] = uniform(s, shape, -0.1, 0.1)
    return out


def init_module_(module, seed: int = 1234):
    """Overwrite every parameter/buffer of a torch module with ``init_state``."""
    import torch

    sd = module.state_dict()
    vals = init_state([(k, tuple(v.shape)) for k, v in sd.items()], seed=seed)
    with torch.no_grad():
        for k, v in sd.items():
            v.copy_(torch.from_numpy(vals[k]).to(v.dtype))
    return module
