"""Shared test helpers: golden loading and hash-initialised oracle parameters."""
import json
import os

import numpy as np
import torch

from foundationstereo_amd import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def reference_keys(vit="vits"):
    with open(os.path.join(GOLDEN, f"state_dict_{vit}.json")) as f:
        return [(k, tuple(s)) for k, s in json.load(f)]


def oracle_params(keys, seed=1234):
    """Hash-initialised params keyed by reference state_dict names (fp32 torch)."""
    vals = synth.init_state(keys, seed=seed)
    return {k: torch.from_numpy(v) for k, v in vals.items()}


def model_keys(args):
    """State-dict (name, shape) list of the reference model for ``args`` (from the product module tree)."""
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    m = FoundationStereo(args)
    return [(k, tuple(v.shape)) for k, v in m.state_dict().items()]


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a))
