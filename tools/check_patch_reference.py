#!/usr/bin/env python3
"""Build-container check of the Python drop-in seam, run by
tests/test_patch_reference.py in a subprocess: import the UNMODIFIED reference
``core.foundation_stereo`` (tools/ref_harness.py stubs; backbone replaced by the
synthetic source), call ``foundationstereo_amd.patch_reference`` on it, construct the
reference's own ``FoundationStereo``, load a state dict written by this package's model
strictly, and report which classes the reference model now instantiates.  Prints one
JSON line.  Needs /root/reference (absent on the GPU box)."""
import json
import os
import sys

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

import torch  # noqa: E402

import foundationstereo_amd  # noqa: E402
from foundationstereo_amd import synth  # noqa: E402
from ref_harness import import_reference, make_synthetic_feature_class  # noqa: E402


def main():
    fs, *_ = import_reference()
    fs.Feature = make_synthetic_feature_class(synth.feature_dims)
    replaced = foundationstereo_amd.patch_reference(fs)
    args = synth.make_args(max_disp=64, corr_levels=4, vit_size="vits")
    ref_model = fs.FoundationStereo(args).eval()
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    ours = FoundationStereo(args)
    synth.init_module_(ours, seed=5)
    ref_model.load_state_dict(ours.state_dict())                      # strict
    mods = {
        "update_block": type(ref_model.update_block).__module__,
        "corr_stem.1": type(ref_model.corr_stem[1]).__module__,
        "cost_agg": type(ref_model.cost_agg).__module__,
        "cost_agg.atts.4": type(ref_model.cost_agg.atts["4"]).__module__,
        "cnet": type(ref_model.cnet).__module__,
        "classifier.0": type(ref_model.classifier[0]).__module__,
        "build_gwc_volume": fs.build_gwc_volume.__module__,
        "Combined_Geo_Encoding_Volume": fs.Combined_Geo_Encoding_Volume.__module__,
    }
    same = all(torch.equal(a, b) for a, b in zip(ref_model.state_dict().values(), ours.state_dict().values()))
    print(json.dumps({"replaced": replaced, "modules": mods, "state_equal": same,
                      "n_keys": len(ref_model.state_dict())}))


if __name__ == "__main__":
    main()
