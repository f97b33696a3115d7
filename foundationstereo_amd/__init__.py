"""FoundationStereo cost-volume + iterative-refinement hot path, MI355X-native.

Hand-written gfx950 HIP kernels (``csrc/``, C ABI in ``include/fsmi.h``,
loaded via ctypes from ``_lib/libfsmi.so``) behind the reference's own module
and function API (``submodule``, ``geometry``, ``update``, ``utils``,
``foundation_stereo``, and the backbone ``backbone.Feature``).  See DESIGN.md.
"""
import os as _os

__version__ = "0.1.0"

# MIOpen runs only the few convs left outside the HIP kernels (the context net's 7x7 stride-1 `conv1`,
# CAM's 1x1 and SAM's 7x7 convs; tools/torch_conv_census.py lists them) and every conv of the torch
# fallback paths.  Its exhaustive Find benchmarks naive kernels (seconds each) on first use; instead ship the
# find-db measured on MI355X for these layer shapes (tuning/miopen) and use
# FAST mode: db hit -> tuned solver, miss -> immediate-mode heuristic, never a
# search.  Both are only defaults; an explicit environment wins.
_TUNING = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "tuning", "miopen")
_os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
if _os.path.isdir(_TUNING):
    _os.environ.setdefault("MIOPEN_USER_DB_PATH", _TUNING)


def patch_reference(core_foundation_stereo_module):
    """Swap the hot-path names in a loaded ``core.foundation_stereo`` module.

    ``core/foundation_stereo.py`` star-imports ``core.update``,
    ``core.submodule`` and ``core.utils.utils`` and imports
    ``Combined_Geo_Encoding_Volume`` by name (lines 16-20); rebinding those
    globals makes an unmodified reference ``FoundationStereo`` build and run
    this package's modules.  Returns the list of names replaced.
    """
    from . import extractor, foundation_stereo, geometry, submodule, update, utils
    replaced = []
    # ContextNetDino (core/extractor.py, star-imported at :17) and hourglass (defined in
    # core/foundation_stereo.py:45-123 itself) carry the halo-kernel / disparity-transformer fast
    # paths; their module trees, hence state_dict keys, are the reference's
    for name, obj in (("ContextNetDino", extractor.ContextNetDino), ("hourglass", foundation_stereo.hourglass)):
        if hasattr(core_foundation_stereo_module, name):
            setattr(core_foundation_stereo_module, name, obj)
            replaced.append(name)
    for mod in (submodule, update, utils):
        for name in getattr(mod, "__all__", []):
            if hasattr(core_foundation_stereo_module, name):
                setattr(core_foundation_stereo_module, name, getattr(mod, name))
                replaced.append(name)
    for name in ("InputPadder", "bilinear_sampler"):
        setattr(core_foundation_stereo_module, name, getattr(utils, name))
        replaced.append(name)
    core_foundation_stereo_module.Combined_Geo_Encoding_Volume = geometry.Combined_Geo_Encoding_Volume
    replaced.append("Combined_Geo_Encoding_Volume")
    return replaced
