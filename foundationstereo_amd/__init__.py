"""FoundationStereo cost-volume + iterative-refinement hot path, MI355X-native.

Hand-written gfx950 HIP kernels (``csrc/``, C ABI in ``include/fsmi.h``,
loaded via ctypes from ``_lib/libfsmi.so``) behind the reference's own module
and function API (``submodule``, ``geometry``, ``update``, ``utils``,
``foundation_stereo``).  See DESIGN.md.
"""
__version__ = "0.1.0"


def patch_reference(core_foundation_stereo_module):
    """Swap the hot-path names in a loaded ``core.foundation_stereo`` module.

    ``core/foundation_stereo.py`` star-imports ``core.update``,
    ``core.submodule`` and ``core.utils.utils`` and imports
    ``Combined_Geo_Encoding_Volume`` by name (lines 16-20); rebinding those
    globals makes an unmodified reference ``FoundationStereo`` build and run
    this package's modules.  Returns the list of names replaced.
    """
    from . import geometry, submodule, update, utils
    replaced = []
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
