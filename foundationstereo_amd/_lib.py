"""ctypes binding of libfsmi.so (the C ABI declared in include/fsmi.h).

There is deliberately no fallback: if the library is missing or fails to load,
every hot-path op raises.  Build it with ``python -m foundationstereo_amd.build``
(or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
import os

from .build import LIB, LIB_FAST

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_PP = ctypes.POINTER(ctypes.c_void_p)

# name -> argtypes, mirroring include/fsmi.h
SIGNATURES = {
    "fsmi_version": [],
    "fsmi_last_error": [],
    "fsmi_arch": [],
    "fsmi_gwc_volume": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _P],
    "fsmi_concat_volume": [_P, _P, _P, _I, _I, _I, _I, _I, _P],
    "fsmi_comb_volume_stem": [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P],
    "fsmi_pointwise_proj": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "fsmi_allpairs_corr": [_P, _P, _PP, _I, _I, _I, _I, _I, _P, _P],
    "fsmi_volume_pyramid": [_P, _PP, _I, _I, _I, _I, _I, _I, _P],
    "fsmi_geo_lookup": [_PP, _PP, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "fsmi_geo_lookup_coords": [_PP, _PP, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "fsmi_bilinear_sampler_1d": [_P, _P, _P, _I, _I, _I, _I, _P],
    "fsmi_disparity_regression": [_P, _P, _I, _I, _I, _I, _P],
    "fsmi_softmax_regression": [_P, _P, _I, _I, _I, _I, _P],
    "fsmi_context_upsample": [_P, _P, _P, _I, _I, _I, _P],
    "fsmi_softmax_context_upsample": [_P, _P, _P, _F, _I, _I, _I, _P],
    "fsmi_gru_reset": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "fsmi_gru_blend": [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P],
    "fsmi_conv3d_direct": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P],
    "fsmi_conv2d_halo_x3": [_PP, ctypes.POINTER(_I), ctypes.POINTER(_I), _I, _P, _P, _P, _P, _P, _I, _P, _I,
                            _I, _I, _I, _I, _I, _I, _I, _F, _I, _I, _P, ctypes.c_longlong, _P],
    "fsmi_conv2d_halo_x3_gate": [_PP, ctypes.POINTER(_I), ctypes.POINTER(_I), _I, _P, _P, _P, _I, _P, _P, _P,
                                 _P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, ctypes.c_longlong, _P],
    "fsmi_conv3d_halo_x3": [_P, _I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P,
                            ctypes.c_longlong, _P],
    "fsmi_conv3d_halo_x3_ex": [_P, _I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I,
                               _P, ctypes.c_longlong, _P],
    "fsmi_conv3d_up2_halo_x3": [_P, _I, _PP, _PP, _PP, _P, _I, _I, _I, _I, _I, _I, _I, _P],
    "fsmi_conv2d_up2_halo_x3": [_P, _I, _PP, _PP, _PP, _P, _I, _I, _I, _I, _I, _I, _P],
    "fsmi_dwconv2d": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "fsmi_dwconv2d_ex": [_P, _I, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P],
    "fsmi_channel_layernorm": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _F, _P],
    "fsmi_vit_attention": [_P, _P, _I, _I, _I, _I, _I, _F, _P, ctypes.c_longlong, _P],
    "fsmi_vit_attention_ws_floats": [_I, _I, _I, _I],
    "fsmi_space_to_depth": [_P, _P, _I, _I, _I, _I, _I, _P],
    "fsmi_depth_to_space": [_P, _P, _I, _I, _I, _I, _I, _P],
    "fsmi_vit_tokens": [_P, _P, _P, _P, _I, _I, _I, _I, _P],
    "fsmi_resize_bicubic": [_P, _P, _I, _I, _I, _I, _I, _I, _P],
    "fsmi_instance_norm": [_P, _P, _P, _I, _I, _F, _I, _I, _P],
    "fsmi_elementwise": [_P, _P, _P, ctypes.c_longlong, ctypes.c_longlong, _I, _P],
    "fsmi_xca": [_P, _P, _P, _P, _I, _I, _I, _I, _P],
    "fsmi_xca_workspace_floats": [_I, _I, _I],
    "fsmi_edgenext_mlp": [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "fsmi_resize_bilinear": [_P, _P, _I, _I, _I, _I, _I, _I, _P],
    "fsmi_pool2x": [_P, _P, _I, _I, _I, _I, _P],
    "fsmi_conv2d_1in": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P],
    "fsmi_conv3x3_cout1": [_P, _I, _P, _P, _P, ctypes.c_longlong, _P, ctypes.c_longlong, _I, _I, _I, _P],
    "fsmi_dt_layer_floats": [],
    "fsmi_dt_patch_embed": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "fsmi_disparity_transformer": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _F, _P],
    "fsmi_upsample4_add": [_P, _P, _I, _I, _I, _I, _I, _P],
    "fsmi_debug_conv_timestamps": [_P],
    "fsmi_range_status": [_I, ctypes.POINTER(_I)],
    "fsmi_set_range_safe": [_I],
    "fsmi_range_poison": [_P, ctypes.c_longlong, _P],
    "fsmi_get_range_safe": [ctypes.POINTER(_I)],
    "fsmi_conv_launch_counts": [ctypes.POINTER(ctypes.c_longlong), _I, _I],
    "fsmi_timer_enable": [_I],
    "fsmi_timer_reset": [],
    "fsmi_timer_query": [_I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong)],
    "fsmi_timer_query_clock": [_I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong)],
    "fsmi_timer_replay": [_I, _I, ctypes.POINTER(ctypes.c_double)],
    "fsmi_timer_query_clock_captured": [_I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong)],
    "fsmi_timer_release_captured": [],
    "fsmi_timer_dump_captured": [ctypes.c_char_p, ctypes.c_longlong, ctypes.POINTER(ctypes.c_longlong)],
    "fsmi_timer_captured_count": [ctypes.POINTER(ctypes.c_longlong)],
}

KERNELS = ["gwc", "concat", "comb", "proj", "corr", "volpyr", "lookup", "sampler", "reg", "upsample",
           "gru_reset", "gru_blend", "conv3d", "conv2d", "dwconv", "resize", "dt", "norm"]

_lib = None


class FsmiError(RuntimeError):
    pass


def precision() -> str:
    """Conv arithmetic of this process: "parity" (default; 3 fp16 MFMA products per MAC on hi/lo
    splits, ~22-bit operands, |dd| < 1e-3 px vs the fp32 CPU reference) or "fast" (FSMI_PRECISION=fast:
    one fp16 product per MAC with fp32 accumulation -- the reference's own fp16-autocast GPU
    precision, not within the parity tolerance).  Volumes, lookup and every non-conv kernel are fp32
    in both."""
    p = os.environ.get("FSMI_PRECISION", "parity").lower()
    if p not in ("parity", "fast"):
        raise FsmiError(f"FSMI_PRECISION={p!r}: 'parity' or 'fast'")
    return p


def library_path() -> str:
    """FSMI_LIB (A/B builds of the same ABI, tools/), else the in-tree library of ``precision()``."""
    return os.environ.get("FSMI_LIB") or (LIB_FAST if precision() == "fast" else LIB)


def load():
    """Load libfsmi.so once; raise if it is absent (no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    if not os.path.exists(path):
        raise FsmiError(f"{os.path.basename(path)} not found at {path}: the HIP hot path is not built "
                        "(run `python -m foundationstereo_amd.build`, or __graft_entry__.build())")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None and (name.startswith("fsmi_debug_") or name == "fsmi_timer_dump_captured"):
            continue                     # diagnostics absent from an older A/B build (FSMI_LIB)
        if fn is None:
            raise FsmiError(f"{path}: missing symbol {name}")
        fn.argtypes = argtypes
        fn.restype = (ctypes.c_char_p if name in ("fsmi_last_error", "fsmi_arch") else
                      ctypes.c_longlong if name.endswith("_floats") and name != "fsmi_dt_layer_floats" else ctypes.c_int)
    _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = load().fsmi_last_error().decode(errors="replace")
        if rc == 1001:
            raise FsmiError(f"{what}: {msg}")
        raise FsmiError(f"{what}: HIP error {rc}: {msg}")


def ptr_array(ptrs):
    arr = (ctypes.c_void_p * len(ptrs))(*ptrs)
    return ctypes.cast(arr, _PP), arr
