"""``torch.ops.fsmi``: the hot-path entry points registered with the PyTorch dispatcher.

``csrc/torch_ops.cpp`` wraps the C ABI of libfsmi.so (include/fsmi.h) in a
``TORCH_LIBRARY(fsmi, ...)`` block (CUDA key = HIP devices on ROCm).  It is
compiled in-tree by ``torch.utils.cpp_extension`` at ``build()`` time into
``_lib/fsmi_torch.so`` (linked against libfsmi.so with an ``$ORIGIN`` rpath) and
loaded at run time with ``torch.ops.load_library`` -- the GPU box never
recompiles.  Like ``ops``, there is no CPU kernel: CPU tensors raise.

    from foundationstereo_amd import torch_ops
    torch_ops.load()
    vol = torch.ops.fsmi.gwc_volume(fl, fr, 48, 8)
"""
from __future__ import annotations

import os
import shutil

from .build import LIB, LIB_DIR, PKG, build_library

SRC = os.path.join(PKG, "csrc", "torch_ops.cpp")
EXT = os.path.join(LIB_DIR, "fsmi_torch.so")
_BUILD_DIR = os.path.join(os.path.dirname(PKG), "build", "fsmi_torch")
_loaded = False

OPS = ("gwc_volume", "concat_volume", "allpairs_corr", "volume_pyramid", "geo_lookup", "bilinear_sampler_1d",
       "disparity_regression", "softmax_regression", "context_upsample", "softmax_context_upsample")


def build_extension(force: bool = False, verbose: bool = False) -> str:
    """Compile csrc/torch_ops.cpp with torch.utils.cpp_extension into _lib/fsmi_torch.so."""
    import torch
    from torch.utils import cpp_extension

    lib = build_library()
    deps = [SRC, os.path.join(os.path.dirname(PKG), "include", "fsmi.h"), lib]
    if not force and os.path.exists(EXT) and all(os.path.getmtime(d) <= os.path.getmtime(EXT) for d in deps):
        return EXT
    os.makedirs(_BUILD_DIR, exist_ok=True)
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    so = cpp_extension.load(
        name="fsmi_torch", sources=[SRC], build_directory=_BUILD_DIR, is_python_module=False,
        extra_include_paths=["/opt/rocm/include"],
        extra_cflags=["-O2", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1"],
        # ninja turns '$$' into '$' and the quotes keep the shell off it; the second runpath entry
        # lets cpp_extension import the copy it links under build/ before it sits next to libfsmi.so
        extra_ldflags=[f"-L{tlib}", "-lc10_hip", f"-L{LIB_DIR}", "-lfsmi",
                       "-Wl,-rpath,'$$ORIGIN:$$ORIGIN/../../foundationstereo_amd/_lib'"],
        verbose=verbose)
    del so
    shutil.copy2(os.path.join(_BUILD_DIR, "fsmi_torch.so"), EXT)
    return EXT


def load() -> None:
    """Register torch.ops.fsmi.* from the prebuilt _lib/fsmi_torch.so (raises when it is missing)."""
    global _loaded
    if _loaded:
        return
    import torch
    if not os.path.exists(EXT):
        raise RuntimeError(f"{EXT} missing: build it with `python -m foundationstereo_amd.torch_ops` "
                           "(or __graft_entry__.build())")
    if not os.path.exists(LIB):
        raise RuntimeError(f"{LIB} missing")
    torch.ops.load_library(EXT)
    _loaded = True


def op(name: str, *tensors):
    """``torch.ops.fsmi.<name>`` after the same input checks as ``ops`` (HIP device, fp32, no grad)."""
    from . import ops
    ops._check(name, *tensors)
    load()
    import torch
    return getattr(torch.ops.fsmi, name)


if __name__ == "__main__":
    print(build_extension(force=True, verbose=True))
