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

from .build import LIB, LIB_DIR, PKG, build_library

SRC = os.path.join(PKG, "csrc", "torch_ops.cpp")
EXT = os.path.join(LIB_DIR, "fsmi_torch.so")
_BUILD_DIR = os.path.join(os.path.dirname(PKG), "build", "fsmi_torch")
_loaded = False

OPS = ("gwc_volume", "concat_volume", "allpairs_corr", "volume_pyramid", "geo_lookup", "bilinear_sampler_1d",
       "disparity_regression", "softmax_regression", "context_upsample", "softmax_context_upsample")


def build_extension(force: bool = False, verbose: bool = False) -> str:
    """Compile csrc/torch_ops.cpp into _lib/fsmi_torch.so.

    The compile and link run as plain subprocesses with the include / library paths
    torch.utils.cpp_extension reports, and nothing is loaded into the building process:
    ``cpp_extension.load`` would dlopen its build/ copy and register ``TORCH_LIBRARY(fsmi)``,
    and a later ``load()`` of the _lib copy would register the namespace a second time (a
    c10::Error thrown from a static constructor aborts the process)."""
    import subprocess
    from torch.utils import cpp_extension

    lib = build_library()
    deps = [SRC, os.path.join(os.path.dirname(PKG), "include", "fsmi.h"), lib]
    if not force and os.path.exists(EXT) and all(os.path.getmtime(d) <= os.path.getmtime(EXT) for d in deps):
        return EXT
    os.makedirs(_BUILD_DIR, exist_ok=True)
    obj = os.path.join(_BUILD_DIR, "torch_ops.o")
    tmp = os.path.join(_BUILD_DIR, "fsmi_torch.so")
    incs = [f"-I{d}" for d in cpp_extension.include_paths("cuda")]
    libs = [f"-L{d}" for d in cpp_extension.library_paths("cuda")]
    cxx = os.environ.get("CXX", "c++")
    cmds = [
        [cxx, "-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DHIPBLAS_V2",
         *incs, "-c", SRC, "-o", obj],
        # $ORIGIN: the .so sits next to libfsmi.so in _lib/
        [cxx, "-shared", obj, "-o", tmp, *libs, f"-L{LIB_DIR}", "-lfsmi", "-lc10_hip", "-lc10", "-ltorch_cpu",
         "-ltorch", "-Wl,-rpath,$ORIGIN"],
    ]
    for cmd in cmds:
        if verbose:
            print(" ".join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"torch_ops build failed ({' '.join(cmd)}):\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, EXT)
    return EXT


def _registered() -> bool:
    import torch
    try:
        torch.ops.fsmi.gwc_volume        # resolves only once TORCH_LIBRARY(fsmi) has run
        return True
    except (AttributeError, RuntimeError):
        return False


def available() -> bool:
    """Whether the operator library is built (or already registered in this process)."""
    return _loaded or os.path.exists(EXT)


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
    if not _registered():                # a second TORCH_LIBRARY(fsmi) registration aborts
        # map the runtime this process selected (libfsmi.so, or libfsmi_fast.so under
        # FSMI_PRECISION=fast) first: every build carries the SONAME libfsmi.so, so the loader
        # satisfies fsmi_torch.so's dependency with it instead of mapping a second runtime with its
        # own timers, range flag and safe-mode switch
        from . import _lib
        _lib.load()
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
