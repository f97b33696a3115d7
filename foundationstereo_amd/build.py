"""Build libfsmi.so (gfx950) in-tree with hipcc.

    python -m foundationstereo_amd.build [--force]

Each ``csrc/*.hip`` compiles to an object under ``build/`` and the objects
link into ``foundationstereo_amd/_lib/libfsmi.so``.  The ``.so`` is git-ignored
but travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(REPO, "build", "fsmi")
LIB_DIR = os.path.join(PKG, "_lib")
LIB = os.path.join(LIB_DIR, "libfsmi.so")
# reference-precision variant (FSMI_PRECISION=fast): one fp16 MFMA product per MAC instead of the
# 3-product split (csrc/conv_halo.h FSMI_NPROD); same ABI
LIB_FAST = os.path.join(LIB_DIR, "libfsmi_fast.so")
FAST_DEFINES = ("FSMI_NPROD=1",)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function"]


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs.append(os.path.join(REPO, "include", "fsmi.h"))
    return hs


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_library(force: bool = False, verbose: bool = False, defines=(), variant: str = "") -> str:
    """Compile every csrc/*.hip and link libfsmi.so.  ``defines`` / ``variant``: an A/B build of
    the same ABI with extra -D flags, linked to _lib/libfsmi_<variant>.so (load it with FSMI_LIB)."""
    obj_dir = OBJ if not variant else OBJ + "_" + variant
    lib = LIB if not variant else os.path.join(LIB_DIR, f"libfsmi_{variant}.so")
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    hdrs = _headers()
    jobs = []
    objs = []
    dflags = [f"-D{d}" for d in defines]
    for src in _sources():
        obj = os.path.join(obj_dir, os.path.basename(src)[:-4] + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + hdrs):
            jobs.append([HIPCC, *FLAGS, *dflags, "-c", src, "-o", obj])

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed ({' '.join(cmd)}):\n{r.stdout}\n{r.stderr}")
        if verbose and (r.stderr.strip()):
            print(r.stderr, file=sys.stderr)
        return cmd[-1]

    if jobs:
        with ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
            list(ex.map(run, jobs))
    if force or jobs or _stale(lib, objs):
        # one SONAME for every build of the ABI: fsmi_torch.so's DT_NEEDED "libfsmi.so" then resolves to
        # whichever build _lib.load() mapped first (e.g. libfsmi_fast.so), never to a second copy
        run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-Wl,-soname,libfsmi.so", *objs, "-o", lib])
    return lib


def build_timeline(force: bool = False, verbose: bool = False) -> str:
    """The diagnostic build whose conv / MLP / aux kernels stamp in-kernel clocks in timer mode 3
    (_lib/libfsmi_timeline.so, tools/replay_timeline.py); not built by __graft_entry__.build()."""
    return build_library(force=force, verbose=verbose, defines=("FSMI_TIMELINE=1",), variant="timeline")


def build_fast(force: bool = False, verbose: bool = False) -> str:
    """The reference-precision library (one fp16 MFMA product per MAC), _lib/libfsmi_fast.so."""
    return build_library(force=force, verbose=verbose, defines=FAST_DEFINES, variant="fast")


if __name__ == "__main__":
    # python -m foundationstereo_amd.build [--force] [--variant NAME -DMACRO=V ...]
    argv = sys.argv[1:]
    variant = argv[argv.index("--variant") + 1] if "--variant" in argv else ""
    defs = [a[2:] for a in argv if a.startswith("-D")]
    print(build_library(force="--force" in argv, verbose=True, defines=defs, variant=variant))
