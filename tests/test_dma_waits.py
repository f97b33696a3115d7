"""Static check of the pointwise tiles' LDS-DMA waits in the shipped code (CPU, no GPU).

``conv_pw_kernel`` waits for its inline-asm LDS-DMA ring with hand-computed ``s_waitcnt vmcnt(N)``
(csrc/conv_pw.hip).  Round 4's one-product build waited for weight loads the compiler had dropped and
read a ring slot before its DMA landed.  tools/check_dma_waits.py disassembles every
conv_pw_kernel instantiation embedded in both libraries and checks, on every control-flow path, that
at least N vector-memory instructions were issued after the DMA each ring wait is for.  The same
check must flag a build compiled with a deliberately wrong weight-load count (FSMI_PW_WLD_ADJ).
Layers: the GRU's 1x1 convs, e.g. convc1 (/root/reference/core/update.py:51-70).
"""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import check_dma_waits as cdw  # noqa: E402

LIBS = [os.path.join(REPO, "foundationstereo_amd", "_lib", f) for f in ("libfsmi.so", "libfsmi_fast.so")]
PW_TILES = 6          # cfg 24-29 (csrc/conv_pw.hip launch_pw)


def _summary(res):
    return {cdw.short(k): [(w["vmcnt"], w["min_after_dma"], w["unsafe"]) for w in v["waits"]] for k, v in res.items()}


@pytest.mark.parametrize("lib", LIBS, ids=os.path.basename)
def test_shipped_dma_waits_cover_their_chunk(lib):
    if not os.path.exists(lib):
        pytest.skip(f"{os.path.basename(lib)} not built (__graft_entry__.build())")
    res = cdw.check_library(lib)
    assert len(res) == PW_TILES, sorted(res)
    for name, r in res.items():
        # the prologue/steady/tail steps each carry one ring wait (the steady pair shares one code copy
        # per parity, so at least 3 distinct waits)
        assert len(r["waits"]) >= 3, (cdw.short(name), r["waits"])
        for w in r["waits"]:
            assert not w["unsafe"], (os.path.basename(lib), cdw.short(name), w)
        # the first step's wait is exact: N == the ops issued after chunk 0's DMA (no over-wait)
        assert min(w["min_after_dma"] - w["vmcnt"] for w in r["waits"]) == 0, _summary(res)


def test_wrong_weight_load_count_is_flagged(tmp_path):
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not shutil.which(hipcc) and not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    obj = tmp_path / "conv_pw_bad.o"
    src = os.path.join(REPO, "foundationstereo_amd", "csrc", "conv_pw.hip")
    # two more weight loads counted than issued: the first chunk's wait no longer covers its DMA
    subprocess.run([hipcc, "-O3", "--offload-arch=gfx950", "-fPIC", "-std=c++17", "-DFSMI_PW_WLD_ADJ=2", "-c", src,
                    "-o", str(obj)], check=True, capture_output=True)
    res = cdw.check_library(str(obj))
    assert len(res) == PW_TILES
    for name, r in res.items():
        assert any(w["unsafe"] for w in r["waits"]), (cdw.short(name), r["waits"])


@pytest.mark.parametrize("lib", LIBS, ids=os.path.basename)
def test_no_flat_memory_ops(lib):
    """No kernel accesses memory through FLAT instructions.  A flat load counts in lgkmcnt as well as
    vmcnt, so the LDS-operand waits of the conv main loops also waited for the halo loads in flight
    (HBM latency inside the MFMA stream): round 4's halo staging built its pointers from integers
    (conv_halo.h SegBases) and every halo conv kernel staged through flat_load_dword."""
    if not os.path.exists(lib):
        pytest.skip(f"{os.path.basename(lib)} not built (__graft_entry__.build())")
    bad = {}
    for co in cdw.code_objects(lib):
        cur = None
        for line in cdw.disassemble(co).splitlines():
            m = cdw._SYM.match(line)
            if m:
                cur = m.group(2)
            elif "\tflat_" in line:
                bad[cur] = bad.get(cur, 0) + 1
    assert not bad, {k[:90]: v for k, v in list(bad.items())[:10]}
