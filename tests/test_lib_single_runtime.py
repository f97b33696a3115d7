"""One runtime per process: under FSMI_PRECISION=fast the operator library (fsmi_torch.so, linked
against libfsmi.so) must reuse the already-loaded libfsmi_fast.so -- both builds carry the SONAME
libfsmi.so -- instead of mapping the parity runtime as a second copy with its own timers, range
flag and safe-mode switch.  Loading needs no GPU."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys
sys.path.insert(0, {repo!r})
from foundationstereo_amd import _lib, torch_ops
torch_ops.load()
maps = open("/proc/self/maps").read()
names = sorted({{l.split()[-1].rsplit("/", 1)[-1] for l in maps.splitlines() if "libfsmi" in l}})
print("LOADED", ",".join(names))
"""


@pytest.mark.parametrize("precision,expect", [("fast", "libfsmi_fast.so"), ("parity", "libfsmi.so")])
def test_one_runtime_mapped(precision, expect):
    from foundationstereo_amd import _lib, torch_ops
    if not (os.path.exists(_lib.LIB_FAST) and os.path.exists(_lib.LIB) and os.path.exists(torch_ops.EXT)):
        pytest.skip("libraries not built")
    env = dict(os.environ, FSMI_PRECISION=precision)
    env.pop("FSMI_LIB", None)
    r = subprocess.run([sys.executable, "-c", CHILD.format(repo=REPO)], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("LOADED")][-1]
    assert line.split()[1].split(",") == [expect], line
