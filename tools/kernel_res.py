#!/usr/bin/env python3
"""VGPR / AGPR / spill / LDS figures of the kernels in a built library whose symbol matches a regex
(llvm-readelf --notes on the embedded gfx950 code objects).

    python tools/kernel_res.py [--lib foundationstereo_amd/_lib/libfsmi.so] REGEX"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import check_dma_waits as c  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("regex")
ap.add_argument("--lib", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                              "foundationstereo_amd", "_lib", "libfsmi.so"))
a = ap.parse_args()
pat = re.compile(a.regex)
FIELDS = (".vgpr_count", ".agpr_count", ".vgpr_spill_count", ".sgpr_spill_count", ".private_segment_fixed_size",
          ".group_segment_fixed_size")
for co in c.code_objects(a.lib):
    with tempfile.NamedTemporaryFile() as f:
        f.write(co)
        f.flush()
        notes = subprocess.run([c.LLVM + "llvm-readelf", "--notes", f.name], capture_output=True, text=True).stdout
    # one YAML map per kernel: split at each "- .agpr_count" (the first key of a kernel's map)
    for blk in re.split(r"\n\s+- \.agpr_count", notes)[1:]:
        blk = ".agpr_count" + blk
        m = re.search(r"\.name:\s+(\S+)", blk)
        if not m or not pat.search(m.group(1)):
            continue
        vals = {k[1:]: (re.search(re.escape(k) + r":\s+(\d+)", blk) or [None, "?"])[1] for k in FIELDS}
        print(m.group(1)[:90], vals)
