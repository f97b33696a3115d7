#!/usr/bin/env python3
"""Per-kernel register / scratch / LDS usage of a hipcc object (gfx950), from its code-object notes.

    python tools/kernel_regs.py build/fsmi/conv_halo_x3.o [name-filter]
"""
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin/"
obj, filt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
with tempfile.TemporaryDirectory() as d:
    subprocess.run([LLVM + "llvm-objcopy", f"--dump-section=.hip_fatbin={d}/fb", obj], check=True)
    subprocess.run([LLVM + "clang-offload-bundler", "--unbundle", "--type=o", f"--input={d}/fb",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={d}/co"], check=True)
    notes = subprocess.run([LLVM + "llvm-readelf", "--notes", f"{d}/co"], capture_output=True, text=True).stdout
cur = {}
rows = []
for line in notes.splitlines():
    m = re.match(r"\s+-?\s*\.(\w+):\s+(\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "agpr_count" and cur:
        rows.append(cur)
        cur = {}
    cur[k] = v
rows.append(cur)
print(f"{'vgpr':>5} {'agpr':>5} {'sgpr':>5} {'scratch':>7} {'lds':>6}  kernel")
for r in rows:
    n = r.get("name", "?")
    if filt in n and "vgpr_count" in r:
        n = re.sub(r"_ZN4fsmi12_GLOBAL__N_1\d+", "", n)
        print(f"{r['vgpr_count']:>5} {r.get('agpr_count', '0'):>5} {r.get('sgpr_count', '?'):>5} "
              f"{r.get('private_segment_fixed_size', '?'):>7} {r.get('group_segment_fixed_size', '?'):>6}  {n}")
