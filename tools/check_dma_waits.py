#!/usr/bin/env python3
"""Static check of the pointwise tiles' LDS-DMA ring waits in the shipped gfx950 code.

    python tools/check_dma_waits.py [lib.so ...]      (default: _lib/libfsmi.so and _lib/libfsmi_fast.so)

``conv_pw_kernel`` (csrc/conv_pw.hip) moves input chunks global -> LDS with inline-asm
``global_load_lds_dwordx4`` the compiler does not see, and waits for them with hand-computed
``s_waitcnt vmcnt(N)`` before the barrier that opens each chunk: N counts the memory operations the
kernel issues AFTER the chunk's DMA (the later chunks' DMAs and the weight loads, ``WLD``).  vmcnt
retires in issue order, so the wait covers chunk q's DMA iff at least N vector-memory instructions
were issued after chunk q's youngest DMA instruction on EVERY path that reaches the wait.  Round 4
shipped a build whose compiler dropped loads the count still included (the one-product build's lo
weight halves): the first chunk was read before it landed.

This tool disassembles the code object embedded in each library (the offload bundle of every
translation unit in ``.hip_fatbin``), splits every ``conv_pw_kernel`` instantiation into basic blocks
and, for every ``s_waitcnt`` carrying a vmcnt right before an ``s_barrier``, walks all paths backward
(through the loop back edge and into the prologue) to chunk q's DMA -- the ((NS-2)*OPS + 1)-th DMA
instruction back, NS and OPS from the template arguments -- counting the vector-memory instructions
in between.  A wait is UNSAFE when some path has fewer than N; it is reported EXACT when N equals the
minimum over paths of the operations issued after chunk q's DMA or chunk q's weights, whichever
retires later (the weights of chunk q are waited for by the same instruction by design).

Test infrastructure: tests/test_dma_waits.py runs it on both libraries and on a build compiled with a
deliberately wrong WLD (``-DFSMI_PW_WLD_ADJ=...``), which must be flagged.
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin/"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TRIPLE = "hipv4-amdgcn-amd-amdhsa--gfx950"

_INSN = re.compile(r"^\s+([a-z_0-9]+)(.*?)\s*//\s*([0-9A-Fa-f]+):")
_SYM = re.compile(r"^([0-9a-f]+) <(.+)>:$")
_TARGET = re.compile(r"<(.+?)\+0x([0-9a-f]+)>|<(.+?)>\s*$")
_PW = re.compile(r"conv_pw_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELb([01])E")


def code_objects(path: str):
    """The gfx950 ELF code objects of every offload bundle in ``path``'s .hip_fatbin section
    (an object file holds one bundle, a linked library one per translation unit)."""
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fb")
        subprocess.run([LLVM + "llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", path, os.path.join(d, "x")],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    out = []
    for s in starts:
        p = s + len(MAGIC)
        (n,) = struct.unpack_from("<Q", data, p)
        p += 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tlen].decode()
            p += tlen
            if triple == TRIPLE and size:
                out.append(data[s + off:s + off + size])
    return out


def disassemble(co: bytes) -> str:
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, "co")
        open(f, "wb").write(co)
        return subprocess.run([LLVM + "llvm-objdump", "-d", "--no-show-raw-insn", f], check=True,
                              capture_output=True, text=True).stdout


def kernels(dis: str):
    """{symbol: [(addr, mnemonic, operands, target_addr or None)]} for every conv_pw_kernel."""
    out, cur, base = {}, None, 0
    for line in dis.splitlines():
        m = _SYM.match(line)
        if m:
            name = m.group(2)
            cur = name if _PW.search(name) else None
            base = int(m.group(1), 16)
            if cur:
                out[cur] = []
            continue
        if cur is None:
            continue
        m = _INSN.match(line)
        if not m:
            continue
        mn, ops, addr = m.group(1), m.group(2), int(m.group(3), 16)
        tgt = None
        if mn.startswith("s_branch") or mn.startswith("s_cbranch"):
            t = _TARGET.search(line)
            if t and t.group(2):
                tgt = base + int(t.group(2), 16)
            elif t:
                tgt = base
        out[cur].append((addr, mn, ops, tgt))
    return out


def is_vmem(mn: str) -> bool:
    return mn.startswith(("global_", "buffer_", "flat_", "scratch_"))


def is_dma(mn: str) -> bool:
    return mn.startswith("global_load_lds") or (mn.startswith("buffer_load") and "lds" in mn)


def vmcnt(ops: str):
    m = re.search(r"vmcnt\((\d+)\)", ops)
    return int(m.group(1)) if m else None


def blocks(insns):
    """Basic blocks: list of (start_index, end_index_exclusive), plus predecessor lists."""
    addr_idx = {a: i for i, (a, *_r) in enumerate(insns)}
    leaders = {0}
    for i, (_a, mn, _o, tgt) in enumerate(insns):
        if tgt is not None:
            if tgt in addr_idx:
                leaders.add(addr_idx[tgt])
            leaders.add(i + 1)
        elif mn in ("s_endpgm", "s_setpc_b64"):
            leaders.add(i + 1)
    ls = sorted(x for x in leaders if x < len(insns))
    spans = [(s, (ls[k + 1] if k + 1 < len(ls) else len(insns))) for k, s in enumerate(ls)]
    blk_of = {}
    for b, (s, e) in enumerate(spans):
        for i in range(s, e):
            blk_of[i] = b
    preds = [[] for _ in spans]
    for b, (s, e) in enumerate(spans):
        last = insns[e - 1]
        mn, tgt = last[1], last[3]
        if tgt is not None and tgt in addr_idx:
            preds[blk_of[addr_idx[tgt]]].append(b)
        falls = not (mn.startswith("s_branch") or mn in ("s_endpgm", "s_setpc_b64"))
        if falls and b + 1 < len(spans):
            preds[b + 1].append(b)
    return spans, blk_of, preds


def weight_loads(mn: str) -> bool:
    """The register-staged weight fragments (load_wf): 16-B global loads."""
    return mn == "global_load_dwordx4"


def walk_back(insns, spans, blk_of, preds, i0, need_dma):
    """Every backward path from instruction i0 (exclusive) to the need_dma-th DMA instruction back:
    (minimum over paths of the vector-memory instructions issued after that DMA, whether some path
    reaches the kernel entry first).  Memoised on (block, DMAs seen): a path entering a block with as
    many DMAs behind it and no fewer memory ops than an earlier one cannot lower the minimum, so
    loops without DMAs terminate and the diamond branches of a step do not multiply."""
    best = {}
    y_min = None
    entry = False
    stack = [(blk_of[i0], i0 - 1, 0, 0)]     # (block, index, dma seen, vmem seen)
    while stack:
        b, i, nd, nv = stack.pop()
        s, _e = spans[b]
        done = False
        while i >= s:
            mn = insns[i][1]
            if is_dma(mn):
                nd += 1
                if nd == need_dma:
                    y_min = nv if y_min is None else min(y_min, nv)
                    done = True
                    break
            if is_vmem(mn):
                nv += 1
            i -= 1
        if done:
            continue
        if not preds[b]:
            entry = True            # reached the kernel entry without passing chunk q's DMA
            continue
        for p in preds[b]:
            key = (p, nd)
            if key in best and best[key] <= nv:
                continue
            best[key] = nv
            stack.append((p, spans[p][1] - 1, nd, nv))
    return y_min, entry


def check_kernel(name, insns):
    """Findings for one instantiation: list of dicts (one per ring wait)."""
    m = _PW.search(name)
    BM, PX, WM, NS, coop = (int(x) for x in m.groups())
    OPS = 32 * PX // 1024
    need = (NS - 2) * OPS + 1
    spans, blk_of, preds = blocks(insns)
    found = []
    for i, (addr, mn, ops, _t) in enumerate(insns):
        if mn != "s_barrier":
            continue
        # the nearest s_waitcnt before the barrier in its block, with no memory op between
        j = i - 1
        s = spans[blk_of[i]][0]
        w = None
        while j >= s:
            mj = insns[j][1]
            if is_vmem(mj):
                break
            if mj == "s_waitcnt":
                w = j
                break
            j -= 1
        if w is None or vmcnt(insns[w][2]) is None:
            continue
        n = vmcnt(insns[w][2])
        y, entry = walk_back(insns, spans, blk_of, preds, w, need)
        unsafe = entry or y is None or y < n
        found.append({"addr": addr, "vmcnt": n, "min_after_dma": y, "from_entry": entry, "unsafe": unsafe})
    return {"BM": BM, "PX": PX, "WM": WM, "NS": NS, "coop": bool(coop), "OPS": OPS, "waits": found}


def check_library(path):
    """{kernel symbol: check_kernel result} over every conv_pw_kernel in ``path``."""
    res = {}
    for co in code_objects(path):
        dis = disassemble(co)
        if "conv_pw_kernel" not in dis:
            continue
        for name, insns in kernels(dis).items():
            res[name] = check_kernel(name, insns)
    return res


def short(name):
    m = _PW.search(name)
    return "conv_pw_kernel<%s,%s,%s,%s,%s>" % m.groups()


def main(argv):
    libs = argv or [os.path.join(REPO, "foundationstereo_amd", "_lib", f) for f in ("libfsmi.so", "libfsmi_fast.so")]
    bad = 0
    for lib in libs:
        res = check_library(lib)
        print(f"{lib}: {len(res)} conv_pw_kernel instantiations")
        for name, r in sorted(res.items()):
            for w in r["waits"]:
                tag = "UNSAFE" if w["unsafe"] else "ok"
                bad += w["unsafe"]
                print(f"  {short(name):38s} wait@{w['addr']:#x} vmcnt({w['vmcnt']:2d})  min ops after chunk DMA "
                      f"{w['min_after_dma']}{'  (a path from the entry has no such DMA)' if w['from_entry'] else ''}"
                      f"  {tag}")
            if not r["waits"]:
                print(f"  {short(name)}: NO ring waits found")
                bad += 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
