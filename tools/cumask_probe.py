#!/usr/bin/env python3
"""Do CU masks (hipExtStreamCreateWithCUMask, fsmi_stream_create_cumask) hold for this package's kernels,
eagerly and through hipGraph capture / replay?  Times one cfg2 loop conv (gru04.conv1, 512 -> 512 3x3
at 120x160, ~240 blocks) as the mean over 20 launches:
  eager on the default stream / eager on a stream masked to 64 of the CUs / captured on the masked
  stream and replayed on it / captured on it and replayed on the default stream;
then two convs on two streams at once (64-CU mask vs the rest) against the same pair unmasked.
A masked launch taking ~4x the unmasked one means the mask holds.  GPU box: python tools/cumask_probe.py"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from foundationstereo_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
ncu = torch.cuda.get_device_properties(dev).multi_processor_count


def masked_stream(cus):
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint * words)()
    for c in cus:
        mask[c // 32] |= 1 << (c % 32)
    ptr = ctypes.c_void_p()
    _lib.check(lib.fsmi_stream_create_cumask(ctypes.cast(mask, ctypes.c_void_p), words, ctypes.byref(ptr)),
               "stream_create_cumask")
    return torch.cuda.ExternalStream(ptr.value, device=dev)


def events_us(fn, stream, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        fn()
        torch.cuda.synchronize()
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / reps, 1)


with torch.no_grad():
    x = torch.randn(1, 512, 120, 160, device=dev).abs()
    pk = ops.PackedConv(torch.randn(512, 512, 3, 3, device=dev) * 0.02, mode="halo")
    b = torch.randn(512, device=dev)
    out = torch.empty(1, 512, 120, 160, device=dev)
    conv = lambda: ops.conv2d([x], pk, bias=b, act="relu", out=out)   # noqa: E731
    conv()
    torch.cuda.synchronize()
    default = torch.cuda.current_stream(dev)
    quarter = masked_stream(range(0, ncu, 4))          # every 4th CU: 64 of 256
    first = masked_stream(range(ncu // 4))             # CUs 0 .. 63 in the runtime's numbering
    res = {"ncu": ncu, "eager_default_us": events_us(conv, default), "eager_mask_every4th_us": events_us(conv, quarter),
           "eager_mask_first64_us": events_us(conv, first)}
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(first):
        with torch.cuda.graph(g, stream=first):
            for _ in range(20):
                conv()
    torch.cuda.synchronize()
    for name, st in (("graph_mask_first64_replayed_on_it_us", first), ("graph_mask_first64_replayed_on_default_us", default)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(st):
            g.replay()
            e0.record(st)
            g.replay()
            e1.record(st)
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) * 1e3 / 20, 1)
    print(json.dumps(res), flush=True)
