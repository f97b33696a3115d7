#!/usr/bin/env python3
"""Is the captured forward bound by the host's graph launch?  Times, for the cfg2 forward captured
as one hipGraph (bench.py's timed step): the host time of ``replay()`` (hipGraphLaunch returning),
the device time of the replay (events around it), and back-to-back replays.  If the launch call
takes about as long as the device work, the GPU waits on the host submitting the graph's nodes.

    python tools/graph_launch_probe.py [--config cfg2] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from foundationstereo_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg2")
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda:0")
H, W, md, iters, vit, per = bench.CONFIGS[a.config]
args = synth.make_args(max_disp=md, corr_levels=4, vit_size=vit)
model = bench.make_model(args, dev, 0)
feats = [synth.backbone_features(1, H, W, vit, seed=0x5EED + i, shift_px=8) for i in range(per)]
fl = [torch.from_numpy(np.concatenate([f[0][j] for f in feats])).to(dev) for j in range(4)]
fr = [torch.from_numpy(np.concatenate([f[1][j] for f in feats])).to(dev) for j in range(4)]
vf = torch.from_numpy(np.concatenate([f[2] for f in feats])).to(dev)
model.feature.set_features(fl, fr, vf, size=(H, W))
left, right = synth.stereo_images(per, H, W)
L, R = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
from foundationstereo_amd import update as fupdate  # noqa: E402


def fwd():
    return model(L, R, iters=iters, test_mode=True)


def probe(mode):
    """mode: graph4 (bench.py's step: 4 streams, captured), graph1 (one stream, captured), eager4."""
    fupdate.OVERLAP = mode != "graph1"
    with torch.no_grad():
        for _ in range(2):
            fwd()
        torch.cuda.synchronize()
        run = fwd
        if mode.startswith("graph"):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fwd()
            run = g.replay
        run()
        torch.cuda.synchronize()
        res = {"mode": mode, "single": []}
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            t0 = time.perf_counter()
            run()
            t1 = time.perf_counter()
            e1.record()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            res["single"].append({"host_ms": round((t1 - t0) * 1e3, 2), "device_ms": round(e0.elapsed_time(e1), 2),
                                  "wall_ms": round((t2 - t0) * 1e3, 2)})
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            run()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res["batch"] = {"host_ms_per": round((t1 - t0) * 1e3 / a.reps, 2),
                        "wall_ms_per": round((t2 - t0) * 1e3 / a.reps, 2)}
    fupdate.OVERLAP = True
    print(json.dumps(res), flush=True)


for m in ("graph4", "graph1", "eager4"):
    probe(m)
