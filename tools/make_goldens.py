#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE modules on the CPU.

Runs only in the build container (``/root/reference`` is absent on the GPU
box).  Inputs and weights come from ``foundationstereo_amd.synth`` (hash PRNG),
so only outputs and small per-op inputs are stored; tests regenerate the rest.

    PYTHONDONTWRITEBYTECODE=1 python tools/make_goldens.py

Writes ``tests/golden/*.npz`` and ``tests/golden/state_dict_*.json``.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

from foundationstereo_amd import synth  # noqa: E402
from ref_harness import import_reference, import_reference_extractor, make_synthetic_feature_class  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")
torch.set_num_threads(8)


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def ops_small(sm, geo_mod, ut):
    g = {}
    # a1: gwc volume, border case D close to W
    for tag, (B, C, G, H, W, D) in {"a": (2, 32, 8, 4, 24, 8), "b": (1, 64, 8, 3, 16, 16)}.items():
        fl = synth.normal(synth.name_seed(f"gwcL{tag}"), (B, C, H, W))
        fr = synth.normal(synth.name_seed(f"gwcR{tag}"), (B, C, H, W))
        out = sm.build_gwc_volume(t(fl), t(fr), D, G)
        g[f"gwc_{tag}_fl"], g[f"gwc_{tag}_fr"], g[f"gwc_{tag}_out"] = fl, fr, out.numpy()
        g[f"gwc_{tag}_meta"] = np.array([B, C, G, H, W, D])
    # a2: concat volume
    B, C, H, W, D = 2, 12, 4, 24, 8
    pl = synth.normal(synth.name_seed("catL"), (B, C, H, W))
    pr = synth.normal(synth.name_seed("catR"), (B, C, H, W))
    g["concat_pl"], g["concat_pr"] = pl, pr
    g["concat_out"] = sm.build_concat_volume(t(pl), t(pr), D).numpy()
    g["concat_meta"] = np.array([B, C, H, W, D])
    # a4: softmax + regression
    logits = synth.normal(synth.name_seed("reg"), (2, 16, 4, 6), std=3.0)
    prob = torch.softmax(t(logits), 1)
    g["reg_logits"] = logits
    g["reg_prob"] = prob.numpy()
    g["reg_out"] = sm.disparity_regression(prob, 16).numpy()
    # a9: context upsample
    dl = synth.normal(synth.name_seed("upd"), (2, 1, 4, 6), std=5.0)
    w = torch.softmax(t(synth.normal(synth.name_seed("upw"), (2, 9, 16, 24))), 1)
    g["up_disp"], g["up_w"] = dl, w.numpy()
    g["up_out"] = sm.context_upsample(t(dl), w).numpy()
    # a5/a6: geometry encoding init + lookup, L in {2,4}; border cases in disp
    for L in (2, 4):
        B, C, Cv, D, H, W = 2, 32, 28, 16, 4, 24
        f1 = synth.normal(synth.name_seed(f"geo1_{L}"), (B, C, H, W))
        f2 = synth.normal(synth.name_seed(f"geo2_{L}"), (B, C, H, W))
        vol = synth.normal(synth.name_seed(f"geov_{L}"), (B, Cv, D, H, W))
        disp = synth.uniform(synth.name_seed(f"geod_{L}"), (B, 1, H, W), -6.0, D + 6.0)
        disp[0, 0, 0, :4] = [0.0, 3.0, D - 1.0, -4.0]     # exact integers / far outside
        disp[0, 0, 1, :3] = [D + 4.0, 0.5, 1e-3]
        dx = torch.linspace(-4, 4, 9).reshape(1, 1, 9, 1)
        ge = geo_mod.Combined_Geo_Encoding_Volume(t(f1), t(f2), t(vol), num_levels=L, dx=dx)
        coords = torch.arange(W, dtype=torch.float).reshape(1, 1, W, 1).repeat(B, H, 1, 1)
        out = ge(t(disp), coords)
        p = f"geo{L}_"
        g[p + "f1"], g[p + "f2"], g[p + "vol"], g[p + "disp"] = f1, f2, vol, disp
        g[p + "out"] = out.numpy()
        g[p + "corr"] = geo_mod.Combined_Geo_Encoding_Volume.corr(t(f1), t(f2)).numpy()
        for i, c in enumerate(ge.init_corr_pyramid):
            g[p + f"corrpyr{i}"] = c.numpy()
        g[p + "volpyr1"] = ge.geo_volume_pyramid[1].numpy()
    # bilinear_sampler 1-D (utils.py:44-55)
    img = synth.normal(synth.name_seed("bs_img"), (6, 3, 1, 11))
    x = synth.uniform(synth.name_seed("bs_x"), (6, 1, 9, 1), -2.0, 12.0)
    coords = np.concatenate([x, np.zeros_like(x)], -1)
    g["bs_img"], g["bs_coords"] = img, coords
    g["bs_out"] = ut.bilinear_sampler(t(img), t(coords)).numpy()
    np.savez_compressed(os.path.join(OUT, "ops_small.npz"), **g)
    print("ops_small", sum(v.nbytes for v in g.values()) / 1e6, "MB raw")


def update_step(up_mod):
    args = synth.make_args(max_disp=64, corr_levels=2)
    blk = up_mod.BasicSelectiveMultiUpdateBlock(args, 128, volume_dim=28).eval()
    synth.init_module_(blk, seed=77)
    B, H, W = 1, 8, 12
    cor_planes = 2 * 9 * 29
    sizes = [(H, W), (H // 2, W // 2), (H // 4, W // 4)]
    net = [synth.normal(synth.name_seed(f"net{i}"), (B, 128) + s, 0.5) for i, s in enumerate(sizes)]
    inp = [np.abs(synth.normal(synth.name_seed(f"inp{i}"), (B, 128) + s, 0.5)) for i, s in enumerate(sizes)]
    att = [synth.uniform(synth.name_seed(f"att{i}"), (B, 1) + s) for i, s in enumerate(sizes)]
    corr = synth.normal(synth.name_seed("ucorr"), (B, cor_planes, H, W), 0.5)
    disp = synth.uniform(synth.name_seed("udisp"), (B, 1, H, W), 0.0, 16.0)
    with torch.no_grad():
        onet, mask, delta = blk([t(x) for x in net], [t(x) for x in inp], t(corr), t(disp), [t(x) for x in att])
    g = {"disp": disp, "corr": corr, "mask": mask.numpy(), "delta": delta.numpy()}
    for i in range(3):
        g[f"net{i}"], g[f"inp{i}"], g[f"att{i}"], g[f"onet{i}"] = net[i], inp[i], att[i], onet[i].numpy()
    np.savez_compressed(os.path.join(OUT, "update_step.npz"), **g)
    print("update_step done")


E2E_CASES = {
    # name: (H, W, max_disp, iters, vit, corr_levels, shift)
    "e2e_tiny": (64, 96, 32, 4, "vits", 2, 2),
    "e2e_cfg1_L2": (256, 320, 64, 8, "vits", 2, 6),
    "e2e_cfg1_L4": (256, 320, 64, 8, "vits", 4, 6),
}


def e2e(fs):
    Syn = make_synthetic_feature_class(synth.feature_dims)
    fs.Feature = Syn
    for name, (H, W, md, iters, vit, L, shift) in E2E_CASES.items():
        args = synth.make_args(max_disp=md, corr_levels=L, vit_size=vit)
        model = fs.FoundationStereo(args).eval()
        synth.init_module_(model, seed=1234)
        fl, fr, vf = synth.backbone_features(1, H, W, vit, shift_px=shift)
        left, right = synth.stereo_images(1, H, W)
        model.feature.preset = ([t(x) for x in fl], [t(x) for x in fr], t(vf))
        cap = {}

        orig_call = fs.Combined_Geo_Encoding_Volume.__call__

        def hook(self, disp, coords, low_memory=False):
            out = orig_call(self, disp, coords, low_memory)
            if "geo0" not in cap:
                cap["geo0"] = out.detach().clone()
                cap["init_disp"] = disp.detach().clone()
            return out

        fs.Combined_Geo_Encoding_Volume.__call__ = hook
        try:
            with torch.no_grad():
                out = model(t(left), t(right), iters=iters, test_mode=True)
        finally:
            fs.Combined_Geo_Encoding_Volume.__call__ = orig_call
        g = {"disp": out.numpy(), "init_disp": cap["init_disp"].numpy(),
             "geo0_sum": np.float64(cap["geo0"].double().sum()),
             "geo0_abs": np.float64(cap["geo0"].double().abs().sum()),
             "geo0_row": cap["geo0"][0, :, 3, :].numpy(),
             "meta": np.array([H, W, md, iters, L, shift])}
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **g)
        print(name, "disp mean", float(out.mean()), "init mean", float(cap["init_disp"].mean()))
        if name == "e2e_tiny":
            for v in ("vits", "vitl"):
                a2 = synth.make_args(max_disp=192, corr_levels=4, vit_size=v)
                m2 = fs.FoundationStereo(a2)
                keys = [[k, list(p.shape)] for k, p in m2.state_dict().items()]
                with open(os.path.join(OUT, f"state_dict_{v}.json"), "w") as f:
                    json.dump(keys, f)


# name: (H, W, max_disp, iters, vit, corr_levels, shift): both passes need /32 padding, so the
# reference's ``+= padder._pad[0]`` (core/foundation_stereo.py:270) is exercised (_pad[0] = 10)
HIERA_CASES = {"hiera_small": (200, 300, 64, 4, "vits", 2, 3)}


def hiera(fs):
    """run_hierachical (core/foundation_stereo.py:257-274) with the backbone stand-in synthesising
    features at each pass's padded size (as the product's SyntheticFeature does unpreset)."""
    Syn = make_synthetic_feature_class(synth.feature_dims)
    fs.Feature = Syn
    for name, (H, W, md, iters, vit, L, shift) in HIERA_CASES.items():
        args = synth.make_args(max_disp=md, corr_levels=L, vit_size=vit)
        model = fs.FoundationStereo(args).eval()
        synth.init_module_(model, seed=1234)
        model.feature.by_size = (vit, shift)
        left, right = synth.stereo_images(1, H, W)
        cap = []
        orig_fwd = fs.FoundationStereo.forward

        def fwd(self, *a, **k):
            out = orig_fwd(self, *a, **k)
            cap.append(out.detach().clone())
            return out

        fs.FoundationStereo.forward = fwd
        try:
            with torch.no_grad():
                out = model.run_hierachical(t(left), t(right), iters=iters, test_mode=True)
        finally:
            fs.FoundationStereo.forward = orig_fwd
        g = {"disp": out.numpy(), "disp_small_padded": cap[0].numpy(),
             "meta": np.array([H, W, md, iters, L, shift])}
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **g)
        print(name, "disp", tuple(out.shape), "mean", float(out.mean()))


BACKBONE_CASES = {
    # name: (encoder, input shape) -- DepthAnythingFeature on an already /14 input
    "dav2_vits": ("vits", (2, 3, 56, 70)),
    "dav2_vitl": ("vitl", (1, 3, 28, 42)),
}
FEATURE_CASES = {"feature_vits": ("vits", (2, 3, 64, 96))}


def backbone():
    """DepthAnythingFeature (core/extractor.py:286-320) and Feature (:323-369) run by the reference,
    hash-initialised; inputs from synth (regenerated by the tests)."""
    ext = import_reference_extractor()
    for name, (enc, shape) in BACKBONE_CASES.items():
        m = ext.DepthAnythingFeature(encoder=enc).eval()
        synth.init_module_(m, seed=4321)
        x = synth.normal(synth.name_seed(name + "_x"), shape)
        with torch.no_grad():
            out = m(t(x))
        g = {k: out[k].numpy() for k in ("out", "path_1", "path_2", "path_3", "path_4", "disp")}
        for i, (tok, cls) in enumerate(out["features"]):
            g[f"feat{i}"], g[f"cls{i}"] = tok.numpy(), cls.numpy()
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **g)
        with open(os.path.join(OUT, f"state_dict_{name}.json"), "w") as f:
            json.dump([[k, list(v.shape)] for k, v in m.state_dict().items()], f)
        print(name, {k: v.shape for k, v in g.items()})
    for name, (vit, shape) in FEATURE_CASES.items():
        args = synth.make_args(vit_size=vit)
        m = ext.Feature(args).eval()
        synth.init_module_(m, seed=4321)
        x = synth.normal(synth.name_seed(name + "_x"), shape)
        with torch.no_grad():
            feats, vit_feat = m(t(x))
        g = {f"x{4 << i}": f.numpy() for i, f in enumerate(feats)}
        g["vit_feat"] = vit_feat.numpy()
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **g)
        with open(os.path.join(OUT, f"state_dict_{name}.json"), "w") as f:
            json.dump([[k, list(v.shape)] for k, v in m.state_dict().items()], f)
        print(name, {k: v.shape for k, v in g.items()})
    # the whole model with its real backbone: the checkpoint layout (feature.* included)
    fs, *_ = import_reference()
    fs.Feature = ext.Feature
    for vit in ("vits", "vitl"):
        m = fs.FoundationStereo(synth.make_args(max_disp=192, corr_levels=4, vit_size=vit))
        with open(os.path.join(OUT, f"state_dict_full_{vit}.json"), "w") as f:
            json.dump([[k, list(v.shape)] for k, v in m.state_dict().items()], f)


def main():
    os.makedirs(OUT, exist_ok=True)
    fs, sm, geo_mod, up_mod, ut = import_reference()
    which = sys.argv[1:] or ["ops", "update", "e2e", "hiera", "backbone"]
    if "backbone" in which:
        backbone()
    if "hiera" in which:
        hiera(fs)
    if "ops" in which:
        ops_small(sm, geo_mod, ut)
    if "update" in which:
        update_step(up_mod)
    if "e2e" in which:
        e2e(fs)


if __name__ == "__main__":
    main()
