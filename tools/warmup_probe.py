"""Find what makes the first forward slow: per-leaf-module wall time with syncs."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from foundationstereo_amd import synth
from foundationstereo_amd.foundation_stereo import FoundationStereo
torch.backends.cudnn.benchmark = bool(int(os.environ.get("CB", "1")))
dev = torch.device("cuda:0")
args = synth.make_args(max_disp=192, corr_levels=4, vit_size="vits")
m = FoundationStereo(args).eval(); synth.init_module_(m); m = m.to(dev)
fl, fr, vf = synth.backbone_features(1, 480, 640, "vits", shift_px=8)
m.feature.set_features([torch.from_numpy(a).to(dev) for a in fl], [torch.from_numpy(a).to(dev) for a in fr], torch.from_numpy(vf).to(dev))
l, r = synth.stereo_images(1, 480, 640)
l, r = torch.from_numpy(l).to(dev), torch.from_numpy(r).to(dev)
times = {}
def pre(mod, inp):
    torch.cuda.synchronize(); mod._t0 = time.perf_counter()
def post(mod, inp, out):
    torch.cuda.synchronize(); dt = time.perf_counter() - mod._t0
    w = getattr(mod, 'weight', None)
    key = (type(mod).__name__, str(tuple(w.shape)) if w is not None else '')
    times[key] = times.get(key, 0) + dt
hs = []
for name, mod in m.named_modules():
    if len(list(mod.children())) == 0:
        hs.append(mod.register_forward_pre_hook(pre)); hs.append(mod.register_forward_hook(post))
t0 = time.perf_counter()
with torch.no_grad():
    m(l, r, iters=2, test_mode=True)
torch.cuda.synchronize()
print("first forward", time.perf_counter() - t0)
for k, v in sorted(times.items(), key=lambda kv: -kv[1])[:25]:
    print(f"{v:8.2f}s {k}")
for h in hs: h.remove()
t0 = time.perf_counter()
with torch.no_grad():
    m(l, r, iters=2, test_mode=True)
torch.cuda.synchronize()
print("second forward", time.perf_counter() - t0)
