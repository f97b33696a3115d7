import sys, numpy as np, torch
sys.path.insert(0, '/root/repo')
import oracle
from foundationstereo_amd import synth, ops
from foundationstereo_amd.geometry import Combined_Geo_Encoding_Volume
L, D, W = 4, 80, 96
B, C, Cv, H = 1, 64, 28, 4
dev = 'cuda'
f1, f2 = synth.normal(61, (B, C, H, W)), synth.normal(62, (B, C, H, W))
vol = synth.normal(63, (B, Cv, D, H, W))
disp = synth.uniform(64, (B, 1, H, W), -8.0, D + 8.0)
disp[0, 0, 0, :6] = [0.0, 1.0, D - 1.0, D, -1.0, 2.5]
T = lambda a: torch.from_numpy(a)
ge = Combined_Geo_Encoding_Volume(T(f1).to(dev), T(f2).to(dev), T(vol).to(dev), num_levels=L, dx=torch.linspace(-4, 4, 9))
out = ge(T(disp).to(dev)).cpu()
ref = oracle.GeoEncoding(T(f1), T(f2), T(vol), L, 4)
coords = torch.arange(W, dtype=torch.float).view(1, 1, W, 1).repeat(B, H, 1, 1)
r = ref(T(disp), coords)
d = (out - r).abs()
print("max", d.max().item(), "n>1e-5", (d > 1e-5).sum().item(), "n>2e-6", (d > 2e-6).sum().item())
print("vol exact copy? ", out[0,0,0,2].item(), r[0,0,0,2].item(), vol[0,0,75,0,2])
idx = torch.nonzero(d > 3e-6)[:20]
K=9
for b,ch,h,w in idx.tolist():
    lvl = ch // (K*(Cv+1)); rem = ch % (K*(Cv+1))
    kind = 'geo' if rem < K*Cv else 'corr'
    print(lvl, kind, rem//K, rem%K, h, w, 'disp', disp[0,0,h,w], 'gpu', out[b,ch,h,w].item(), 'ora', r[b,ch,h,w].item())
# corr pyramid diff
for i in range(L):
    print('corr lvl', i, (ge.init_corr_pyramid[i].cpu().reshape(-1) - ref.cor[i].reshape(-1)).abs().max().item())
print('vol lvl', [ (ge.geo_volume_pyramid[i].cpu().permute(0,3,4,1,2).reshape(-1) - ref.geo[i].reshape(-1)).abs().max().item() for i in range(L)])
