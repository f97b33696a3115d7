import torch, sys
sys.path.insert(0, '.')
from foundationstereo_amd import ops
dev = torch.device('cuda:0')
for C, H, W in ((128, 120, 160), (256, 120, 160), (128, 60, 80)):
    x = torch.randn(1, C, H, W, device=dev); w = torch.randn(C, 1, 7, 7, device=dev); b = torch.randn(C, device=dev)
    f = lambda: ops.dwconv2d(x, w, b)
    f(); torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20): f()
    g.replay(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    print(C, H, W, round(us, 1), 'us', round(2 * 4 * C * H * W / us / 1e6, 2), 'TB/s')
