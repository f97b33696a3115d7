"""World-size-2 sharding of the REAL model on the GPU box: two spawned processes (both on
cuda:0, gloo collectives staged through the host -- one card on the box), each running
``ShardedStereo`` over ``FoundationStereo`` eagerly and then from its captured hipGraph, vs one
process running the same two pairs as one batch.  The RCCL path is the same code with device
tensors in the collectives (bench.py under torchrun)."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

H, W, MD, ITERS = 64, 96, 32, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(seed):
    from foundationstereo_amd import synth
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    args = synth.make_args(max_disp=MD, corr_levels=2, vit_size="vits")
    m = FoundationStereo(args).eval()
    synth.init_module_(m, seed=seed)
    return m.to("cuda:0")


def _features(lo, hi):
    from foundationstereo_amd import synth
    fl, fr, vf = synth.backbone_features(2, H, W, "vits", shift_px=2)
    dev = "cuda:0"
    return ([torch.from_numpy(a[lo:hi]).to(dev) for a in fl], [torch.from_numpy(a[lo:hi]).to(dev) for a in fr],
            torch.from_numpy(vf[lo:hi]).to(dev))


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from foundationstereo_amd import dist as fdist, synth
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        m = _model(seed=1234 if rank == 0 else 99)        # rank 1 starts with other weights
        fdist.broadcast_module_(m, src=0)
        lo, hi = fdist.shard_range(2, rank, world)
        m.feature.set_features(*_features(lo, hi))
        left, right = synth.stereo_images(2, H, W)
        full = torch.from_numpy(np.stack([left, right], 1)).to("cuda:0")
        batch = full if rank == 0 else torch.zeros_like(full)
        runner = fdist.ShardedStereo(lambda lf, rt: m(lf, rt, iters=ITERS, test_mode=True), rank, world)
        with torch.no_grad():
            eager = runner.step(batch, (1, H, W)).cpu()
            runner.capture(batch)
            replay = runner.step(batch, (1, H, W)).cpu()
        q.put((rank, eager.numpy(), replay.numpy()))
    finally:
        dist.destroy_process_group()


def test_sharded_real_model_world2():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda r: r[0])
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    from foundationstereo_amd import synth
    m = _model(seed=1234)
    m.feature.set_features(*_features(0, 2))
    left, right = synth.stereo_images(2, H, W)
    with torch.no_grad():
        single = m(torch.from_numpy(left).cuda(), torch.from_numpy(right).cuda(), iters=ITERS,
                   test_mode=True).cpu().numpy()
    for rank, eager, replay in res:
        assert eager.shape == (2, 1, H, W)
        np.testing.assert_allclose(eager, single, atol=1e-4, rtol=0)    # batch invariance (fp32 order)
        np.testing.assert_allclose(replay, eager, atol=1e-5, rtol=0)     # graph == eager


def _nccl_worker(port, q):
    import torch.distributed as dist
    from foundationstereo_amd import dist as fdist, ops, synth
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    rank, _, world = fdist.init_from_env("nccl", force=True)
    try:
        assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
        m = _model(seed=1234)
        fdist.broadcast_module_(m, src=0)
        m.feature.set_features(*_features(0, 2))
        left, right = synth.stereo_images(2, H, W)
        batch = torch.from_numpy(np.stack([left, right], 1)).to("cuda:0")
        runner = fdist.ShardedStereo(lambda lf, rt: m(lf, rt, iters=ITERS, test_mode=True), rank, world)
        with torch.no_grad():
            eager = runner.step(batch, (1, H, W)).cpu()
            runner.capture(batch)
            replay = runner.step(batch, (1, H, W)).cpu()
        q.put((eager.numpy(), replay.numpy()))
    finally:
        dist.destroy_process_group()


def test_sharded_real_model_rccl_world1():
    """The "nccl" (RCCL) branch of ShardedStereo on hardware: a process group of one rank, so the
    step's scatter and all_gather_into_tensor run as RCCL collectives on device tensors (the 8-GPU
    path bench.py takes under torchrun), eagerly and around a captured replay; same result as the
    single-process forward."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), q))
    p.start()
    try:
        eager, replay = q.get(timeout=240)
    finally:
        p.join(timeout=60)
    assert p.exitcode == 0
    from foundationstereo_amd import synth
    m = _model(seed=1234)
    m.feature.set_features(*_features(0, 2))
    left, right = synth.stereo_images(2, H, W)
    with torch.no_grad():
        single = m(torch.from_numpy(left).cuda(), torch.from_numpy(right).cuda(), iters=ITERS,
                   test_mode=True).cpu().numpy()
    assert eager.shape == (2, 1, H, W)
    np.testing.assert_allclose(eager, single, atol=1e-5, rtol=0)
    np.testing.assert_allclose(replay, eager, atol=1e-5, rtol=0)
