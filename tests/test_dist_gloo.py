"""World-size-2 tests of the batch-sharding path on the CPU (gloo).

The GPU run uses backend "nccl" (RCCL); the sharding, broadcast and gather
logic is backend-independent and exercised here with a CPU stand-in for the
per-pair compute.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from foundationstereo_amd.dist import ShardedStereo, broadcast_module_, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pair_fn(left, right):
    # per-pair compute stand-in: any function that treats pairs independently
    return (left - right).abs().mean(1, keepdim=True) + left[:, :1] * 0.5


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(100 + rank)          # ranks start with DIFFERENT weights
        m = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 3), torch.nn.BatchNorm2d(4))
        broadcast_module_(m, src=0)
        sig = torch.cat([p.detach().reshape(-1) for p in m.state_dict().values() if p.is_floating_point()])
        B, H, W = 4, 6, 8
        g = torch.Generator().manual_seed(7)
        full = torch.rand(B, 2, 3, H, W, generator=g)
        batch = full.clone() if rank == 0 else torch.zeros_like(full)   # only rank 0 holds the request
        out = ShardedStereo(_pair_fn, rank, world).step(batch, (1, H, W))
        q.put((rank, sig.numpy(), out.numpy(), _pair_fn(full[:, 0], full[:, 1]).numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_step_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    import numpy as np
    for r in res[1:]:
        np.testing.assert_array_equal(r[1], res[0][1])          # weights broadcast
    for _, _, out, ref in res:
        np.testing.assert_allclose(out, ref, atol=1e-6)         # every rank ends with the full, ordered batch


def test_shard_range_partitions():
    for total in (1, 4, 7, 32):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1
