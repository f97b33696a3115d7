"""Batch sharding across the GPUs of one node.

Stereo pairs are independent (eval-mode BN, per-sample InstanceNorm, no
cross-pair op), so the refinement loop partitions by pair with no
per-iteration communication.  The only exchanges are real data movement:

1. ``broadcast_module_``: rank 0's weights to every rank, once, as ONE
   flattened fp32 buffer per dtype (one RCCL broadcast over xGMI instead of
   ~700 small ones);
2. ``ShardedStereo.step``: rank 0 (the rank that owns the request queue)
   scatters the pairs -- rank k receives only its pairs ``[k*b, (k+1)*b)`` --
   and the disparities come back with one ``all_gather_into_tensor``.

One process per GPU, ``torch.distributed`` with backend "nccl" (= RCCL on
ROCm); the same code runs on "gloo" for the CPU tests.
"""
from __future__ import annotations

import os
from typing import Callable, Tuple

import torch
import torch.distributed as dist

from . import foundation_stereo as _fs
from . import ops


def env_world() -> Tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def init_from_env(backend: str = "nccl", force: bool = False) -> Tuple[int, int, int]:
    """Join the torchrun process group (world > 1).  ``force``: create the group even for a single
    process (rank 0 of 1, on 127.0.0.1), so that a one-GPU run moves its batch and results through
    the same collectives as a multi-GPU one (RCCL with ``backend`` "nccl")."""
    rank, local, world = env_world()
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            import socket
            s = socket.socket()
            s.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(s.getsockname()[1])
            s.close()
        kw = dict(rank=rank, world_size=world)
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local), **kw)
        else:
            dist.init_process_group(backend, **kw)
    return rank, local, world


def shard_range(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced shard [lo, hi) of ``total`` pairs for ``rank``."""
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


@torch.no_grad()
def broadcast_module_(module: torch.nn.Module, src: int = 0):
    """Make every rank's parameters and buffers equal to ``src``'s (flattened per dtype)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return module
    tensors = [t for t in list(module.parameters()) + list(module.buffers())]
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault(t.dtype, []).append(t)
    for dtype, ts in sorted(by_dtype.items(), key=lambda kv: str(kv[0])):
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        if _host_staged():
            flat = flat.cpu()
        dist.broadcast(flat, src=src)
        off = 0
        for t in ts:
            n = t.numel()
            t.copy_(flat[off:off + n].view_as(t))
            off += n
    return module


def _host_staged() -> bool:
    """gloo collectives take host tensors (the CPU tests, and multi-process GPU tests that share
    one device); RCCL ("nccl") moves device memory directly over xGMI."""
    return dist.get_backend() == "gloo"


class ShardedStereo:
    """Run ``fn(left, right) -> disp`` on this rank's shard of a batch held by rank 0.

    Per step, rank 0 SCATTERS the pairs (``batch`` of shape ``(B, 2, 3, H, W)``, [left, right]
    per pair): rank k receives only its ``B / world`` pairs ``[k*b, (k+1)*b)`` into a
    persistent local buffer (1/world of the bytes a broadcast would move to every rank), runs
    them, and the disparities come back with ONE all-gather (every rank ends with the full,
    ordered batch).  ``B % world == 0`` so both collectives are equal-size.  Non-zero ranks may
    pass any tensor of the batch's shape and dtype (only its shape is used).
    """

    def __init__(self, fn: Callable, rank: int, world: int):
        self.fn = fn
        self.rank = rank
        self.world = world
        self._local = None          # this rank's shard, (b, 2, 3, H, W), fixed storage
        self._graph = None          # (hipGraph, static output) after capture()
        self._dtype_checked = False
        # after each replay: synchronise, read the range flag, recover in safe mode (True); or leave
        # it to the graph's NaN fill and the caller's ops.check_range(), with no host sync (False)
        self.recover = True
        # per-phase timing of step() (scatter / this rank's forward / all-gather): None = off, else the
        # marks of each timed step -- HIP events on the current stream (RCCL collectives are ordered
        # with it), host clocks for host-staged gloo; read with phase_times()
        self.timing = None

    def _mark(self, dev):
        if dev.type == "cuda":
            e = torch.cuda.Event(enable_timing=True)
            e.record(torch.cuda.current_stream(dev))
            return e
        import time
        return time.perf_counter()

    @staticmethod
    def _span_ms(a, b):
        if isinstance(a, float):
            return 1e3 * (b - a)
        return float(a.elapsed_time(b))

    def phase_times(self):
        """Mean ms per timed step of each phase {"scatter", "run", "allgather", "step"} (synchronises)."""
        if not self.timing:
            return {}
        if torch.cuda.is_available() and not isinstance(self.timing[0][0], float):
            torch.cuda.synchronize()
        n = len(self.timing)
        tot = {"scatter": 0.0, "run": 0.0, "allgather": 0.0, "step": 0.0}
        for m0, m1, m2, m3 in self.timing:
            tot["scatter"] += self._span_ms(m0, m1)
            tot["run"] += self._span_ms(m1, m2)
            tot["allgather"] += self._span_ms(m2, m3)
            tot["step"] += self._span_ms(m0, m3)
        return {k: v / n for k, v in tot.items()}

    def _local_buffer(self, batch):
        b = batch.shape[0] // self.world
        shape = (b,) + tuple(batch.shape[1:])
        if (self._local is None or tuple(self._local.shape) != shape or self._local.device != batch.device
                or self._local.dtype != batch.dtype):
            self._local = torch.empty(shape, device=batch.device, dtype=batch.dtype)
            self._graph = None
        return self._local

    def _scatter(self, batch):
        """rank 0's batch -> every rank's local buffer (no collective at world 1)."""
        local = self._local_buffer(batch)
        if not dist.is_initialized():            # a process group of one still runs the collectives
            local.copy_(batch)
            return local
        host = _host_staged()
        if not self._dtype_checked:
            # non-zero ranks pass a placeholder: its dtype must be rank 0's or the scatter mismatches
            codes = [torch.float32, torch.float16, torch.bfloat16, torch.float64, torch.uint8]
            assert batch.dtype in codes, f"unsupported batch dtype {batch.dtype}"
            code = torch.tensor([codes.index(batch.dtype)], dtype=torch.int64,
                                device="cpu" if host else batch.device)
            dist.broadcast(code, src=0)
            if codes[int(code.item())] != batch.dtype:
                raise TypeError(f"rank {self.rank}: batch dtype {batch.dtype} != rank 0's {codes[int(code.item())]}")
            self._dtype_checked = True
        chunks = None
        if self.rank == 0:
            chunks = list((batch.cpu() if host else batch).chunk(self.world, 0))
            chunks = [c.contiguous() for c in chunks]
        recv = torch.empty(local.shape, dtype=local.dtype) if host else local
        dist.scatter(recv, scatter_list=chunks, src=0)
        if host:
            local.copy_(recv)
        return local

    def capture(self, batch: torch.Tensor):
        """Capture this rank's forward on its local shard buffer (fixed storage) into a hipGraph;
        later ``step`` calls scatter into that buffer and replay.  The scatter and the gather
        stay outside the graph.  Warm up eagerly first (MIOpen find, weight packing, workspaces)."""
        local = self._local_buffer(batch)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = self.fn(local[:, 0], local[:, 1])
        self._graph = (g, out)

    def _run(self, local):
        if self._graph is None:
            return self.fn(local[:, 0], local[:, 1])      # an eager FoundationStereo guards itself
        self._graph[0].replay()
        if not (local.is_cuda and _fs.RANGE_GUARD and self.recover):
            return self._graph[1]        # the graph NaN-fills its output on overflow (range_poison_)
        # range guard once per replay (one synchronisation): a replay whose flag came back set is
        # recomputed eagerly in safe range mode, and the graph re-captured in that mode
        if not ops.range_overflowed(reset=True):
            return self._graph[1]
        ops.set_range_safe(True)
        ops.RANGE_RECOVERIES[0] += 1
        out = self.fn(local[:, 0], local[:, 1]).clone()
        ops.check_range()
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            gout = self.fn(local[:, 0], local[:, 1])
        self._graph = (g, gout)
        return out

    def step(self, batch: torch.Tensor, out_shape_per_pair: Tuple[int, ...]) -> torch.Tensor:
        B = batch.shape[0]
        if B % self.world:
            raise ValueError(f"batch {B} not divisible by world size {self.world}")
        timed = self.timing is not None
        dev = batch.device
        m0 = self._mark(dev) if timed else None
        local = self._scatter(batch)
        m1 = self._mark(dev) if timed else None
        disp = self._run(local)
        m2 = self._mark(dev) if timed else None
        if not dist.is_initialized():
            out = disp
        elif _host_staged():
            parts = [torch.empty_like(disp, device="cpu") for _ in range(self.world)]
            dist.all_gather(parts, disp.contiguous().cpu())
            out = torch.cat(parts, 0).to(disp.device)
        else:
            out = torch.empty((B,) + tuple(out_shape_per_pair), device=disp.device, dtype=disp.dtype)
            dist.all_gather_into_tensor(out, disp.contiguous())
        if timed:
            self.timing.append((m0, m1, m2, self._mark(dev)))
        return out


def rank_attribution(runner: ShardedStereo, elapsed_s: float, steps: int, device) -> dict:
    """Every rank's own timed-region step time and phase split, gathered to all ranks: the fields a
    multi-GPU line carries so a shortfall from linear scaling can be attributed (a slow rank, the
    scatter, or the all-gather).  Collective over the group; {} without one."""
    if not (dist.is_available() and dist.is_initialized()):
        return {}
    ph = runner.phase_times()
    row = [1e3 * elapsed_s / max(steps, 1), ph.get("scatter", 0.0), ph.get("run", 0.0), ph.get("allgather", 0.0),
           float(dist.get_world_size()), float(dist.get_rank())]
    host = _host_staged()
    mine = torch.tensor(row, dtype=torch.float64, device="cpu" if host else device)
    parts = [torch.empty_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, mine)
    rows = [p.cpu().tolist() for p in parts]
    return {"per_rank_ms": [round(r[0], 4) for r in rows],
            "scatter_ms": [round(r[1], 4) for r in rows],
            "run_ms": [round(r[2], 4) for r in rows],
            "allgather_ms": [round(r[3], 4) for r in rows],
            "rank_world_size": [int(r[4]) for r in rows],
            "ranks": [int(r[5]) for r in rows],
            "timed_by": "HIP events on each rank's stream around its scatter / forward / all-gather"
                        if not host else "host clocks around each rank's scatter / forward / all-gather (gloo)"}
