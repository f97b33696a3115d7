"""Drop-in for ``core/update.py``: the selective ConvGRU refinement block.

Every 1x1 / 3x3 convolution of the loop (motion encoder, SelectiveConvGRU,
DispHead incl. the EdgeNeXt MLPs, mask head) runs on the halo-tiled
split-precision MFMA kernel (``ops.conv2d``, ``fsmi_conv2d_halo_x3``) with
the reference's cats done as zero-copy input segments and bias / ReLU / GELU /
layer-scale / residual / 0.25-scale fused into the epilogue.  Weights are
packed once per (module, weight version).  The gates between the convs --
sigmoid of z/r, ``r*h``, ``cat([r*h, x])``, ``tanh``, ``(1-z)h + zq`` and the
``small*att + large*(1-att)`` selection -- are two fused kernels per
SelectiveConvGRU (``ops.gru_reset``, ``ops.gru_blend``); ``convz`` and
``convr`` run as ONE conv with stacked weights.  The two 7x7 convs run on their
own kernels: ``convd1`` (1 -> 64, + ReLU) on ``ops.conv2d_1in``, the depthwise
``dwconv`` on ``ops.dwconv2d``; ``pool2x`` is ``ops.pool2x`` and ``interp``
``ops.resize_bilinear``.  Under the reference's autocast the same HIP path runs
(fp16 inputs cast up, fp32 compute); with grad enabled the module runs the plain
torch path (``CONV_ENGINE = "miopen"`` forces it, for A/B).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .submodule import HIP_DTYPES, EdgeNextConvEncoder, _f32

import os

CONV_ENGINE = "fsmi"
# A/B knobs (default on): motion path on a side stream; GRU gates in the conv epilogues
OVERLAP = os.environ.get("FSMI_OVERLAP", "1") != "0"
FUSED_GATES = os.environ.get("FSMI_FUSED_GATES", "1") != "0"
# gru16 / gru08 pipelined one iteration ahead (BasicSelectiveMultiUpdateBlock.run_pipelined);
# PIPE_BRANCH: gru04's small branch on its own stream there
PIPELINE = os.environ.get("FSMI_PIPELINE", "1") != "0"
PIPE_BRANCH = os.environ.get("FSMI_PIPE_BRANCH", "1") != "0"
# run_pipelined: the motion path (lookup + encoder) on the main stream -- it is on the iteration's
# critical chain between head(t-1) and gru04(t), both on main, with nothing beside it on main -- instead
# of the motion stream (two cross-stream edges per iteration on that chain); A/B knob
MOTION_ON_MAIN = os.environ.get("FSMI_MOTION_ON_MAIN", "0") != "0"


# SelectiveConvGRU.conv0's context segment convolved once per forward (context_pre); 0: every iteration
CTX_PRE = os.environ.get("FSMI_CTX_PRE", "1") != "0"
# DispHead's last conv (128 -> 1) on its own fp32 kernel (ops.conv3x3_cout1); 0: the halo conv tile
COUT1 = os.environ.get("FSMI_COUT1", "1") != "0"
# the disparity head writes disp + delta into the next encoder buffer (A/B knob)
HEAD_INPLACE = os.environ.get("FSMI_HEAD_INPLACE", "1") != "0"
_CONVD1_MIOPEN = os.environ.get("FSMI_CONVD1_MIOPEN", "0") == "1"
_POOL_TORCH = os.environ.get("FSMI_POOL_TORCH", "0") == "1"        # A/B knob: torch avg_pool2d


def _fast(x) -> bool:
    """The HIP path applies: ROCm tensor, no grad.  Under the reference's autocast
    (scripts/run_demo.py:161) fp16 / bf16 inputs are cast up and the loop still runs on the HIP
    kernels in fp32."""
    return CONV_ENGINE == "fsmi" and x.is_cuda and x.dtype in HIP_DTYPES and not torch.is_grad_enabled()


def _f32s(xs):
    return [_f32(x) for x in xs]


def _packed(*mods, cin_order=None):
    """Halo-kernel weights of one Conv2d/Linear (or several stacked along Cout),
    cached on the first module and rebuilt when any weight/bias changes.  ``cin_order``: input
    channels packed in this order (the caller passes its segments in the same order); a subset of
    the input channels packs the conv restricted to them (one cache entry per order)."""
    key = tuple((id(m), m.weight.data_ptr(), m.weight._version, m.bias.data_ptr(), m.bias._version)
                for m in mods) + (tuple(cin_order) if cin_order is not None else None,)
    if cin_order is None:
        slot, d = "_fsmi_pack", mods[0].__dict__
    else:
        slot, d = tuple(cin_order), mods[0].__dict__.setdefault("_fsmi_pack_perm", {})
    hit = d.get(slot)
    if hit is None or hit[0] != key:
        with torch.no_grad():
            ws = [m.weight if m.weight.dim() == 4 else m.weight[:, :, None, None] for m in mods]
            if cin_order is not None:
                # runs of consecutive channels as slices: no index tensor to upload (a pack first built
                # under a stream capture must not copy from the host)
                runs = []
                for c in cin_order:
                    if runs and c == runs[-1][1]:
                        runs[-1][1] = c + 1
                    else:
                        runs.append([c, c + 1])
                ws = [torch.cat([w[:, a:b] for a, b in runs], 1) for w in ws]
            pk = ops.PackedConv(*ws, mode="halo")
            bias = torch.cat([m.bias.detach().float() for m in mods]).contiguous()
        hit = (key, pk, bias)
        d[slot] = hit
    return hit[1], hit[2]


_SIDE = {}


def _side_stream(device, idx=0):
    """Side stream ``idx`` of ``device`` (0: motion path, 1: GRU small branches / mask head, 3: the
    gru16 / gru08 pipeline of ``run_pipelined``)."""
    s = _SIDE.get((device, idx))
    if s is None:
        # all at default priority: ANY side stream at high priority -- motion (round 4), the branch or
        # the pipeline stream (round 5) -- measured 14.5-14.7 vs 19.0-20.9 pairs/s
        s = _SIDE[(device, idx)] = torch.cuda.Stream(device=device)
    return s


# capture_fork -- the rule every fork / join of a side stream here follows under hipGraph capture:
# a side stream waits only on the capture's origin stream (or on a stream that never waits on it in
# turn); it may be waited on by any stream, and is joined back by the origin.  On this ROCm (HIP 7,
# torch 2.10) a side stream X that waits on side stream A which later waits on X (a fork from a side
# stream plus its join) makes hipStreamEndCapture segfault: tools/capture_fork_probe.py reproduces it
# with plain torch ops (variants a_only, two_parents, enter_main_wait_side segfault; main_only,
# via_main pass).  Hence gru08's small branch on the pipeline stream runs in order, and the motion
# path's disparity branch forks from main, not from the motion stream.
#
#
# Enforced by ``stream_wait`` (every wait between streams here goes through it): while a capture is in
# progress it records the waits between side streams and raises before a wait that would close a cycle
# (X waiting on A after A waited on X, directly or through other side streams) -- every variant the
# probe saw segfault has such a mutual wait, every variant that passed has none.
_CAPTURE_EDGES = {}          # key(waiter) -> set of key(waited), side streams only, current capture


def _skey(s):
    """A stream's identity: its HIP handle (torch.cuda.current_stream() returns a new Python wrapper on
    every call, so id() of the wrapper does not identify the stream); id() for handle-less stand-ins."""
    h = getattr(s, "cuda_stream", None)
    return ("hip", h) if h is not None else ("obj", id(s))


class CaptureForkError(RuntimeError):
    """A stream wait that would make hipStreamEndCapture segfault on this ROCm (capture_fork)."""


def capture_fork_check(waiter, waited, capturing: bool, side_ids=None):
    """Record ``waiter`` waiting on ``waited`` for the capture in progress; raise CaptureForkError when
    ``waited`` already (transitively) waits on ``waiter``.  Only edges between side streams count (the
    capture origin forks and joins every side stream).  ``side_ids``: ``_skey`` of the side streams (default
    the ones ``_side_stream`` made).  Not capturing: forget the edges (a new capture starts clean)."""
    if not capturing:
        _CAPTURE_EDGES.clear()
        return
    side = side_ids if side_ids is not None else {_skey(v) for v in _SIDE.values()}
    a, b = _skey(waiter), _skey(waited)
    if a == b or a not in side or b not in side:
        return
    seen, todo = set(), [b]
    while todo:                                  # does `waited` reach `waiter` through recorded waits?
        x = todo.pop()
        if x == a:
            raise CaptureForkError("capture_fork: a side stream would wait on a side stream that already waits "
                                   "on it inside this hipGraph capture (hipStreamEndCapture segfaults on this "
                                   "ROCm; tools/capture_fork_probe.py) -- fork from the capture origin instead")
        if x not in seen:
            seen.add(x)
            todo.extend(_CAPTURE_EDGES.get(x, ()))
    _CAPTURE_EDGES.setdefault(a, set()).add(b)


# diagnostics (tools/replay_timeline.py): while a list, every wait issued during a capture is logged as
# (waiter stream handle, waited stream handle, number of clocked launches captured so far), which with
# the capture-ordered clock records gives the captured graph's cross-stream edges
WAIT_LOG = None


def stream_wait(waiter, waited):
    """``waiter.wait_stream(waited)`` with the capture_fork check while a capture is in progress."""
    capturing = torch.cuda.is_current_stream_capturing()
    capture_fork_check(waiter, waited, capturing)
    if WAIT_LOG is not None and capturing:
        WAIT_LOG.append((waiter.cuda_stream, waited.cuda_stream, ops.timer_captured_count()))
    waiter.wait_stream(waited)


# side stream the SelectiveConvGRU small branch forks to (1); 0: the branches run in order on the
# caller's stream (run_pipelined: the pipeline stream is itself a side stream, see capture_fork)
_BRANCH = [1]
# run_pipelined: gru08(t+1)'s interp(gru16(t+1)) enqueued right after gru16(t+1), beside gru04(t)
# (FSMI_EARLY_INTERP=0: after gru04(t), as the reference orders it)
EARLY_INTERP = os.environ.get("FSMI_EARLY_INTERP", "1") != "0"
# DispHead's EdgeNeXt MLPs as one fused kernel (ops.edgenext_mlp); FSMI_FUSED_MLP=0: the two 1x1 convs
_FUSED_MLP = os.environ.get("FSMI_FUSED_MLP", "1") != "0"


def _branch_stream(device):
    return _side_stream(device, _BRANCH[0])


def _conv(mods, segs, act=None, **kw):
    mods = mods if isinstance(mods, tuple) else (mods,)
    pk, bias = _packed(*mods)
    return ops.conv2d(segs, pk, bias=bias, act=act, **kw)


__all__ = ["DispHead", "ConvGRU", "BasicMotionEncoder", "pool2x", "pool4x", "interp", "RaftConvGRU",
           "SelectiveConvGRU", "BasicSelectiveMultiUpdateBlock"]


class DispHead(nn.Module):
    """core/update.py:20-32."""

    def __init__(self, input_dim=128, hidden_dim=256, output_dim=1):
        super().__init__()
        self.conv = nn.Sequential(
            nn.Conv2d(input_dim, input_dim, kernel_size=3, padding=1), nn.ReLU(),
            EdgeNextConvEncoder(input_dim, expan_ratio=4, kernel_size=7, norm=None),
            EdgeNextConvEncoder(input_dim, expan_ratio=4, kernel_size=7, norm=None),
            nn.Conv2d(input_dim, output_dim, 3, padding=1))

    def forward(self, x, res=None, out=None, co0=0):
        """``res``: returns res + head(x) from the last conv's epilogue (the loop's ``disp + delta``,
        same fp32 sum), written into channel ``co0`` of ``out`` when given (HIP path only)."""
        if not _fast(x):
            y = self.conv(x)
            return y if res is None else res + y
        y = _conv(self.conv[0], [_f32(x)], "relu")
        for enc in (self.conv[2], self.conv[3]):
            d = ops.dwconv2d(y, enc.dwconv.weight, enc.dwconv.bias)   # depthwise 7x7; norm=None
            if _FUSED_MLP and enc.pwconv1.out_features == 4 * enc.pwconv1.in_features == 512:
                # x + gamma * pw2(gelu(pw1(.))) in one kernel: the 4C GELU map stays in LDS
                pk1, b1 = _packed(enc.pwconv1)
                pk2, b2 = _packed(enc.pwconv2)
                y = ops.edgenext_mlp(d, y, pk1, b1, pk2, b2, gamma=enc.gamma)
            else:
                e = _conv(enc.pwconv1, [d], "gelu")
                y = _conv(enc.pwconv2, [e], gamma=enc.gamma, res=y)  # x + gamma * pw2(gelu(pw1(.)))
        if res is not None:
            res = res.float()
            if not res.is_contiguous():
                res = res.contiguous()
        last = self.conv[4]
        if COUT1 and last.out_channels == 1 and last.kernel_size == (3, 3):
            # one output channel: a per-pixel fp32 dot product, not a 32-row MFMA tile
            return ops.conv3x3_cout1(y, last.weight, last.bias, res=res, out=out, co0=co0)
        return _conv(last, [y], res=res, out=out, co0=co0)


class ConvGRU(nn.Module):
    """core/update.py:34-48 (unused by FoundationStereo; kept for API parity)."""

    def __init__(self, hidden_dim, input_dim, kernel_size=3):
        super().__init__()
        p = kernel_size // 2
        self.convz = nn.Conv2d(hidden_dim + input_dim, hidden_dim, kernel_size, padding=p)
        self.convr = nn.Conv2d(hidden_dim + input_dim, hidden_dim, kernel_size, padding=p)
        self.convq = nn.Conv2d(hidden_dim + input_dim, hidden_dim, kernel_size, padding=p)

    def forward(self, h, cz, cr, cq, *x_list):
        x = torch.cat(x_list, dim=1)
        hx = torch.cat([h, x], dim=1)
        z = torch.sigmoid(self.convz(hx) + cz)
        r = torch.sigmoid(self.convr(hx) + cr)
        q = torch.tanh(self.convq(torch.cat([r * h, x], dim=1)) + cq)
        return (1 - z) * h + z * q


class BasicMotionEncoder(nn.Module):
    """core/update.py:51-70."""

    def __init__(self, args, ngroup=8):
        super().__init__()
        self.args = args
        cor_planes = args.corr_levels * (2 * args.corr_radius + 1) * (ngroup + 1)
        self.convc1 = nn.Conv2d(cor_planes, 256, 1, padding=0)
        self.convc2 = nn.Conv2d(256, 256, 3, padding=1)
        self.convd1 = nn.Conv2d(1, 64, 7, padding=3)
        self.convd2 = nn.Conv2d(64, 64, 3, padding=1)
        self.conv = nn.Conv2d(64 + 256, 128 - 1, 3, padding=1)

    def encode_into(self, disp, corr, out):
        """Writes cat([relu(conv(...)), disp]) into ``out`` (B, 128, H, W) without the cat copy."""
        return self._encode_rest(disp, _conv(self.convc1, [corr], "relu"), out)

    def motion_into(self, disp, geo_fn, out):
        """The motion path of one iteration: the lookup ``geo_fn(disp)`` and this encoder."""
        return self.encode_into(disp, geo_fn(disp), out)

    def _disp_feat(self, disp, out=None):
        if _CONVD1_MIOPEN:                                     # A/B knob: the MIOpen conv + ReLU
            d = F.relu_(self.convd1(disp))
        else:
            d = ops.conv2d_1in(disp, self.convd1.weight, self.convd1.bias, relu=True)   # 7x7, 1 -> 64
        return _conv(self.convd2, [d], "relu", out=out)

    def _encode_rest(self, disp, c1, out):
        c = _conv(self.convc2, [c1], "relu")
        d = self._disp_feat(disp)
        # cat([cor, dsp]) with the disparity features (~disp magnitude: ~200 at cfg5) as the FIRST
        # segment: the halo conv fixes a block's exponent from its first chunk (conv_halo.h)
        nc, nd = c.shape[1], d.shape[1]
        pk, b = _packed(self.conv, cin_order=tuple(range(nc, nc + nd)) + tuple(range(nc)))
        ops.conv2d([d, c], pk, bias=b, act="relu", out=out, co0=0)
        tail = out[:, self.conv.out_channels:]
        if tail.data_ptr() != disp.data_ptr():        # run_pipelined has the head write it in place
            tail.copy_(disp)
        return out

    def forward(self, disp, corr):
        if _fast(corr):
            corr, disp = _f32(corr), _f32(disp)
            B, _, H, W = corr.shape
            return self.encode_into(disp, corr, corr.new_empty(B, self.conv.out_channels + 1, H, W))
        cor = F.relu(self.convc2(F.relu(self.convc1(corr))))
        dsp = F.relu(self.convd2(F.relu(self.convd1(disp))))
        out = F.relu(self.conv(torch.cat([cor, dsp], dim=1)))
        return torch.cat([out, disp], dim=1)


def pool2x(x):
    if _fast(x) and not _POOL_TORCH:
        return ops.pool2x(_f32(x))
    return F.avg_pool2d(x, 3, stride=2, padding=1)


def pool4x(x):
    return F.avg_pool2d(x, 5, stride=4, padding=1)


def interp(x, dest):
    if _fast(x):
        return ops.resize_bilinear(_f32(x), dest.shape[2:])
    return F.interpolate(x, dest.shape[2:], mode="bilinear", align_corners=True)


def _stacked_zr(gru, cache):
    """[convz; convr] weights stacked along out-channels (cached per weight version)."""
    wz, wr, bz, br = gru.convz.weight, gru.convr.weight, gru.convz.bias, gru.convr.bias
    key = tuple((t.data_ptr(), t._version) for t in (wz, wr, bz, br))
    hit = cache.get(id(gru))
    if hit is None or hit[0] != key:
        with torch.no_grad():
            hit = (key, torch.cat([wz, wr], 0).contiguous(), torch.cat([bz, br], 0).contiguous())
        cache[id(gru)] = hit
    return hit[1], hit[2]


class RaftConvGRU(nn.Module):
    """core/update.py:83-95."""

    def __init__(self, hidden_dim=128, input_dim=256, kernel_size=3):
        super().__init__()
        p = kernel_size // 2
        self.convz = nn.Conv2d(hidden_dim + input_dim, hidden_dim, kernel_size, padding=p)
        self.convr = nn.Conv2d(hidden_dim + input_dim, hidden_dim, kernel_size, padding=p)
        self.convq = nn.Conv2d(hidden_dim + input_dim, hidden_dim, kernel_size, padding=p)
        self._zr_cache = {}

    def zr(self, hx):
        w, b = _stacked_zr(self, self._zr_cache)
        return F.conv2d(hx, w, b, padding=self.convz.padding)

    def zr_fast(self, hx):
        return _conv((self.convz, self.convr), [hx])

    def forward(self, h, x, hx):
        fast = _fast(hx)
        if fast:
            h, x, hx = _f32(h), _f32(x), _f32(hx)
        zr = self.zr_fast(hx) if fast else self.zr(hx).float()
        qin, _ = ops.gru_reset(zr, zr, h.float(), x.float())
        q = _conv(self.convq, [qin]) if fast else self.convq(qin).float()
        ones = torch.ones_like(h[:, :1])
        return ops.gru_blend(zr, zr, q, q, h, ones)


class SelectiveConvGRU(nn.Module):
    """core/update.py:98-119 with fused gate kernels."""

    def __init__(self, hidden_dim=128, input_dim=256, small_kernel_size=1, large_kernel_size=3, patch_size=None):
        super().__init__()
        self.conv0 = nn.Sequential(nn.Conv2d(input_dim, input_dim, kernel_size=3, padding=1), nn.ReLU())
        self.conv1 = nn.Sequential(nn.Conv2d(input_dim + hidden_dim, input_dim + hidden_dim, kernel_size=3,
                                             padding=1), nn.ReLU())
        self.small_gru = RaftConvGRU(hidden_dim, input_dim, small_kernel_size)
        self.large_gru = RaftConvGRU(hidden_dim, input_dim, large_kernel_size)

    def context_pre(self, inp):
        """conv0's contribution of the context segment plus its bias, ``W0[:, :Ci] * inp + b0``.

        ``x[0]`` of every call is the level's context feature ``inp[i]``, fixed for the whole
        refinement loop (core/foundation_stereo.py:222-226 build it once; core/update.py:142-151 pass
        it each iteration), and conv0 is linear in its input channels: this part is computed once
        per forward and passed back as ``forward(..., pre=)``, which convolves only the remaining
        channels and adds it before the ReLU (act 7) -- 1/3 (gru04 / gru08) and 1/2 (gru16) of
        conv0's MACs per iteration.  HIP path only."""
        inp = _f32(inp)
        pk, b = _packed(self.conv0[0], cin_order=tuple(range(inp.shape[1])))
        return ops.conv2d([inp], pk, bias=b)

    def _conv0_rest(self, segs, pre):
        """ReLU(W0[:, segs] * cat(segs) + pre), ``segs`` the (tensor, conv0 input channel offset) pairs
        ``pre`` does not cover (see ``context_pre``).  The first segment's LAST 32 channels go first:
        the motion features (gru04) carry the disparity (~1e2 px) as their last channel, and the kernel
        fixes a tile's block exponent from its first 32-channel chunk (range mode 2, conv_halo.h
        chunk_exp), as the motion encoder orders its own cat."""
        t0, c0 = segs[0]
        c1 = t0.shape[1]
        if c1 > 32 and (c1 - 32) % 8 == 0:
            ss = [(t0, c1 - 32, 32), (t0, 0, c1 - 32)]
            order = list(range(c0 + c1 - 32, c0 + c1)) + list(range(c0, c0 + c1 - 32))
        else:
            ss, order = [t0], list(range(c0, c0 + c1))
        for t, c in segs[1:]:
            ss.append(t)
            order += list(range(c, c + t.shape[1]))
        pk, _ = _packed(self.conv0[0], cin_order=tuple(order))
        return ops.conv2d(ss, pk, act="relu_pre", res=pre)

    def forward(self, att, h, *x, pre=None):
        """``pre``: ``context_pre(x[0])`` of this forward's context feature (HIP path; x[0] is then not read;
        the torch path ignores it, its conv0 takes the whole cat)."""
        if _fast(h):
            h = _f32(h)
            if pre is not None:
                segs, c = [], x[0].shape[1]
                for t in x[1:]:
                    segs.append((_f32(t), c))
                    c += t.shape[1]
                xc = self._conv0_rest(segs, pre)
            else:
                xc = _conv(self.conv0[0], _f32s(x), "relu")          # cat(x) as input segments
            hx = _conv(self.conv1[0], [xc, h], "relu")
            # gates in the conv epilogues: z / r*h from the stacked zr convs, then each convq reads
            # [r*h, x] as two segments and blends straight into the new state
            if not FUSED_GATES:
                zr_s = self.small_gru.zr_fast(hx)
                zr_l = self.large_gru.zr_fast(hx)
                qs_in, ql_in = ops.gru_reset(zr_s, zr_l, h, xc)
                q_s = _conv(self.small_gru.convq, [qs_in])
                q_l = _conv(self.large_gru.convq, [ql_in])
                return ops.gru_blend(zr_s, zr_l, q_s, q_l, h, att.float())
            att = att.float().contiguous()
            out = torch.empty_like(h)

            def branch(gru, mode):
                z, rh = torch.empty_like(h), torch.empty_like(h)
                pk, b = _packed(gru.convz, gru.convr)
                ops.conv2d_gate([hx], pk, b, "zr", h=h, z=z, rh=rh)
                pk, b = _packed(gru.convq)
                return pk, b, z, rh

            sg = self.small_gru

            def small():                                 # out = small branch * att
                pk, b, z, rh = branch(sg, "blend_small")
                ops.conv2d_gate([rh, xc], pk, b, "blend_small", h=h, z=z, att=att, out=out)

            if OVERLAP and _BRANCH[0]:
                # small (1x1) branch on a side stream beside the large branch's zr conv; the
                # large blend adds into ``out`` after the small blend has written it
                main = torch.cuda.current_stream(h.device)
                side = _branch_stream(h.device)
                stream_wait(side, main)
                with torch.cuda.stream(side):
                    small()
                pk, b, z, rh = branch(self.large_gru, "blend_large")
                stream_wait(main, side)
                ops.conv2d_gate([rh, xc], pk, b, "blend_large", h=h, z=z, att=att, out=out)
                return out
            small()
            pk, b, z, rh = branch(self.large_gru, "blend_large")
            ops.conv2d_gate([rh, xc], pk, b, "blend_large", h=h, z=z, att=att, out=out)
            return out
        x = torch.cat(x, dim=1) if len(x) > 1 else x[0]
        x = self.conv0(x)
        hx = self.conv1(torch.cat([x, h], dim=1))
        # .float(): no-ops in fp32; under the reference's fp16 autocast the gates stay fp32
        zr_s = self.small_gru.zr(hx).float()
        zr_l = self.large_gru.zr(hx).float()
        h = h.float()
        qs_in, ql_in = ops.gru_reset(zr_s, zr_l, h, x.float())
        q_s = self.small_gru.convq(qs_in).float()
        q_l = self.large_gru.convq(ql_in).float()
        return ops.gru_blend(zr_s, zr_l, q_s, q_l, h, att.float())


class BasicSelectiveMultiUpdateBlock(nn.Module):
    """core/update.py:122-159."""

    def __init__(self, args, hidden_dim=128, volume_dim=8):
        super().__init__()
        self.args = args
        self.encoder = BasicMotionEncoder(args, volume_dim)
        n = args.n_gru_layers
        if n == 3:
            self.gru16 = SelectiveConvGRU(hidden_dim, hidden_dim * 2)
        if n >= 2:
            self.gru08 = SelectiveConvGRU(hidden_dim, hidden_dim * (n == 3) + hidden_dim * 2)
        self.gru04 = SelectiveConvGRU(hidden_dim, hidden_dim * (n > 1) + hidden_dim * 2)
        self.disp_head = DispHead(hidden_dim, 256)
        self.mask = nn.Sequential(nn.Conv2d(128, 64, 3, padding=1), nn.ReLU(inplace=True),
                                  nn.Conv2d(64, 32, 3, padding=1), nn.ReLU(inplace=True))

    def forward(self, net, inp, corr, disp, att):
        if _fast(corr):
            return self._forward_fast(_f32s(net), _f32s(inp), _f32(corr), _f32(disp), _f32s(att))
        n = self.args.n_gru_layers
        if n == 3:
            net[2] = self.gru16(att[2], net[2], inp[2], pool2x(net[1]))
        if n >= 2:
            if n > 2:
                net[1] = self.gru08(att[1], net[1], inp[1], pool2x(net[0]), interp(net[2], net[1]))
            else:
                net[1] = self.gru08(att[1], net[1], inp[1], pool2x(net[0]))
        motion = torch.cat([inp[0], self.encoder(disp, corr)], dim=1)
        if n > 1:
            net[0] = self.gru04(att[0], net[0], motion, interp(net[1], net[0]))
        delta_disp = self.disp_head(net[0])
        mask = .25 * self.mask(net[0])
        return net, mask, delta_disp

    def context_pre(self, inp):
        """Per GRU level (gru04, gru08, gru16 as ``inp``), ``SelectiveConvGRU.context_pre`` of its context
        feature: the loop-invariant part of conv0, computed once per forward (HIP path; None otherwise or
        with FSMI_CTX_PRE=0)."""
        if not CTX_PRE or not inp or not _fast(inp[0]):
            return None
        grus = [self.gru04, getattr(self, "gru08", None), getattr(self, "gru16", None)]
        return [g.context_pre(x) for g, x in zip(grus, inp) if g is not None]

    def forward_overlapped(self, net, inp, geo_fn, disp, att, pre=None):
        """``forward(net, inp, geo_fn(disp), disp, att)`` with the motion path -- the lookup and
        the motion encoder, which depend only on ``disp`` -- on a side stream, concurrently with
        gru16 / gru08 (small 1/16 and 1/8 maps that leave most CUs idle).  Joined before gru04.
        Cross-stream buffers (``enc``) are allocated on the calling stream and ``disp`` is only
        released by the caller after the join, so the caching allocator never recycles memory a
        pending side-stream kernel still reads.  Captures into a hipGraph as a fork/join."""
        main = torch.cuda.current_stream(disp.device)
        side = _side_stream(disp.device)
        B, _, H, W = disp.shape
        enc = disp.new_empty(B, self.encoder.conv.out_channels + 1, H, W)
        stream_wait(side, main)
        with torch.cuda.stream(side):
            self.encoder.motion_into(disp, geo_fn, enc)
        n = self.args.n_gru_layers
        p0, p1, p2 = (list(pre) + [None] * 3)[:3] if pre is not None else (None, None, None)
        if n == 3:
            net[2] = self.gru16(att[2], net[2], inp[2], pool2x(net[1]), pre=p2)
        if n >= 2:
            if n > 2:
                net[1] = self.gru08(att[1], net[1], inp[1], pool2x(net[0]), interp(net[2], net[1]), pre=p1)
            else:
                net[1] = self.gru08(att[1], net[1], inp[1], pool2x(net[0]), pre=p1)
        stream_wait(main, side)
        if n > 1:
            net[0] = self.gru04(att[0], net[0], inp[0], enc, interp(net[1], net[0]), pre=p0)
        # mask head beside the disparity head (both read net[0] only)
        side1 = _side_stream(disp.device, 1)
        stream_wait(side1, main)
        with torch.cuda.stream(side1):
            mask = _conv(self.mask[2], [_conv(self.mask[0], [net[0]], "relu")], "relu", alpha=0.25)
        delta_disp = self.disp_head(net[0])
        stream_wait(main, side1)
        return net, mask, delta_disp

    def run_pipelined(self, net, inp, geo_fn, disp, att, iters, pre=None):
        """``iters`` refinement iterations (``disp += forward(net, inp, geo_fn(disp), disp, att)[2]``
        each) with gru16 / gru08 running one iteration ahead on a stream of their own.

        gru16(t+1) needs only net[1](t) and net[2](t), so it runs beside gru04(t) and the heads;
        gru08(t+1) needs net[0](t), so it starts as soon as gru04(t) is done, beside the disparity
        head and the motion path of t+1 (lookup + encoder, on the motion stream, which need only
        disp(t+1)).  The critical path per iteration is gru04 + max(head + motion, gru08) instead of
        gru16 + gru08 + gru04 + head.  Every value is computed by the same kernels from the same
        inputs as ``forward`` (bit-identical); only the order of independent work changes.
        One pipeline stream and whole-stream joins: ``stream_wait(main, s_gru)`` is issued after
        gru08(t) and before gru16(t+1) is enqueued, so gru04(t) waits for the former only.  The
        mask head shares the motion stream.  A tensor read on another stream is freed only after
        the freeing stream has joined the reader, so the caching allocator never recycles memory
        a pending kernel still reads.  Returns (net, mask, disp); the mask head runs in the last
        iteration only (test mode discards the others).  ``pre``: ``context_pre(inp)`` (loop-invariant
        conv0 parts per level) or None."""
        dev = disp.device
        main = torch.cuda.current_stream(dev)
        s_mot, s_gru = _side_stream(dev, 0), _side_stream(dev, 3)
        n0, n1, n2 = net
        p0, p1, p2 = pre if pre is not None else (None, None, None)
        B, _, H, W = disp.shape
        main_branch = PIPE_BRANCH                        # gru04's small branch on stream 1 (4th stream)
        nc = self.encoder.conv.out_channels
        stream_wait(s_gru, main)
        _BRANCH[0] = 0                                   # pipeline-stream GRUs: branches in order
        with torch.cuda.stream(s_gru):
            n2 = self.gru16(att[2], n2, inp[2], pool2x(n1), pre=p2)
            n1 = self.gru08(att[1], n1, inp[1], pool2x(n0), interp(n2, n1), pre=p1)
        _BRANCH[0] = 1
        mask = None
        # the disparity lives in the last channel of the encoder output it feeds: the disparity head
        # writes disp + delta straight into the next iteration's buffer (no cat copy, no add pass)
        enc = disp.new_empty(B, nc + 1, H, W)                                   # on main
        if HEAD_INPLACE:
            enc[:, nc:].copy_(disp)
            disp = enc[:, nc:]
        for t in range(iters):
            if not HEAD_INPLACE and t:
                enc = disp.new_empty(B, nc + 1, H, W)
            if MOTION_ON_MAIN:
                self.encoder.motion_into(disp, geo_fn, enc)
            else:
                stream_wait(s_mot, main)
                with torch.cuda.stream(s_mot):
                    self.encoder.motion_into(disp, geo_fn, enc)
            stream_wait(main, s_gru)                      # gru08(t): enqueued last on s_gru so far
            if not MOTION_ON_MAIN:
                stream_wait(main, s_mot)                  # motion(t)
            if t + 1 < iters:
                _BRANCH[0] = 0
                with torch.cuda.stream(s_gru):           # gru16(t+1), beside gru04(t)
                    n2 = self.gru16(att[2], n2, inp[2], pool2x(n1), pre=p2)
                    # gru08(t+1)'s upsampled gru16 input, also beside gru04(t): one kernel less between
                    # gru04(t) and gru08(t+1)
                    up2 = interp(n2, n1) if EARLY_INTERP else None
                _BRANCH[0] = 1
            _BRANCH[0] = 1 if main_branch else 0
            n0 = self.gru04(att[0], n0, inp[0], enc, interp(n1, n0), pre=p0)
            _BRANCH[0] = 1
            if t + 1 < iters:
                stream_wait(s_gru, main)                  # gru04(t)
                # gru08's branches in order on the pipeline stream: a fork from it would be a side
                # stream waiting on the pipeline stream and waited on by it (capture_fork)
                _BRANCH[0] = 0
                with torch.cuda.stream(s_gru):           # gru08(t+1), beside the heads + motion(t+1)
                    n1 = self.gru08(att[1], n1, inp[1], pool2x(n0), up2 if EARLY_INTERP else interp(n2, n1), pre=p1)
                _BRANCH[0] = 1
            if t + 1 == iters:
                # test mode upsamples only the last iteration's disparity: the reference computes the
                # mask head every iteration and discards all but the last (core/foundation_stereo.py:243-244)
                stream_wait(s_mot, main)
                with torch.cuda.stream(s_mot):
                    mask = _conv(self.mask[2], [_conv(self.mask[0], [n0], "relu")], "relu", alpha=0.25)
            if t + 1 < iters and HEAD_INPLACE:
                enc = disp.new_empty(B, nc + 1, H, W)
                self.disp_head(n0, res=disp, out=enc, co0=nc)
                disp = enc[:, nc:]
            elif HEAD_INPLACE:
                disp = self.disp_head(n0, res=disp)
            else:
                disp = disp + self.disp_head(n0).float()
            if not MOTION_ON_MAIN or t + 1 == iters:
                stream_wait(main, s_mot)
        stream_wait(main, s_gru)
        return [n0, n1, n2], mask, disp

    def _forward_fast(self, net, inp, corr, disp, att):
        n = self.args.n_gru_layers
        if n == 3:
            net[2] = self.gru16(att[2], net[2], inp[2], pool2x(net[1]))
        if n >= 2:
            if n > 2:
                net[1] = self.gru08(att[1], net[1], inp[1], pool2x(net[0]), interp(net[2], net[1]))
            else:
                net[1] = self.gru08(att[1], net[1], inp[1], pool2x(net[0]))
        B, _, H, W = corr.shape
        enc = self.encoder.encode_into(disp, corr, corr.new_empty(B, self.encoder.conv.out_channels + 1, H, W))
        # motion = cat([inp[0], enc]) stays two segments of gru04.conv0's input
        if n > 1:
            net[0] = self.gru04(att[0], net[0], inp[0], enc, interp(net[1], net[0]))
        delta_disp = self.disp_head(net[0])
        mask = _conv(self.mask[2], [_conv(self.mask[0], [net[0]], "relu")], "relu", alpha=0.25)
        return net, mask, delta_disp
