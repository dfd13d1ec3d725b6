"""Point-sharded multi-GPU GASFM: one process per GPU, RCCL (torch.distributed "nccl") over xGMI.

The reference runs one scene on one device (main.py:77-78); this module splits a
scene's 3D points into contiguous ranges balanced by edge count:

  local       every edge of a rank's points, the point-direction attention, all
              point MLPs, the per-edge block body (LN, projection update,
              residual), the point head.
  replicated  camera (view) and global node computations and the view head:
              identical on every rank, from identical inputs.
  exchange    the camera-direction attention and the points->global attention
              produce per-rank partial softmax states (max, sum, acc) for their
              destinations; ONE all-gather of the packed partial rows
              (m x (HC + 2H) floats) per half-layer, then every rank merges
              the W partials in rank order with gasfm_gat_attn_combine, so all
              ranks hold bitwise-identical camera / global aggregates.
Backward: a replicated tensor consumed by local computation (camera XR, Sv, Sg,
global XR) receives a partial gradient from each rank -> ``AllReduceGrad`` sums
it (one all-reduce, m x 32 floats) before the replicated backward continues, so
replicated parameters get identical full gradients without any collective.
Parameters used by local computation get partial gradients, summed by one
bucketed all-reduce in ``sync_grads`` (~1.3 MB for 12 blocks).  No DDP
all-reduce of the 145 M replicated parameters.

Loss convention: each rank's loss must contain the replicated outputs'
(Ps_norm) term in full and its own points' (pts3D[:, point_slice]) term.
``gasfm_amd.ESFMLoss`` on a sharded scene follows it: every rank computes the
global loss (one 2-float all-reduce) and its Ps gradient is all-reduced.

Camera sharding (``shard_scene(..., cameras=True)``, the default of bench.py at N > 1):
the m x 1024 view chain (Proj2View tail + MLP, the view hub, view->global lin_l,
the final update's view tail and the view head) is split too: rank r owns the
camera rows [r*ceil(m/W), ...) and runs the 1024 x 1024 GEMMs and view kernels on
them only.  Per block, forward: the camera aggregate (replicated after the
all-gather combine) is sliced to the own rows (``OwnRowsFn``; backward: one
all-gather of the own-row gradients); the view hub's 32-wide outputs that every
rank's edges read (the projection-update term SV and the next block's camera
target rows XR) are all-gathered in ONE collective (``GatherRowsFn``); the
view->global and points->global attentions exchange their partial softmax states
in ONE all-gather (``ShardedGlobalAttentionFn``).  Backward: the (SV, SG, next
XR) gradients are all-reduced in one collective (``AllReduceGradN``), the two
global target rows in one more.  The view-side parameters then hold partial
gradients like the point-side ones: ``sync_grads`` all-reduces every parameter
except the replicated global chain's (``REPLICATED_CAM_PATTERNS``).
"""
import copy
import fnmatch

import numpy as np
import torch
import torch.distributed as dist

from . import _native
from .attention import (AttnPlan, attn_backward_raw, attn_forward_partial, camera_max_piece, combine_partials,
                        gatt_dxl, gatt_ok, gatt_prob)
from .scene import MIN_N_POINTS_PER_VIEW, MIN_N_VIEWS_PER_POINT, SceneData, build_graph_wrappers

# parameters whose gradient comes from rank-local computation (edges / points); everything
# else is computed identically on all ranks from all-reduced boundary gradients
LOCAL_PARAM_PATTERNS = (
    "embed.*",
    "equivariant_blocks.*.prev_projfeat_norm_layer.*",
    "*proj2scenepoint.*",
    "*proj2view.graph_conv.lin_l.*",
    "*proj2view.graph_conv.att",
    "*graph_conv_scenepoint2global.lin_l.*",
    "*graph_conv_scenepoint2global.att",
    "*projection_feature_update.lin_proj.*",
    "*projection_feature_update.scenepoint_norm_layer.*",
    "*projection_feature_update.lin_scenepoint.*",
    "*residual_skipconn_proj_norm_layer.*",
    "*skip_projection.*",
    "scenepoint_head.*",
    "depth_head.*",
)


# camera sharding: the only parameters whose gradients are computed identically on every rank
# (the global node's chain, from replicated inputs and all-reduced boundary gradients, and the
# attention biases, whose gradients are sums of replicated output gradients)
REPLICATED_CAM_PATTERNS = (
    "*view_and_scenepoint2global.norm_and_proj_global2view.*",
    "*view_and_scenepoint2global.norm_and_proj_global2scenepoint.*",
    "*view_and_scenepoint2global.graph_conv_view2global.lin_r.*",
    "*view_and_scenepoint2global.graph_conv_scenepoint2global.lin_r.*",
    "*view_and_scenepoint2global.graph_conv_view2global.bias",
    "*view_and_scenepoint2global.graph_conv_scenepoint2global.bias",
    "*view_and_scenepoint2global.proj_view_and_scenepoint2global.*",
    "*view_and_scenepoint2global.norm_pre_mlp.*",
    "*view_and_scenepoint2global.mlp.*",
    "*projection_feature_update.global_norm_layer.*",
    "*projection_feature_update.lin_global.*",
    "*proj2view.graph_conv.bias",
    # block 0 is stateless: its camera target rows are lin_r(0), the same replicated row everywhere
    "equivariant_blocks.0.global_feature_update.proj2view.graph_conv.lin_r.*",
)


def is_local_param(name, cameras=False):
    """True when the parameter's gradient is partial per rank (summed by ``sync_grads``)."""
    if cameras:
        return not any(fnmatch.fnmatchcase(name, p) for p in REPLICATED_CAM_PATTERNS)
    return any(fnmatch.fnmatchcase(name, p) for p in LOCAL_PARAM_PATTERNS)


class AsyncGradReducer:
    """Overlaps the camera-sharded path's large weight-gradient all-reduces with the rest of the
    backward: a post-accumulate-grad hook on each 1024 x 1024 view-side weight (Proj2View's MLP,
    graph_conv_view2global.lin_l, the view head: 113 of the 120 MB of partial gradients at the
    learning conf) hands its fresh .grad over as soon as autograd has set it; it is all-reduced
    in place, asynchronously on RCCL's stream, while the backward of the blocks below runs.
    ``sync_grads`` waits for them and leaves them out of its bucket.  Armed only when every .grad
    was unset at forward time (each hooked .grad is then that pass's gradient alone)."""

    def __init__(self, shard):
        self.shard = shard
        self.works = []
        self.ptrs = set()
        # the forward's capture state: the hooks run on autograd's device thread, under the stream
        # autograd guards for the AccumulateGrad node.  A hook that saw no capture while the
        # forward was captured would issue its all-reduce outside the graph (eagerly, once, on
        # gradients not yet computed) and put its Work on the watchdog's list mid-capture.
        self.capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()

    def launch(self, t):
        if t.data_ptr() in self.ptrs:  # a second accumulation into a tensor already in flight
            raise RuntimeError("camera-sharded backward: a parameter's gradient was accumulated twice in one pass "
                               "(several forwards before one backward); run forward/backward/sync_grads per step")
        if t.is_cuda and torch.cuda.is_current_stream_capturing() != self.capturing:
            raise RuntimeError("camera-sharded backward: a gradient hook ran on a stream whose capture state differs "
                               "from the forward's; its all-reduce would not be part of the captured step")
        sh = self.shard
        if sh.emulate:
            self.ptrs.add(t.data_ptr())
            return
        if sh._staged(t):  # gloo: synchronous host staging
            sh.all_reduce_(t)
        else:
            self.works.append(dist.all_reduce(t, group=sh.group, async_op=True))
        self.ptrs.add(t.data_ptr())

    def wait(self):
        for w in self.works:
            w.wait()
        self.works.clear()


def camera_rows(m, world, rank):
    """Contiguous equal camera chunks: (c0, c1, chunk) of rank ``rank``; the last chunk may be short."""
    chunk = -(-m // world)
    c0 = min(m, rank * chunk)
    return c0, min(m, c0 + chunk), chunk


class ShardContext:
    """rank / world / process group of a sharded scene.

    cams: (c0, c1, chunk, m) when the camera rows are sharded too (None: replicated views).
    emulate: no process group -- all_gather returns ``world`` copies of this rank's tensor and
    all_reduce_ is the identity.  Runs one rank's share of an N-GPU step on one GPU with the real
    kernels and tensor shapes (the per-rank proxy of bench.py --emulate-world); numerically
    meaningless."""

    def __init__(self, rank, world, group=None, cams=None, emulate=False):
        self.rank, self.world, self.group = rank, world, group
        self.cams = cams
        self.emulate = bool(emulate)
        self._combine_cache = {}

    def pack_items(self, specs, device):
        """Combine items (seg 0, slot_begin, count, stride) for rows inside gathered send blocks."""
        key = (tuple(specs), str(device))
        if key not in self._combine_cache:
            self._combine_cache[key] = [torch.tensor([[0, b, c, s]], dtype=torch.int32).to(device)
                                        for b, c, s in specs]
        return self._combine_cache[key]

    def combine_items(self, N, device):
        key = (N, str(device))
        if key not in self._combine_cache:
            s = torch.arange(N, dtype=torch.int32)
            items = torch.stack([s, s, torch.full_like(s, self.world), torch.full_like(s, N)], 1)
            self._combine_cache[key] = items.contiguous().to(device)
        return self._combine_cache[key]

    # collectives: RCCL for GPU tensors on the nccl backend; gloo stages through the host
    def _staged(self, t):
        return dist.get_backend(self.group) == "gloo" and t.is_cuda

    def all_gather(self, t):
        t = t.contiguous()
        if self.emulate:  # one copy kernel of the gathered size (stands in for the RCCL kernel)
            out = torch.empty((self.world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            out.view((self.world,) + tuple(t.shape)).copy_(t.unsqueeze(0).expand((self.world,) + tuple(t.shape)))
            return out
        if self._staged(t):
            parts = [torch.empty_like(t, device="cpu") for _ in range(self.world)]
            dist.all_gather(parts, t.cpu(), group=self.group)
            return torch.cat(parts, 0).to(t.device)
        out = torch.empty((self.world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t, group=self.group)
        return out

    def all_reduce_(self, t):
        if self.emulate:
            return t
        if self._staged(t):
            c = t.cpu()
            dist.all_reduce(c, group=self.group)
            t.copy_(c)
        else:
            dist.all_reduce(t, group=self.group)
        return t


class AllReduceGrad(torch.autograd.Function):
    """Identity forward; sums the gradient over ranks (replicated -> local boundary)."""

    @staticmethod
    def forward(ctx, x, shard):
        ctx.shard = shard
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return ctx.shard.all_reduce_(g.contiguous().clone()), None


class AllReduceGradN(torch.autograd.Function):
    """Identity forward on several tensors; their gradients are summed over ranks with ONE
    all-reduce of the concatenation (the view and global terms of the projection update reach
    the edge backward together)."""

    @staticmethod
    def forward(ctx, shard, *xs):
        ctx.shard = shard
        ctx.shapes = [x.shape for x in xs]
        ctx.devdtype = (xs[0].device, xs[0].dtype)
        return tuple(x.view_as(x) for x in xs)

    @staticmethod
    def backward(ctx, *gs):
        dev, dt = ctx.devdtype
        flat = _adjacent_flat(gs, ctx.shapes)
        if flat is None:
            flat = torch.cat([(g if g is not None else torch.zeros(sh, device=dev, dtype=dt)).reshape(-1)
                              for g, sh in zip(gs, ctx.shapes)])
        ctx.shard.all_reduce_(flat)
        out, at = [], 0
        for sh in ctx.shapes:
            k = int(torch.Size(sh).numel())
            out.append(flat[at:at + k].view(sh))
            at += k
        return (None,) + tuple(out)


def _adjacent_flat(gs, shapes):
    """The one flat buffer the gradients gs already are consecutive contiguous views of, in order
    (the edge backward writes the boundary's dSv | dSg | dXR that way: edge_block._boundary_buffers),
    else None (then they are concatenated)."""
    if any(g is None or not g.is_contiguous() or g.shape != sh for g, sh in zip(gs, shapes)):
        return None
    at = gs[0].data_ptr()
    for g in gs:
        if g.data_ptr() != at or g.untyped_storage().data_ptr() != gs[0].untyped_storage().data_ptr():
            return None
        at += g.numel() * g.element_size()
    total = sum(g.numel() for g in gs)
    base = gs[0]
    return base.as_strided((total,), (1,), base.storage_offset())


def _pad_rows(x, rows):
    if x.shape[0] == rows:
        return x.contiguous()
    return torch.cat([x, x.new_zeros((rows - x.shape[0],) + tuple(x.shape[1:]))])


def _c4(n):
    return -(-n // 4) * 4


class BlockExchange:
    """A camera-sharded block's collectives, two per block instead of four (round 5):

    forward   ONE all-gather of [own SV | XR rows (chunk x 64) | view->global partial row |
              points->global partial row] per rank (view hub -> send block <- global convs'
              partial rows), then ONE launch merges the global partials and unpacks every rank's
              rows (gasfm_gatt_merge_unpack): ShardedGlobalExchangeFn.
    backward  ONE all-gather of [own camera-aggregate gradient rows (chunk x 32) | this rank's
              partial gradient of the two global target rows] (OwnRowsFn), then ONE launch unpacks
              the rows and sums the W partial target-row gradients in rank order into ``red``
              (gasfm_exchange_unpack).  The global convs' backward (which runs first) writes its
              partial into the send block and hands ``red`` to autograd before it is filled: its
              consumer, the previous block's GlobalChainFn, runs only after this block's camera
              attention backward (which needs OwnRowsFn's output), see ShardedGlobalExchangeFn."""

    def __init__(self, shard, HCv, HCp, heads, dev):
        c0, c1, chunk, m = shard.cams
        self.shard, self.chunk, self.m, self.own = shard, chunk, m, c1 - c0
        self.HCv, self.HCp, self.dev = HCv, HCp, dev
        self.Lv, self.Lp = HCv + 2 * heads, HCp + 2 * heads
        self.f_ov = chunk * 64
        self.f_op = _c4(self.f_ov + self.Lv)
        self.f_blk = _c4(self.f_op + self.Lp)
        self.b_rows = chunk * 32
        self.b_blk = _c4(self.b_rows + HCv + HCp)
        self.send_f = torch.empty(self.f_blk, dtype=torch.float32, device=dev)
        self.send_b = None
        self.red = None  # [HCv + HCp]: the reduced target-row gradient (filled by OwnRowsFn.backward)

    def rows_out(self):
        """The view hub's [own, 64] SV | XR destination inside the forward send block."""
        return self.send_f[:self.own * 64].view(self.own, 64)

    def backward_block(self):
        if self.send_b is None:
            self.send_b = torch.empty(self.b_blk, dtype=torch.float32, device=self.dev)
        return self.send_b

    def dagg_out(self):
        """The view tail's own-row camera-aggregate gradient [own, 32] inside the backward send block."""
        return self.backward_block()[:self.own * 32].view(self.own, 32)


class OwnRowsFn(torch.autograd.Function):
    """Replicated camera rows [m, ...] -> this rank's rows [c0, c1); the backward all-gathers the
    own-row gradients (each rank's slice is the full gradient of its rows).  exch (BlockExchange):
    the gather also carries the global target rows' partial gradients (and sums them)."""

    @staticmethod
    def forward(ctx, x, shard, exch=None):
        ctx.shard, ctx.exch = shard, exch
        c0, c1, _, _ = shard.cams
        return x[c0:c1]

    @staticmethod
    def backward(ctx, g):
        shard, ex = ctx.shard, ctx.exch
        _, _, chunk, m = shard.cams
        if ex is None or g.dim() != 2 or g.shape[1] != 32:
            return shard.all_gather(_pad_rows(g, chunk))[:m], None, None
        send = ex.backward_block()
        head = ex.dagg_out()
        if g.data_ptr() != head.data_ptr() or not g.is_contiguous():  # the view tail wrote elsewhere
            head.copy_(g)
        G = shard.all_gather(send.view(1, -1)).view(-1)
        full = torch.empty((m, 32), dtype=torch.float32, device=g.device)
        sums = (ex.b_rows, ex.red) if ex.red is not None else None
        _native.exchange_unpack(G, shard.world, ex.b_blk, rows=(0, chunk, full), sums=sums)
        ctx.exch = None
        return full, None, None


def _packed_block(xs):
    """The [rows, sum of widths] block when the 2-D tensors xs are consecutive column ranges of one
    row-major buffer (ViewHubFn(packed=True)'s SV | XR), else None."""
    if len(xs) < 2 or any(x.dim() != 2 or x.stride(1) != 1 for x in xs):
        return None
    rows, tot = xs[0].shape[0], sum(x.shape[1] for x in xs)
    at = 0
    for x in xs:
        if x.shape[0] != rows or (rows > 1 and x.stride(0) != tot) or \
                x.data_ptr() != xs[0].data_ptr() + at * x.element_size():
            return None
        at += x.shape[1]
    return xs[0].as_strided((rows, tot), (tot, 1))


def _as_rows(x):
    """[rows, prod(other dims)] (reshape(rows, -1) is ambiguous for 0 rows)."""
    return x.reshape(x.shape[0], int(np.prod(x.shape[1:])))


class GatherRowsFn(torch.autograd.Function):
    """Own camera rows of several [own, w_k] tensors -> the full [m, w_k] tensors, with ONE
    all-gather of their concatenation (no concatenation when they already are one row block:
    ViewHubFn(packed=True)); 2-D outputs are column views of the gathered block.  The backward
    slices the own rows of each gradient (the gradients arriving here are already summed over
    ranks: AllReduceGradN downstream, or replicated losses)."""

    @staticmethod
    def forward(ctx, shard, *xs):
        ctx.shard = shard
        _, _, chunk, m = shard.cams
        flat = _packed_block(xs)
        if flat is None:
            # explicit widths: a rank without camera rows (camera_rows past m) has 0-row blocks
            flat = torch.cat([_as_rows(x) for x in xs], 1) if len(xs) > 1 else _as_rows(xs[0])
        full = shard.all_gather(_pad_rows(flat, chunk))[:m]
        out, at = [], 0
        for x in xs:
            k = int(np.prod(x.shape[1:]))
            o = full[:, at:at + k]
            out.append(o if x.dim() == 2 else o.reshape((m,) + tuple(x.shape[1:])))
            at += k
        return tuple(out)

    @staticmethod
    def backward(ctx, *gs):
        c0, c1, _, _ = ctx.shard.cams
        return (None,) + tuple(None if g is None else g[c0:c1].contiguous() for g in gs)


def own_rows(x, shard, exch=None):
    return x if shard is None or shard.cams is None else OwnRowsFn.apply(x, shard, exch)


def gather_rows(shard, *xs):
    if shard is None or shard.cams is None:
        return xs
    return GatherRowsFn.apply(shard, *xs)


def replicated_to_local(x, shard):
    return x if shard is None else AllReduceGrad.apply(x, shard)


def replicated_to_local_n(shard, *xs):
    return xs if shard is None else AllReduceGradN.apply(shard, *xs)


class ShardedAttentionFn(torch.autograd.Function):
    """GATv2 attention whose destinations are replicated but whose edges are sharded.

    forward: local partial -> all-gather -> ordered combine (identical on all ranks)
    backward: local edges against the global max/sum/out -> dXL (local), dXR and datt
              (partial: summed by AllReduceGrad / sync_grads), dbias (already full).
    """

    @staticmethod
    def forward(ctx, XL, XR, att, bias, plan, plan_partial, heads, slope, shard):
        part = attn_forward_partial(XL, XR, att, plan_partial, heads, slope)
        gathered = shard.all_gather(part)
        N = plan.num_targets
        out, smax, ssum = combine_partials(gathered, shard.world, N, heads, bias, shard.combine_items(N, XL.device))
        ctx.plan, ctx.heads, ctx.slope = plan, heads, slope
        ctx.defer = _native.defer_token(att, bias)
        ctx.save_for_backward(XL, XR, att, bias, out, smax, ssum)
        return out

    @staticmethod
    def backward(ctx, g):
        XL, XR, att, bias, out, smax, ssum = ctx.saved_tensors
        dXL, dXR, datt, dbias = attn_backward_raw(XL, XR, att, bias, ctx.plan, ctx.heads, ctx.slope, out, smax,
                                                  ssum, g, defer=ctx.defer)
        if ctx.plan.num_targets > 1:  # replicated targets: the rank-independent sum (edge_block.replicated_dbias)
            from .edge_block import replicated_dbias
            dbias = replicated_dbias(g, ctx.defer)
        return dXL, dXR, datt.view_as(att), dbias, None, None, None, None, None


class ShardedGlobalAttentionFn(torch.autograd.Function):
    """The view->global and points->global GATv2 attentions of a block (one replicated target
    each) when both the views and the points are sharded: each rank attends over its own views /
    points, the two packed partial rows go out in ONE all-gather and are merged in rank order
    (identical on all ranks).  Backward: local edges against the global statistics; the two
    target-row gradients (partial per rank) are summed in ONE all-reduce."""

    @staticmethod
    def forward(ctx, XLv, XRv, att_v, bias_v, XLp, XRp, att_p, bias_p, plans, heads, slope, shard):
        """-> [1, HCv + HCp]: the two aggregates side by side (the global MLP's input)."""
        plan_v, plan_vp, plan_p, plan_pp = plans
        HCv, HCp = att_v.numel(), att_p.numel()
        Lv, Lp = HCv + 2 * heads, HCp + 2 * heads
        dev = XLv.device
        f32 = dict(dtype=torch.float32, device=dev)
        B, ov = _pack_layout(Lv, Lp)
        # both partial rows straight into one send block: v at float 0, p at float ov, B floats
        # per rank, so that in the gathered [W*B] buffer rank r's rows are slots r*B/Lv (v) and
        # (r*B + ov)/Lp (p) of row width Lv / Lp: the combines read them in place
        pack = torch.empty(B, **f32)
        ctx.fused = gatt_ok(plan_v, heads, XLv, XRv, att_v, bias_v) and gatt_ok(plan_p, heads, XLp, XRp, att_p, bias_p)
        if ctx.fused:  # both partial rows from one launch (global_attn.hip)
            _native.gatt_fwd([gatt_prob(plan_v, XLv, XRv, att_v, bias_v, part=pack[:Lv]),
                              gatt_prob(plan_p, XLp, XRp, att_p, bias_p, part=pack[ov:ov + Lp])], slope)
        else:
            attn_forward_partial(XLv, XRv, att_v, plan_vp, heads, slope, dst=pack[:Lv].view(1, Lv))
            attn_forward_partial(XLp, XRp, att_p, plan_pp, heads, slope, dst=pack[ov:ov + Lp].view(1, Lp))
        g = shard.all_gather(pack.view(1, B)).view(-1)
        xcat = torch.empty((1, HCv + HCp), **f32)
        stats = torch.empty((4, heads), **f32)
        W = shard.world
        if ctx.fused:  # both merges in one launch
            _native.gatt_merge([dict(part=g, bias=bias_v, out=xcat[:, :HCv], smax=stats[0], ssum=stats[1]),
                                dict(part=g[ov:], bias=bias_p, out=xcat[:, HCv:], smax=stats[2], ssum=stats[3])],
                               W, B)
        else:
            items = shard.pack_items(((0, W, B // Lv), (ov // Lp, W, B // Lp)), dev)
            _native.attn_combine(items[0], 1, heads, HCv // heads, g.view(-1, Lv), bias_v, True, xcat[:, :HCv],
                                 stats[0:1], stats[1:2])
            _native.attn_combine(items[1], 1, heads, HCp // heads, g.view(-1, Lp), bias_p, True, xcat[:, HCv:],
                                 stats[2:3], stats[3:4])
        ctx.plans, ctx.heads, ctx.slope, ctx.shard, ctx.HCv = (plan_v, plan_p), heads, slope, shard, HCv
        ctx.defer = _native.defer_token(att_v, bias_v, att_p, bias_p)
        ctx.save_for_backward(XLv, XRv, att_v, bias_v, XLp, XRp, att_p, bias_p, xcat, stats)
        return xcat

    @staticmethod
    def backward(ctx, g):
        XLv, XRv, att_v, bias_v, XLp, XRp, att_p, bias_p, xcat, stats = ctx.saved_tensors
        plan_v, plan_p = ctx.plans
        HCv = ctx.HCv
        g = g.contiguous()
        flat = torch.empty_like(xcat)  # [dXRv | dXRp]: the all-reduce payload, written in place
        if ctx.fused:
            HCp = xcat.shape[1] - HCv
            dXLv, dXLp = gatt_dxl(plan_v, XLv, HCv), gatt_dxl(plan_p, XLp, HCp)
            dab = torch.empty(2 * (HCv + HCp), dtype=torch.float32, device=xcat.device)
            _native.gatt_bwd([gatt_prob(plan_v, XLv, XRv, att_v, bias_v, out=xcat[:, :HCv], smax=stats[0],
                                        ssum=stats[1], gout=g[:, :HCv], dXL=dXLv, dXR=flat[:, :HCv],
                                        datt=dab[:2 * HCv]),
                              gatt_prob(plan_p, XLp, XRp, att_p, bias_p, out=xcat[:, HCv:], smax=stats[2],
                                        ssum=stats[3], gout=g[:, HCv:], dXL=dXLp, dXR=flat[:, HCv:],
                                        datt=dab[2 * HCv:])], ctx.slope)
            ctx.shard.all_reduce_(flat)
            o = 2 * HCv
            return (dXLv, flat[:, :HCv].view_as(XRv), dab[:HCv].view_as(att_v), dab[HCv:o].view_as(bias_v), dXLp,
                    flat[:, HCv:].view_as(XRp), dab[o:o + HCp].view_as(att_p), dab[o + HCp:].view_as(bias_p), None,
                    None, None, None)
        dXLv, _, dattv, dbv = attn_backward_raw(XLv, XRv, att_v, bias_v, plan_v, ctx.heads, ctx.slope,
                                                xcat[:, :HCv], stats[0:1], stats[1:2], g[:, :HCv],
                                                defer=ctx.defer, dXR=flat[:, :HCv])
        dXLp, _, dattp, dbp = attn_backward_raw(XLp, XRp, att_p, bias_p, plan_p, ctx.heads, ctx.slope,
                                                xcat[:, HCv:], stats[2:3], stats[3:4], g[:, HCv:],
                                                defer=ctx.defer, dXR=flat[:, HCv:])
        ctx.shard.all_reduce_(flat)
        return (dXLv, flat[:, :HCv], dattv.view_as(att_v), dbv, dXLp, flat[:, HCv:], dattp.view_as(att_p), dbp,
                None, None, None, None)


class ShardedGlobalExchangeFn(torch.autograd.Function):
    """ShardedGlobalAttentionFn and GatherRowsFn(SV, XR) of a camera-sharded block with ONE
    all-gather (BlockExchange): the view hub wrote this rank's [own, 64] SV | XR rows into the
    forward send block, the global convs write their two partial rows after them; one launch merges
    the partials and unpacks every rank's rows.  -> (xcat [1, HCv + HCp], SV [m, 32], XR [m, 32]).

    Backward: the global convs against the merged statistics; their target-row gradients (partial
    per rank) go into the backward send block and are summed by the NEXT collective of this block,
    OwnRowsFn's (defer_xr; the returned gradients are views of exch.red, filled there: their
    consumer is the previous block's GlobalChainFn, whose backward also needs this block's boundary
    all-reduce, which comes after OwnRowsFn's).  Without defer_xr (block 0: the target rows are
    lin_r(0), consumed at once) they are all-reduced here.  SV / XR: own-row slices of the
    (already summed) gradients, as GatherRowsFn."""

    @staticmethod
    def forward(ctx, XLv, XRv, att_v, bias_v, XLp, XRp, att_p, bias_p, SV_own, XR_own, plans, heads, slope, shard,
                exch, defer_xr):
        plan_v, plan_p = plans
        HCv, HCp = att_v.numel(), att_p.numel()
        dev = XLv.device
        f32 = dict(dtype=torch.float32, device=dev)
        ex = exch
        rows = ex.rows_out()
        if ex.own and (SV_own.data_ptr() != rows.data_ptr() or XR_own.data_ptr() != rows[:, 32:].data_ptr()):
            rows[:, :32].copy_(SV_own)
            rows[:, 32:].copy_(XR_own)
        send = ex.send_f
        _native.gatt_fwd([gatt_prob(plan_v, XLv, XRv, att_v, bias_v, part=send[ex.f_ov:ex.f_ov + ex.Lv]),
                          gatt_prob(plan_p, XLp, XRp, att_p, bias_p, part=send[ex.f_op:ex.f_op + ex.Lp])], slope)
        G = shard.all_gather(send.view(1, -1)).view(-1)
        xcat = torch.empty((1, HCv + HCp), **f32)
        stats = torch.empty((4, heads), **f32)
        full = torch.empty((ex.m, 64), **f32)
        _native.gatt_merge([dict(part=G[ex.f_ov:], bias=bias_v, out=xcat[:, :HCv], smax=stats[0], ssum=stats[1]),
                            dict(part=G[ex.f_op:], bias=bias_p, out=xcat[:, HCv:], smax=stats[2], ssum=stats[3])],
                           shard.world, ex.f_blk, unpack=(G, ex.f_blk, 0, ex.chunk, full))
        ctx.plans, ctx.heads, ctx.slope, ctx.shard, ctx.HCv = (plan_v, plan_p), heads, slope, shard, HCv
        ctx.exch, ctx.defer_xr = ex, bool(defer_xr)
        ctx.defer = _native.defer_token(att_v, bias_v, att_p, bias_p)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(XLv, XRv, att_v, bias_v, XLp, XRp, att_p, bias_p, xcat, stats)
        return xcat, full[:, :32], full[:, 32:]

    @staticmethod
    def backward(ctx, g, gSV, gXR):
        XLv, XRv, att_v, bias_v, XLp, XRp, att_p, bias_p, xcat, stats = ctx.saved_tensors
        plan_v, plan_p = ctx.plans
        HCv = ctx.HCv
        HCp = xcat.shape[1] - HCv
        ex, shard = ctx.exch, ctx.shard
        c0, c1, _, _ = shard.cams
        dev = xcat.device
        g = g.contiguous() if g is not None else torch.zeros_like(xcat)
        if ctx.defer_xr:  # the partial into the backward send block, summed by OwnRowsFn's gather
            send = ex.backward_block()
            flat = send[ex.b_rows:ex.b_rows + HCv + HCp].view(1, HCv + HCp)
            ex.red = torch.empty(HCv + HCp, dtype=torch.float32, device=dev)
            red = ex.red.view(1, HCv + HCp)
        else:
            flat = torch.empty_like(xcat)
            red = flat
        dXLv, dXLp = gatt_dxl(plan_v, XLv, HCv), gatt_dxl(plan_p, XLp, HCp)
        dab = torch.empty(2 * (HCv + HCp), dtype=torch.float32, device=dev)
        _native.gatt_bwd([gatt_prob(plan_v, XLv, XRv, att_v, bias_v, out=xcat[:, :HCv], smax=stats[0], ssum=stats[1],
                                    gout=g[:, :HCv], dXL=dXLv, dXR=flat[:, :HCv], datt=dab[:2 * HCv]),
                          gatt_prob(plan_p, XLp, XRp, att_p, bias_p, out=xcat[:, HCv:], smax=stats[2], ssum=stats[3],
                                    gout=g[:, HCv:], dXL=dXLp, dXR=flat[:, HCv:], datt=dab[2 * HCv:])], ctx.slope)
        if not ctx.defer_xr:
            shard.all_reduce_(flat)
        o = 2 * HCv
        own = lambda t: None if t is None else t[c0:c1].contiguous()  # noqa: E731
        return (dXLv, red[:, :HCv].view_as(XRv), dab[:HCv].view_as(att_v), dab[HCv:o].view_as(bias_v), dXLp,
                red[:, HCv:].view_as(XRp), dab[o:o + HCp].view_as(att_p), dab[o + HCp:].view_as(bias_p),
                own(gSV), own(gXR), None, None, None, None, None, None)


def _pack_layout(a, b):
    """(B, ov): a send block of B floats holding an a-float row at 0 and a b-float row at ov, with
    B a multiple of both a and b and ov of b (rows stay addressable as slots after the gather)."""
    from math import gcd
    lcm = a * b // gcd(a, b)
    ov = -(-a // b) * b
    return lcm * max(1, -(-(ov + b) // lcm)), ov


def partition_points(pt, n, world):
    """Contiguous point ranges with ~equal edge counts: returns boundaries [world+1]."""
    counts = np.bincount(np.asarray(pt), minlength=n)
    csum = np.concatenate([[0], np.cumsum(counts)])
    E = csum[-1]
    bounds = [0]
    for r in range(1, world):
        bounds.append(int(np.searchsorted(csum, E * r / world, side="left")))
    bounds.append(n)
    return np.maximum.accumulate(np.asarray(bounds))


def shard_scene(scene, rank, world, max_piece=None, cameras=False, emulate=False, point_bounds=None):
    """Rank-local SceneData of a synthetic (or any cam-major) scene.

    scene: object with m, n, cam, pt (cam-major sorted) and normalized_values().
    cameras: shard the camera (view) rows too (module docstring).  emulate: a ShardContext
    without a process group (see ShardContext).  point_bounds: explicit contiguous point ranges
    [world + 1] (default: partition_points' edge-balanced split).
    """
    cam = np.asarray(scene.cam)
    pt = np.asarray(scene.pt)
    m, n = scene.m, scene.n
    if point_bounds is None:
        bounds = partition_points(pt, n, world)
    else:
        bounds = np.asarray(point_bounds, dtype=np.int64)
        if bounds.shape != (world + 1,) or bounds[0] != 0 or bounds[-1] != n or np.any(np.diff(bounds) < 0):
            raise ValueError(f"point_bounds must be {world + 1} non-decreasing boundaries from 0 to {n}")
    p0, p1 = int(bounds[rank]), int(bounds[rank + 1])
    sel = (pt >= p0) & (pt < p1)
    vals = scene.normalized_values()[sel]
    lcam, lpt = cam[sel], pt[sel] - p0
    data = SceneData.from_sparse(lcam, lpt, vals, m, p1 - p0, scene_name=f"shard{rank}", max_piece=max_piece,
                                 cam_max_piece=camera_max_piece(len(lcam)) if max_piece is None else None)
    gw = data.graph_wrappers
    # view validity is a GLOBAL property (>= 8 points over all ranks): replicated view2global plan
    pts_per_cam = np.bincount(cam, minlength=m)
    vv = torch.from_numpy(np.nonzero(pts_per_cam >= MIN_N_POINTS_PER_VIEW)[0].astype(np.int64))
    gw["view2global"].valid_indices = torch.stack([vv, torch.zeros_like(vv)])
    gw["view2global"].plan = AttnPlan.from_targets(torch.zeros_like(vv), 1, src=vv, src_rows=m, max_piece=8)
    gw["view2global"].plan.tag = "view2global"
    # partial (exchange) plans for the camera direction and the points -> global graph
    data.partial_plans = {
        "proj2view": AttnPlan.from_targets(lcam, m, all_partial=True,
                                           max_piece=camera_max_piece(len(lcam)) if max_piece is None else max_piece),
        "scenepoint2global": AttnPlan.from_targets(
            torch.zeros(gw["scenepoint2global"].plan.num_edges, dtype=torch.int64), 1,
            src=gw["scenepoint2global"].valid_indices[1], src_rows=p1 - p0, all_partial=True,
            max_piece=gw["scenepoint2global"].plan.max_piece),
    }
    for k, p in data.partial_plans.items():
        p.tag = k + "_partial"
    cams = None
    if cameras:
        c0, c1, chunk = camera_rows(m, world, rank)
        cams = (c0, c1, chunk, m)
        own = vv[(vv >= c0) & (vv < c1)] - c0
        kw8 = {"max_piece": 8}
        plan = AttnPlan.from_targets(torch.zeros_like(own), 1, src=own, src_rows=c1 - c0, **kw8)
        plan.tag = "view2global"
        gw["view2global"].plan = plan
        data.partial_plans["view2global"] = AttnPlan.from_targets(torch.zeros_like(own), 1, src=own,
                                                                  src_rows=c1 - c0, all_partial=True, **kw8)
        data.partial_plans["view2global"].tag = "view2global_partial"
        data.camera_slice = slice(c0, c1)
    data.point_slice = slice(p0, p1)
    data.n_global = n
    data.n_edges_global = int(pt.shape[0])
    data.shard = ShardContext(rank, world, cams=cams, emulate=emulate)
    return data


class ShardedGraphAttnSfMNet(torch.nn.Module):
    """Wraps a GraphAttnSfMNet for point-sharded execution on this rank.

    forward(data) with data from ``shard_scene``: returns Ps_norm (replicated, all
    cameras) and pts3D for this rank's points only.  Call ``sync_grads()`` after
    backward (sums the gradients of rank-local parameters over the ranks).
    """

    def __init__(self, net, group=None, cameras=False):
        """cameras: the scenes come from shard_scene(..., cameras=True) (view rows sharded too):
        every parameter outside the global chain then carries a partial gradient."""
        super().__init__()
        self.net = net
        self.group = group
        self.cameras = cameras
        self.local_names = [k for k, _ in net.named_parameters() if is_local_param(k, cameras)]
        self._emulate = None
        self._reducer = None
        if cameras:  # the large partial gradients are all-reduced as soon as they exist
            for k, p in net.named_parameters():
                if k in self.local_names and p.dim() == 2 and p.numel() >= 1 << 20:
                    p.register_post_accumulate_grad_hook(self._reduce_hook)

    def _reduce_hook(self, p):
        if self._reducer is not None:
            self._reducer.launch(p.grad)

    def forward(self, data):
        shard = data.shard
        if (shard.cams is not None) != self.cameras:
            raise ValueError("ShardedGraphAttnSfMNet(cameras=...) must match shard_scene(..., cameras=...)")
        shard.group = self.group
        self._emulate = shard if shard.emulate else None
        self._reducer = None
        if self.cameras and torch.is_grad_enabled() and all(p.grad is None for p in self.net.parameters()):
            self._reducer = AsyncGradReducer(shard)
        return self.net.forward(data, shard=shard, partial_plans=data.partial_plans)

    def sync_grads(self):
        """One all-reduce of every rank-local parameter's gradient, in a fixed layout: a parameter
        without a gradient on this rank contributes zeros (and gets the summed gradient), so all
        ranks reduce buffers of the same size and order."""
        red = getattr(self, "_reducer", None)
        self._reducer = None
        if red is not None:
            red.wait()
        if self._emulate is None and dist.get_world_size(self.group) == 1:
            return
        params = dict(self.net.named_parameters())
        done = red.ptrs if red is not None else ()
        ps = [params[k] for k in self.local_names
              if params[k].grad is None or params[k].grad.data_ptr() not in done]
        if not ps:
            return
        dev = ps[0].device
        flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1).to(dev) for p in ps])
        shard = self._emulate or ShardContext(dist.get_rank(self.group), dist.get_world_size(self.group), self.group)
        shard.all_reduce_(flat)
        # the summed gradients stay in the bucket: each .grad becomes a view of it (a copy back per
        # parameter was ~620 copy launches per step with the camera chain sharded)
        off = 0
        for p in ps:
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
