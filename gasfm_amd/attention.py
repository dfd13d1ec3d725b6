"""Destination-grouped attention plans and the autograd wrapper of the HIP kernels.

An ``AttnPlan`` is the MI355X-side form of one of the reference's star graphs
(``AxialAggregationGraphWrapper.edge_index``, utils/dataset_utils.py:511-537):
instead of an edge_index over E+N concatenated nodes it stores, per
destination segment, the range of its edges in destination order plus (for
the unsorted point direction) the permutation into edge order, and the split
of long segments into balanced work items.  Plans are built once per scene on
the CPU (DataLoader-worker safe) and moved to the device with ``.to``.

``gat_attention`` is the differentiable fused edge-softmax + aggregation:
forward and backward are the HIP kernels of gasfm_amd/csrc/gat_attn.hip; no
PyTorch or CPU fallback exists (a missing library raises).
"""
import copy
import os

import numpy as np
import torch

from . import _native

DEFAULT_MAX_PIECE = int(os.environ.get("GASFM_DEFAULT_PIECE", "256"))  # edges per work item (env: A/B knob)
_MAX_PIECE_ENV = os.environ.get("GASFM_MAX_PIECE")  # A/B knob: a fixed camera-direction piece length


def camera_max_piece(num_edges):
    """Edges per work item of a point shard's camera-direction plan over num_edges edges
    (distributed.shard_scene; whole scenes and training batches keep DEFAULT_MAX_PIECE: a training
    batch is host-bound and measured 6 ms per step slower with the extra split pieces' launches).

    256 (DEFAULT_MAX_PIECE), stepped down through 128, 64 and 48 while the plan would hold fewer than
    ~4 items per resident wave of the camera-item edge kernels (512 workgroups x 4 waves): a
    1/8-points shard (~500 edges per camera) otherwise runs edge_cam_pbwd / edge_seam_fwd /
    edge_epilogue_bwd at about one 16-tile item per wave.  Rank 0 of 8 (bench.py --emulate-world 8):
    9.92 ms at 256, 9.33 at 128, 9.26 at 64 (round 3); the whole config-4 scene stays at 256 (31.94 vs
    32.15 ms at 128).  Round 6, the 48 step: at 64 the shard's 8,277 pieces are 4.04 per resident wave,
    so the 85 waves that take a fifth 4-tile piece set the launch's length (the grid-stride maximum is
    20 tiles per wave against a mean of 16.2); 3-tile pieces spread the tail: edge_cam_pbwd 118.3 ->
    113.4 us, the proxy 7.13-7.14 -> 7.04-7.05 ms (32: 7.11-7.12, 96: 7.13; profiles/r6_ab_cam_piece.txt).
    """
    if _MAX_PIECE_ENV:
        return int(_MAX_PIECE_ENV)
    mp = DEFAULT_MAX_PIECE
    while mp > 48 and num_edges < 8192 * mp:
        mp = mp // 2 if mp > 64 else 48
    return mp
LANES_MAX_AVG = 32  # 4-wide convs with <= this many edges per item on average: one lane per item
# The lane-per-item forward replaced a 226 us launch by a 43 us one at config 4.  The backward with
# one lane per item measured 193 us against 153 us for the wave-per-item kernel (its dXL rows are
# scattered into edge order either way); with a group of 8 lanes per item (round 3: a group's rows
# per step are one 128-B line) it takes 98 us against the wave-per-item kernel's 134 us in the
# config-4 step (tools/gpu_lanes_ab.sh), so it is the default; GASFM_ATTN_BWD_LANES=0 restores the
# general kernel.
BWD_LANES = os.environ.get("GASFM_ATTN_BWD_LANES", "1") != "0"
# The two convs onto the global node as ONE forward and ONE backward launch (global_attn.hip, round
# 4) instead of an attention kernel + ordered combines per conv (~6 launches each way per block).
# Measured in three versions on one box each: 64-view / 2048-point chunks with
# atomic-load merges slower everywhere (profiles/r4_ab3.txt); 8 / 256 chunks with plain batched
# merges faster on a rank's shard only (r4_ab5.txt); with the two-level merge faster at both sizes:
# config 4 29.81-29.85 -> 29.51-29.60 ms, the rank-0-of-8 proxy 7.87-7.88 -> 7.61-7.62 ms
# (r4_ab7.txt).  GASFM_GLOBAL_ATTN=0 restores the plan kernels; GASFM_GATT_MAX_SRC caps the point
# sources it takes (default: no cap).
GLOBAL_ATTN = os.environ.get("GASFM_GLOBAL_ATTN", "1") != "0"
GATT_MAX_SRC = int(os.environ.get("GASFM_GATT_MAX_SRC", str(1 << 62)))


def gatt_ok(plan, heads, XL, XR, att, bias=None):
    """Whether the fused global-conv kernels take this single-target conv (H = 4, C in {16, 256}).
    Inputs the kernels cannot read (dtype, alignment) take the plan kernels instead."""
    HC = att.numel()
    if not GLOBAL_ATTN or plan.num_targets != 1 or heads != 4 or HC not in (64, 1024):
        return False
    if plan.num_edges > GATT_MAX_SRC:
        return False
    if XL.dim() != 2 or XL.shape[1] != HC or XL.stride(1) != 1 or XL.stride(0) % 4 or XL.data_ptr() % 16:
        return False
    if XL.shape[0] < plan.src_rows or (plan.perm is not None and plan.perm.dtype != torch.int32):
        return False
    if any(t.dtype != torch.float32 for t in (XL, XR, att)):
        return False
    # att / bias are read as float4 columns (global_attn.hip): 16-byte aligned, unit stride
    if not att.is_contiguous() or att.data_ptr() % 16:
        return False
    if bias is not None and (bias.dtype != torch.float32 or not bias.is_contiguous() or bias.data_ptr() % 16):
        return False
    return XR.numel() == HC and XR.is_contiguous() and XR.data_ptr() % 16 == 0


def gatt_prob(plan, XL, XR, att, bias, **kw):
    return dict(XL=XL, src=plan.perm, S=plan.num_edges, XR=XR, att=att.reshape(-1), bias=bias, **kw)


def gatt_dxl(plan, XL, HC):
    """The dXL buffer of a fused global conv: only source rows are written, so zero-filled unless
    the plan's sources cover every row."""
    full = plan.num_edges == XL.shape[0] == plan.src_rows
    return (torch.empty if full else torch.zeros)((XL.shape[0], HC), dtype=torch.float32, device=XL.device)


def _lanes(plan, heads, HC):
    """Block 0's point direction (H*C = 4, ~20-edge items): the lane-per-item kernels
    (csrc/attn_lanes.hip)."""
    return HC == 4 and heads == 4 and plan.num_edges <= LANES_MAX_AVG * plan.n_items

# Optional live kernel timer (bench.py): callable(tag, HC) -> bool selecting which
# attention launches to bracket with HIP events on the launch stream.
KERNEL_TIMER = None


class KernelTimer:
    """Records (start, end) torch.cuda.Events around selected kernel launches."""

    def __init__(self, select, hold_cycles=0):
        self.select = select
        self.events = []
        self.enabled = False
        self.hold_cycles = int(hold_cycles)  # hold(): spin-kernel length
        self.gathered = None  # whether the timed launches read XL through perm
        self.launch = None    # closure re-issuing the last timed launch (same inputs / outputs)

    def __call__(self, tag, HC):
        return self.enabled and self.select(tag, HC)

    def hold(self):
        """Before a timed launch: a spin kernel on the stream, so the start event, the kernel and the
        end event are all enqueued before the GPU reaches them -- the events then bracket the
        kernel's execution, not the host's enqueue latency (eager launches at a rank's shard size
        are host-bound: the GPU would otherwise sit idle between the start event and the kernel)."""
        if self.hold_cycles > 0:
            torch.cuda._sleep(self.hold_cycles)

    def mean_ms(self):
        torch.cuda.synchronize()
        if not self.events:
            return None
        return sum(a.elapsed_time(b) for a, b in self.events) / len(self.events)

    def replay_ms(self, reps=20):
        """Mean duration of ``reps`` back-to-back re-launches of the last timed kernel between
        two HIP events on the launch stream: the kernel time without the per-launch event and
        dispatch gaps that bracketing single launches adds (comparable to rocprof's durations)."""
        if self.launch is None:
            return None
        self.launch()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            self.launch()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps


class AttnPlan:
    """Edges grouped by destination segment (CSR), with balanced work items.

    seg_ptr  int32 [N+1]   edge range of each destination segment
    perm     int32 [E]     source row of the k-th edge in segment order, or None
                           when segment order == source row order (identity)
    pos      int32 [E]     inverse of perm (segment position of source row e) when perm
                           is a permutation of the E source rows, else None.  Producers
                           use it to write source rows directly in segment order, so the
                           attention kernels stream them instead of gathering (xl_sorted).
    items    int32 [I, 4]  (seg, begin, end, slot) work items (see gasfm.h)
    combine  int32 [K, 4]  (seg, slot_begin, slot_count, slot_stride)
    combine_l1 int32 [K1, 4] first level of the long combines: (row, slot_begin, count, 1)
                           merges ~sqrt(count) consecutive slots into partial row n_slots + k,
                           and ``combine`` then merges those rows.  One workgroup per entry
                           on both levels, so a single-target plan (points -> global: ~4k
                           slots) is combined by ~64 workgroups instead of one.
    """

    def __init__(self, seg_ptr, perm, items, combine, n_slots, num_targets, num_edges, src_rows,
                 all_partial=False, max_piece=DEFAULT_MAX_PIECE, pos=None, combine_l1=False):
        """combine_l1: the level-1 entries when ``combine`` is already split in two levels
        (scene_device.plan_work_device, on the device; None: one level); False: split here."""
        self.seg_ptr = seg_ptr
        self.perm = perm
        self.items = items
        self.combine = combine
        self.n_slots = int(n_slots)
        self.num_targets = int(num_targets)
        self.num_edges = int(num_edges)
        self.src_rows = int(src_rows)  # number of source rows the perm may reference
        self.all_partial = bool(all_partial)
        self.max_piece = int(max_piece)
        self.n_items = int(items.shape[0])
        dev = items.device
        if combine_l1 is not False:
            self.combine, self.combine_l1 = combine, combine_l1
        else:
            if isinstance(combine, torch.Tensor) and combine.device.type != "cpu":
                combine = combine.cpu()  # the two-level split is host bookkeeping over <= N entries
            self.combine, self.combine_l1 = _two_level(combine, self.n_slots)
            if dev.type != "cpu":
                self.combine = self.combine.to(dev)
                self.combine_l1 = None if self.combine_l1 is None else self.combine_l1.to(dev)
        self.n_combine = int(self.combine.shape[0])
        self.n_l1 = 0 if self.combine_l1 is None else int(self.combine_l1.shape[0])
        self.n_part_rows = self.n_slots + self.n_l1  # partial rows of both combine levels
        self.tag = None  # graph name (proj2view, proj2scenepoint, ...) for timing / logs
        self.pos = pos
        if pos is None and perm is not None and self.src_rows == self.num_edges:
            if isinstance(perm, torch.Tensor) and perm.device.type != "cpu":
                pos = torch.empty(self.num_edges, dtype=torch.int32, device=perm.device)
                pos[perm.long()] = torch.arange(self.num_edges, dtype=torch.int32, device=perm.device)
                self.pos = pos
            else:
                p = perm.numpy() if isinstance(perm, torch.Tensor) else perm
                pos = np.empty(self.num_edges, dtype=np.int32)
                pos[p] = np.arange(self.num_edges, dtype=np.int32)
                self.pos = torch.from_numpy(pos)

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_targets(cls, dst, num_targets, src=None, src_rows=None, max_piece=DEFAULT_MAX_PIECE,
                     all_partial=False):
        """Plan for edges e -> dst[e] (source row src[e], default e).

        ``dst``/``src`` are 1-D integer arrays (numpy or CPU tensors).  Sources must be
        unique (each source row has exactly one out-edge), which holds for every GASFM
        star graph; ``GATv2Conv.forward`` handles general graphs by gathering first.
        """
        dst = np.ascontiguousarray(torch.as_tensor(dst).cpu().numpy(), dtype=np.int32)
        E = int(dst.shape[0])
        if src is not None:
            src = np.ascontiguousarray(torch.as_tensor(src).cpu().numpy(), dtype=np.int32)
            assert src.shape == dst.shape
        if src_rows is None:
            src_rows = E if src is None else (int(src.max()) + 1 if E else 0)
        if E and (dst.min() < 0 or dst.max() >= num_targets):
            raise ValueError("destination index out of range")
        if E and np.all(dst[1:] >= dst[:-1]):
            seg_ptr = np.zeros(num_targets + 1, dtype=np.int32)
            np.cumsum(np.bincount(dst, minlength=num_targets), out=seg_ptr[1:])
            perm = None if src is None or np.array_equal(src, np.arange(E, dtype=np.int32)) else src.copy()
        else:
            seg_ptr, order = _native.build_csr(dst, num_targets)
            perm = order if src is None else src[order]
        items, comb, n_slots = _native.plan_work(seg_ptr, max_piece, all_partial)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a))
        return cls(t(seg_ptr), None if perm is None else t(perm), t(items), t(comb), n_slots, num_targets, E,
                   src_rows, all_partial, max_piece)

    def to(self, device, **kwargs):
        ret = copy.copy(self)
        for k in ("seg_ptr", "perm", "pos", "items", "combine", "combine_l1"):
            v = getattr(self, k)
            if v is not None:
                setattr(ret, k, v.to(device, **kwargs))
        return ret

    @property
    def device(self):
        return self.items.device

    def segment_lengths(self):
        return (self.seg_ptr[1:] - self.seg_ptr[:-1]).cpu().numpy()


L1_THRESHOLD = 32  # combines of more slots are split into two levels


def _two_level(combine, n_slots):
    """Split combine entries with > L1_THRESHOLD slots into ordered groups of ~sqrt(count).

    Returns (combine, combine_l1); level-1 entry k writes partial row n_slots + k, and the
    rewritten level-2 entry merges its group rows in order (deterministic)."""
    c = combine.numpy() if isinstance(combine, torch.Tensor) else np.asarray(combine)
    if c.size == 0 or int(c[:, 2].max()) <= L1_THRESHOLD:
        return combine, None
    assert np.all(c[:, 3] == 1), "plan_work combines use unit slot stride"
    top, l1 = [], []
    for seg, b, cnt, st in c.tolist():
        if cnt <= L1_THRESHOLD:
            top.append((seg, b, cnt, st))
            continue
        g = int(np.ceil(np.sqrt(cnt)))
        ng = -(-cnt // g)
        first = n_slots + len(l1)
        for k in range(ng):
            lo = b + k * g
            l1.append((first + k, lo, min(g, b + cnt - lo), 1))
        top.append((seg, first, ng, 1))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.int32).reshape(-1, 4)))
    return t(top), t(l1)


def combine_fwd_l1(plan, part, heads, C):
    """Level-1 merge of packed partial rows (raw) in place: rows [n_slots, n_part_rows)."""
    if plan.n_l1:
        HC = heads * C
        LDP = HC + 2 * heads
        _native.attn_combine(plan.combine_l1, plan.n_l1, heads, C, part, None, False, part, part[:, HC:],
                             part[:, HC + heads:], ldOut=LDP, ldStat=LDP)


def bwd_combine(plan, part, HC, out):
    """out[seg] = ordered sum of the plan's partial rows (both levels).  A single-target plan's
    (view->global, points->global: hundreds to thousands of pieces) sum is a column sum of all
    its slots: one last-arriver colsum launch instead of the two combine levels."""
    if plan.num_targets == 1 and plan.n_slots > 0 and out.shape[0] == 1:
        _native.colsum(part[:plan.n_slots], out=out.view(-1))
        return
    if plan.n_l1:
        _native.attn_bwd_combine(plan.combine_l1, plan.n_l1, HC, part, part)
    if plan.n_combine:
        _native.attn_bwd_combine(plan.combine, plan.n_combine, HC, part, out)


def _check(t, name, rows=None, cols=None):
    if not t.is_cuda or t.dtype != torch.float32:
        raise TypeError(f"{name}: expected a float32 CUDA tensor (no CPU fallback), got {t.dtype} on {t.device}")
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"{name}: expected 2-D tensor with unit column stride")
    if rows is not None and t.shape[0] < rows:
        raise ValueError(f"{name}: has {t.shape[0]} rows, plan needs {rows}")
    if cols is not None and t.shape[1] != cols:
        raise ValueError(f"{name}: has {t.shape[1]} columns, expected {cols}")


def bwd_combine2(plan, part_a, out_a, part_b, out_b, HC):
    """bwd_combine of two partial-row arrays over the same plan's slots (the camera plan's dXR and
    the folded epilogue's dSv rows), one launch per level instead of two."""
    if plan.num_targets == 1:
        bwd_combine(plan, part_a, HC, out_a)
        bwd_combine(plan, part_b, HC, out_b)
        return
    if plan.n_l1:
        _native.attn_bwd_combine2(plan.combine_l1, plan.n_l1, HC, part_a, part_a, part_b, part_b)
    if plan.n_combine:
        _native.attn_bwd_combine2(plan.combine, plan.n_combine, HC, part_a, out_a, part_b, out_b)


def attn_forward_raw(XL, XR, att, bias, plan, heads, slope, finalize=True, xl_sorted=False, out=None):
    """Launch the forward kernels; returns (out, seg_max, seg_sum) for all plan targets.

    xl_sorted: XL rows are already in segment order (written through plan.pos), so the
    kernel streams them (perm = NULL) instead of gathering.  out: optional [N, HC] row view
    (unit column stride) to write the aggregates into."""
    if plan.all_partial:
        raise ValueError("all-partial plans go through attn_forward_partial")
    HC = att.numel()
    C = HC // heads
    N = plan.num_targets
    dev = XL.device
    _check(XL, "XL", plan.src_rows, HC)
    _check(XR, "XR", N if XR.stride(0) else 1, HC)
    if out is None:
        out = torch.empty((N, HC), dtype=torch.float32, device=dev)
    smax = torch.empty((N, heads), dtype=torch.float32, device=dev)
    ssum = torch.empty((N, heads), dtype=torch.float32, device=dev)
    part = (torch.empty((plan.n_part_rows, HC + 2 * heads), dtype=torch.float32, device=dev)
            if plan.n_slots else None)
    attf = att.reshape(-1).contiguous()
    timed = KERNEL_TIMER is not None and KERNEL_TIMER(plan.tag, HC)
    if timed:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        KERNEL_TIMER.hold()
        ev[0].record()
    def launch():
        _native.attn_fwd(XL, XR, attf, bias, None if xl_sorted else plan.perm, plan.items, plan.n_items, heads, C,
                         slope, finalize, out, smax, ssum, part, lanes=_lanes(plan, heads, HC))
    launch()
    if timed:
        ev[1].record()
        KERNEL_TIMER.events.append(ev)
        KERNEL_TIMER.gathered = plan.perm is not None and not xl_sorted
        KERNEL_TIMER.launch = launch
    combine_fwd_l1(plan, part, heads, C)
    if plan.n_combine:
        _native.attn_combine(plan.combine, plan.n_combine, heads, C, part, bias, finalize, out, smax, ssum)
    return out, smax, ssum


def attn_forward_partial(XL, XR, att, plan, heads, slope, dst=None):
    """Un-normalised per-segment partials of an all-partial plan.

    Returns a packed [N, H*C + 2H] buffer (acc | max | sum) per destination segment —
    what one rank contributes before the cross-rank combine.  dst: an [N, H*C + 2H] row view
    (unit column stride) the merged rows are written to instead (a collective's send buffer).
    """
    assert plan.all_partial
    HC = att.numel()
    C = HC // heads
    N = plan.num_targets
    _check(XL, "XL", plan.src_rows, HC)
    _check(XR, "XR", N if XR.stride(0) else 1, HC)
    LDP = HC + 2 * heads
    part = torch.empty((max(plan.n_part_rows, N), LDP), dtype=torch.float32, device=XL.device)
    attf = att.reshape(-1).contiguous()
    _native.attn_fwd(XL, XR, attf, None, plan.perm, plan.items, plan.n_items, heads, C, slope, False, None, None,
                     None, part)
    out = part if dst is None else dst
    if plan.n_items == 0:  # no local edges: the empty state (acc 0, max -inf, sum 0)
        out[:N, :HC] = 0.0
        out[:N, HC:HC + heads] = -float("inf")
        out[:N, HC + heads:] = 0.0
        return out[:N]
    combine_fwd_l1(plan, part, heads, C)
    if dst is not None and (N > 1 or not plan.n_combine):
        # unsplit segments wrote their partial straight into part row seg (slot == seg); the
        # combine below only rewrites the split ones (all of them when N == 1)
        dst.copy_(part[:N])
    if plan.n_combine:  # merge split pieces (slots >= N) into rows [0, N), raw
        ld = out.stride(0) if N > 1 else LDP
        _native.attn_combine(plan.combine, plan.n_combine, heads, C, part, None, False, out, out[:, HC:],
                             out[:, HC + heads:], ldOut=ld, ldStat=ld)
    return out[:N]


def combine_partials(gathered, world, N, heads, bias, combine_items):
    """Finalize W stacked packed partial blocks [W*N, LDP] -> (out [N,HC], seg_max, seg_sum)."""
    HC = bias.numel()
    C = HC // heads
    out = torch.empty((N, HC), dtype=torch.float32, device=gathered.device)
    smax = torch.empty((N, heads), dtype=torch.float32, device=gathered.device)
    ssum = torch.empty((N, heads), dtype=torch.float32, device=gathered.device)
    _native.attn_combine(combine_items, N, heads, C, gathered, bias, True, out, smax, ssum)
    return out, smax, ssum


def attn_backward_raw(XL, XR, att, bias, plan, heads, slope, out, smax, ssum, gout, dXL=None, xl_sorted=False,
                      defer=False, dXR=None):
    """Launch the backward kernels; returns (dXL, dXR, datt[HC], dbias[HC]).

    dXL is in source-row (edge) order; xl_sorted says XL itself is in segment order.
    dXR: optional [num_targets, HC] row view (unit column stride) to write the target-row
    gradient into."""
    HC = att.numel()
    C = HC // heads
    dev = XL.device
    gout = gout if (gout.stride(1) == 1 and gout.stride(0) >= HC) else gout.contiguous()
    if dXL is None:
        # every source row is written exactly once when the plan's edges cover all rows
        full = plan.num_edges == XL.shape[0] == plan.src_rows
        dXL = (torch.empty if full else torch.zeros)((XL.shape[0], HC), dtype=torch.float32, device=dev)
    if dXR is None:
        dXR = torch.empty((plan.num_targets, HC), dtype=torch.float32, device=dev)
    part = torch.empty((plan.n_part_rows, HC), dtype=torch.float32, device=dev) if plan.n_slots else None
    n_waves = _native.attn_bwd_waves(plan.n_items, heads, C)
    datt_part = torch.empty((max(n_waves, 1), 2 * HC), dtype=torch.float32, device=dev)
    attf = att.reshape(-1).contiguous()
    if plan.n_items:
        _native.attn_bwd(XL, XR, attf, bias, plan.perm, plan.items, plan.n_items, heads, C, slope, out, smax,
                         ssum, gout, dXL, dXR, part, datt_part, xl_by_position=xl_sorted,
                         lanes=BWD_LANES and _lanes(plan, heads, HC))
        bwd_combine(plan, part, HC, dXR)
        tot = _native.param_colsum(datt_part, defer)  # datt | dbias: parameter gradients
        datt, dbias = tot[:HC], tot[HC:]
    else:
        dXR.zero_()
        datt = torch.zeros(HC, dtype=torch.float32, device=dev)
        dbias = torch.zeros(HC, dtype=torch.float32, device=dev)
    return dXL, dXR, datt, dbias


class GatAttentionFn(torch.autograd.Function):
    """out[i] = sum_{j->i} softmax_j(att . leaky_relu(XL[j] + XR[i])) XL[j] + bias."""

    @staticmethod
    def forward(ctx, XL, XR, att, bias, plan, heads, slope, xl_sorted=False):
        """xl_sorted: XL rows in segment order (written through plan.pos); the XL gradient is
        returned in source-row (edge) order."""
        out, smax, ssum = attn_forward_raw(XL, XR, att, bias, plan, heads, slope, finalize=True, xl_sorted=xl_sorted)
        ctx.plan, ctx.heads, ctx.slope = plan, heads, slope
        ctx.xl_sorted = xl_sorted
        ctx.defer = _native.defer_token(att, bias)
        ctx.save_for_backward(XL, XR, att, bias, out, smax, ssum)
        ctx.mark_non_differentiable(smax, ssum)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for the statistics outputs
        return out, smax, ssum

    @staticmethod
    def backward(ctx, gout, _gm, _gs):
        XL, XR, att, bias, out, smax, ssum = ctx.saved_tensors
        if gout is None:
            return None, None, None, None, None, None, None, None
        dXL, dXR, datt, dbias = attn_backward_raw(XL, XR, att, bias, ctx.plan, ctx.heads, ctx.slope, out, smax,
                                                  ssum, gout, xl_sorted=ctx.xl_sorted, defer=ctx.defer)
        return dXL, dXR, datt.view_as(att), dbias, None, None, None, None


class GlobalPairFn(torch.autograd.Function):
    """The view->global and points->global attentions of a block (one target each) written side by
    side into the global MLP's [1, HCv + HCp] input: no concatenation kernel either way."""

    @staticmethod
    def forward(ctx, XLv, XRv, att_v, bias_v, XLp, XRp, att_p, bias_p, plan_v, plan_p, heads, slope):
        HCv, HCp = att_v.numel(), att_p.numel()
        x = torch.empty((1, HCv + HCp), dtype=torch.float32, device=XLv.device)
        ctx.fused = gatt_ok(plan_v, heads, XLv, XRv, att_v, bias_v) and gatt_ok(plan_p, heads, XLp, XRp, att_p, bias_p)
        if ctx.fused:
            st = torch.empty((4, heads), dtype=torch.float32, device=XLv.device)
            mv, sv, mp, sp = st[0:1], st[1:2], st[2:3], st[3:4]
            _native.gatt_fwd([gatt_prob(plan_v, XLv, XRv, att_v, bias_v, out=x[:, :HCv], smax=mv, ssum=sv),
                              gatt_prob(plan_p, XLp, XRp, att_p, bias_p, out=x[:, HCv:], smax=mp, ssum=sp)], slope)
        else:
            _, mv, sv = attn_forward_raw(XLv, XRv, att_v, bias_v, plan_v, heads, slope, out=x[:, :HCv])
            _, mp, sp = attn_forward_raw(XLp, XRp, att_p, bias_p, plan_p, heads, slope, out=x[:, HCv:])
        ctx.plans, ctx.heads, ctx.slope, ctx.HCv = (plan_v, plan_p), heads, slope, HCv
        ctx.defer = _native.defer_token(att_v, bias_v, att_p, bias_p)
        ctx.save_for_backward(XLv, XRv, att_v, bias_v, XLp, XRp, att_p, bias_p, x, mv, sv, mp, sp)
        return x

    @staticmethod
    def backward(ctx, g):
        XLv, XRv, att_v, bias_v, XLp, XRp, att_p, bias_p, x, mv, sv, mp, sp = ctx.saved_tensors
        plan_v, plan_p = ctx.plans
        HCv = ctx.HCv
        g = g.contiguous()
        if ctx.fused:
            HCp = x.shape[1] - HCv
            dXLv, dXLp = gatt_dxl(plan_v, XLv, HCv), gatt_dxl(plan_p, XLp, HCp)
            dXR = torch.empty((1, HCv + HCp), dtype=torch.float32, device=x.device)
            dab = torch.empty(2 * (HCv + HCp), dtype=torch.float32, device=x.device)  # datt|dbias, v then p
            _native.gatt_bwd([gatt_prob(plan_v, XLv, XRv, att_v, bias_v, out=x[:, :HCv], smax=mv, ssum=sv,
                                         gout=g[:, :HCv], dXL=dXLv, dXR=dXR[:, :HCv], datt=dab[:2 * HCv]),
                              gatt_prob(plan_p, XLp, XRp, att_p, bias_p, out=x[:, HCv:], smax=mp, ssum=sp,
                                         gout=g[:, HCv:], dXL=dXLp, dXR=dXR[:, HCv:], datt=dab[2 * HCv:])],
                             ctx.slope)
            o = 2 * HCv
            return (dXLv, dXR[:, :HCv].view_as(XRv), dab[:HCv].view_as(att_v), dab[HCv:o].view_as(bias_v), dXLp,
                    dXR[:, HCv:].view_as(XRp), dab[o:o + HCp].view_as(att_p), dab[o + HCp:].view_as(bias_p), None,
                    None, None, None)
        dXLv, dXRv, dattv, dbv = attn_backward_raw(XLv, XRv, att_v, bias_v, plan_v, ctx.heads, ctx.slope,
                                                   x[:, :HCv], mv, sv, g[:, :HCv], defer=ctx.defer)
        dXLp, dXRp, dattp, dbp = attn_backward_raw(XLp, XRp, att_p, bias_p, plan_p, ctx.heads, ctx.slope,
                                                   x[:, HCv:], mp, sp, g[:, HCv:], defer=ctx.defer)
        return (dXLv, dXRv, dattv.view_as(att_v), dbv, dXLp, dXRp, dattp.view_as(att_p), dbp, None, None, None,
                None)


def gat_attention(XL, XR, att, bias, plan, heads, negative_slope=0.2):
    """Fused GATv2 attention over ``plan``; returns out [num_targets, H*C]."""
    if plan.device != XL.device:
        raise ValueError(f"plan on {plan.device}, features on {XL.device}: call plan.to(device) first")
    out, _, _ = GatAttentionFn.apply(XL, XR, att, bias, plan, heads, negative_slope)
    return out
