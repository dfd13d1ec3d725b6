"""torch-CPU restatement of PyG ``GATv2Conv`` — TEST INFRASTRUCTURE (oracle).

The reference does not vendor the op: it imports ``torch_geometric.nn.GATv2Conv``
(code/models/layers.py:4) and constructs it at layers.py:304-309 (proj2view),
401-406 (proj2scenepoint), 506-511 (view2global) and 521-526
(scenepoint2global), always with ``add_self_loops=False`` and PyG defaults for
everything else (concat=True, negative_slope=0.2, dropout=0.0, bias=True,
share_weights=False, edge_dim=None, aggr='add').  PyG is unpinned in
environment.yml:50 (``pyg::pyg``); the code comments name 2.2.0 as the current
release (train.py:236), so this follows the PyG 2.2 published algorithm:

    x_l = lin_l(x).view(-1, H, C)          # on ALL node rows (sources+targets)
    x_r = lin_r(x).view(-1, H, C)
    for edge j->i (edge_index[0]=j, edge_index[1]=i):
        z   = leaky_relu(x_r[i] + x_l[j], 0.2)
        e   = (z * att).sum(-1)            # [E, H]
    alpha = softmax(e, index=i)            # scatter-max, exp, scatter-sum, +1e-16
    out[i] = sum_j alpha[j] * x_l[j]       # scatter-add, zero for no in-edges
    out = out.view(-1, H*C) + bias

It is written in the same op sequence as PyG (materialised [E,H,C] tensors,
scatter reductions) so that it doubles as the "reference PyG CPU path" that
bench.py times as ``cpu_baseline`` (kind "port").
"""
import math

import torch
import torch.nn.functional as F


def _glorot_(t):
    # PyG inits.glorot: U(-a, a), a = sqrt(6 / (fan_rows + fan_cols)) over the last two dims.
    a = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-a, a)
    return t


def segment_softmax(e, index, num_nodes):
    """PyG ``utils.softmax(src, index, num_nodes=N)`` restated (index path, dim 0)."""
    H = e.shape[1]
    idx = index.view(-1, 1).expand(-1, H)
    emax = torch.zeros((num_nodes, H), dtype=e.dtype).scatter_reduce(
        0, idx, e.detach(), reduce="amax", include_self=False)
    ex = (e - emax.index_select(0, index)).exp()
    esum = torch.zeros((num_nodes, H), dtype=e.dtype).scatter_add(0, idx, ex)
    return ex / (esum.index_select(0, index) + 1e-16)


class GATv2Conv(torch.nn.Module):
    """Drop-in CPU stand-in for ``torch_geometric.nn.GATv2Conv`` (subset used by GASFM)."""

    def __init__(self, in_channels, out_channels, heads=1, concat=True,
                 negative_slope=0.2, dropout=0.0, add_self_loops=True,
                 edge_dim=None, fill_value="mean", bias=True,
                 share_weights=False, **kwargs):
        super().__init__()
        if add_self_loops or edge_dim is not None or share_weights or not concat or dropout != 0.0:
            raise NotImplementedError("GASFM only uses add_self_loops=False, concat, no edge_dim/dropout")
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.heads = heads
        self.negative_slope = negative_slope
        self.lin_l = torch.nn.Linear(in_channels, heads * out_channels, bias=bias)
        self.lin_r = torch.nn.Linear(in_channels, heads * out_channels, bias=bias)
        self.att = torch.nn.Parameter(torch.empty(1, heads, out_channels))
        self.bias = torch.nn.Parameter(torch.empty(heads * out_channels)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        _glorot_(self.lin_l.weight)
        _glorot_(self.lin_r.weight)
        for lin in (self.lin_l, self.lin_r):
            if lin.bias is not None:
                torch.nn.init.zeros_(lin.bias)
        _glorot_(self.att)
        if self.bias is not None:
            torch.nn.init.zeros_(self.bias)

    def forward(self, x, edge_index):
        H, C = self.heads, self.out_channels
        N = x.shape[0]
        x_l = self.lin_l(x).view(-1, H, C)
        x_r = self.lin_r(x).view(-1, H, C)
        src, dst = edge_index[0], edge_index[1]
        x_j = x_l.index_select(0, src)
        x_i = x_r.index_select(0, dst)
        z = F.leaky_relu(x_i + x_j, self.negative_slope)
        e = (z * self.att).sum(dim=-1)
        alpha = segment_softmax(e, dst, N)
        msg = x_j * alpha.unsqueeze(-1)
        out = torch.zeros((N, H, C), dtype=x.dtype).index_add(0, dst, msg)
        out = out.view(N, H * C)
        if self.bias is not None:
            out = out + self.bias
        return out


def gatv2_segment_reference(XL, XR, att, bias, dst, num_targets, negative_slope=0.2):
    """Kernel-level oracle: the attention part of GATv2Conv on pre-projected inputs.

    XL [E, H, C] (already lin_l'd source rows, one per edge), XR [N, H, C] (lin_r'd
    target rows), att [H, C], bias [H*C], dst [E] target of each edge.
    Returns out [N, H*C], seg_max [N, H], seg_sum [N, H] (sum of exp(e - max), no
    epsilon) — the same quantities the HIP kernel returns, in the PyG op sequence.
    """
    E, H, C = XL.shape
    z = F.leaky_relu(XR.index_select(0, dst) + XL, negative_slope)
    e = (z * att.view(1, H, C)).sum(-1)
    idx = dst.view(-1, 1).expand(-1, H)
    dev = XL.device  # the checker may run on the device in fp64 at full config-4 size
    emax = torch.full((num_targets, H), -math.inf, dtype=XL.dtype, device=dev).scatter_reduce(
        0, idx, e.detach(), reduce="amax", include_self=True)
    emax_g = emax.index_select(0, dst)
    ex = (e - emax_g).exp()
    esum = torch.zeros((num_targets, H), dtype=XL.dtype, device=dev).scatter_add(0, idx, ex)
    alpha = ex / (esum.index_select(0, dst) + 1e-16)
    out = torch.zeros((num_targets, H, C), dtype=XL.dtype, device=dev).index_add(0, dst, XL * alpha.unsqueeze(-1))
    out = out.view(num_targets, H * C) + bias
    return out, emax, esum
