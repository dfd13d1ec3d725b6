"""``GATv2Conv`` for MI355X: PyG-compatible parameters, fused HIP attention.

Drop-in for ``torch_geometric.nn.GATv2Conv`` as the reference constructs it
(code/models/layers.py:304-309, 401-406, 506-511, 521-526: concat=True,
negative_slope=0.2, dropout=0, bias=True, share_weights=False, no edge_dim,
add_self_loops=False).  Parameter names/shapes match PyG exactly
(``lin_l.{weight,bias}`` [H*C, F_in], ``lin_r.*``, ``att`` [1, H, C],
``bias`` [H*C]) so reference state_dicts load unchanged.

Two call forms:
  forward(x, edge_index)   the PyG call used by the reference layer code
                           (generic graphs; plan cached on the edge_index tensor)
  attend(x_src, x_tgt, plan)  the MI355X fast path used by gasfm_amd.model:
                           lin_l on source rows only, lin_r on target rows only
                           (PyG computes both on all E+N rows), then the fused
                           edge-softmax + aggregation kernel.
"""
import math

import torch
import torch.nn.functional as F

from . import dense
from .attention import AttnPlan, gat_attention


def _glorot_(t):
    a = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-a, a)



class ZeroTargetRowsFn(torch.autograd.Function):
    """lin_r applied to the reference's zero target features (dataset_utils.py:569-571), broadcast
    over n targets: lin_r(0) == lin_r.bias exactly.  Backward: the bias gradient is the column sum
    of the targets' gradient, deferred into the end-of-backward batched parameter sums (aten ran a
    one-workgroup reduce over the n rows, 21 us for a 25k-point shard, plus a GEMM and a reduce for
    the zero row); the weight gets its zero gradient, as in the reference."""

    @staticmethod
    def forward(ctx, W, b, n):
        from . import _native
        ctx.w_shape = W.shape
        ctx.defer = _native.defer_token(b)
        # a fresh row, broadcast: the output must not alias the bias parameter (a later in-place
        # optimizer step would trip the saved-tensor version checks of its consumers)
        return b.detach().view(1, -1).clone().expand(n, -1)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        return torch.zeros(ctx.w_shape, dtype=g.dtype, device=g.device), dense.bias_colsum(g, ctx.defer), None


def zero_target_rows(lin_r, n, like):
    """XR of n targets whose features are the reference's zeros: lin_r(0) broadcast."""
    if (like.is_cuda and lin_r.bias is not None and lin_r.bias.dtype == torch.float32 and torch.is_grad_enabled()
            and n > 0):
        return ZeroTargetRowsFn.apply(lin_r.weight, lin_r.bias, n)
    zero = torch.zeros((1, lin_r.in_features), dtype=like.dtype, device=like.device)
    return lin_r(zero).expand(n, -1)

class GATv2Conv(torch.nn.Module):
    def __init__(self, in_channels, out_channels, heads=1, concat=True, negative_slope=0.2, dropout=0.0,
                 add_self_loops=True, edge_dim=None, fill_value="mean", bias=True, share_weights=False,
                 **kwargs):
        super().__init__()
        if add_self_loops:
            raise NotImplementedError("GATv2Conv(add_self_loops=True): GASFM builds its star graphs without "
                                      "self loops (layers.py:308); not supported by the MI355X kernel")
        if not concat or dropout != 0.0 or edge_dim is not None or share_weights:
            raise NotImplementedError("only concat=True, dropout=0, edge_dim=None, share_weights=False")
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.heads = heads
        self.negative_slope = float(negative_slope)
        self.lin_l = torch.nn.Linear(in_channels, heads * out_channels, bias=bias)
        self.lin_r = torch.nn.Linear(in_channels, heads * out_channels, bias=bias)
        self.att = torch.nn.Parameter(torch.empty(1, heads, out_channels))
        if bias:
            self.bias = torch.nn.Parameter(torch.empty(heads * out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        # PyG: glorot weights, zero biases, glorot att, zero bias
        _glorot_(self.lin_l.weight)
        _glorot_(self.lin_r.weight)
        for lin in (self.lin_l, self.lin_r):
            if lin.bias is not None:
                torch.nn.init.zeros_(lin.bias)
        _glorot_(self.att)
        if self.bias is not None:
            torch.nn.init.zeros_(self.bias)

    def _bias(self, ref):
        if self.bias is not None:
            return self.bias
        return torch.zeros(self.heads * self.out_channels, dtype=ref.dtype, device=ref.device)

    # ------------------------------------------------------------------ fast path
    def attend(self, x_src, x_tgt, plan):
        """Attention of plan's destinations over source rows.

        x_src [S, F_in]: source node features (rows addressed by plan.perm or edge order)
        x_tgt [N, F_in] target node features, or None for the reference's zero target
              features (dataset_utils.py:569-571), where lin_r(0) == lin_r.bias.
        """
        XL = dense.linear(x_src, self.lin_l)
        if x_tgt is None:
            # one zero row through lin_r (== its bias) broadcast over the targets: lin_r.weight
            # still receives its (zero) gradient, as in the reference, so train.py:137's
            # torch.cat over every p.grad keeps working.
            XR = zero_target_rows(self.lin_r, plan.num_targets, x_src)
        else:
            XR = dense.linear(x_tgt, self.lin_r)
        return gat_attention(XL, XR, self.att, self._bias(XL), plan, self.heads, self.negative_slope)

    # ------------------------------------------------------------------ PyG call form
    def _plan_for(self, edge_index, num_nodes):
        """The attention plan of this edge_index TENSOR, cached on the tensor object itself (so a
        new edge_index that the caching allocator places at a freed tensor's address never finds
        that tensor's plan) and keyed on its version (an in-place edit rebuilds it)."""
        key = (edge_index._version, int(num_nodes), tuple(edge_index.shape))
        cached = getattr(edge_index, "_gasfm_plan", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        src, dst = edge_index[0].cpu(), edge_index[1].cpu()
        unique_src = src.numel() == 0 or int(torch.bincount(src).max()) <= 1
        if unique_src:
            plan = AttnPlan.from_targets(dst, num_nodes, src=src, src_rows=num_nodes).to(edge_index.device)
            plan.gather_src = None
        else:
            # repeated sources: gather per-edge source rows first (edge order == plan order)
            plan = AttnPlan.from_targets(dst, num_nodes).to(edge_index.device)
            plan.gather_src = src.to(edge_index.device)
        edge_index._gasfm_plan = (key, plan)
        return plan

    def forward(self, x, edge_index):
        N = x.shape[0]
        plan = self._plan_for(edge_index, N)
        XL = self.lin_l(x)
        XR = self.lin_r(x)
        if plan.gather_src is not None:
            XL = XL.index_select(0, plan.gather_src)
        return gat_attention(XL, XR, self.att, self._bias(XL), plan, self.heads, self.negative_slope)
