"""Per-edge (E-row) operations of a GASFM block.

layer_norm_relu      ReLU(LayerNorm(P)) on E x F projection features
                     (layers.py:232-234, 972-984)
projection_update    (lin_proj(x_e) + sp[pt_e] + sv[cam_e] + sg) / 4
                     (GraphAttnSfMProjectionFeatureUpdate.forward, layers.py:927-945)
"""
import torch
import torch.nn.functional as F


def layer_norm_relu(P, ln):
    return F.relu(F.layer_norm(P, ln.normalized_shape, ln.weight, ln.bias, ln.eps))


def projection_update(x, lin_proj, sp, sv, sg, edges):
    y = F.linear(x, lin_proj.weight, lin_proj.bias)
    y = y + sp.index_select(0, edges.pt) + sv.index_select(0, edges.cam) + sg
    return y / 4
