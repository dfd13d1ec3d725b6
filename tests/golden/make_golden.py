"""Generate the golden fixtures in tests/golden/*.npz from the REFERENCE's own code.

Run in the build container only (needs /root/reference):
    python tests/golden/make_golden.py

The reference's model/graph modules (models/graph_attn_sfm.py, models/layers.py,
datasets/SceneData.py, utils/dataset_utils.py, utils/sparse_utils.py) are
imported in place via tests/golden/refimport.py, with PyG's GATv2Conv (absent
offline) supplied by oracle/pyg_gatv2.py.  Everything runs in float64 unless
noted.  Outputs are data only (inputs, weights, outputs, gradients).

Fixtures
  scene_config1.npz       config-1 scene as the reference SceneData builds it:
                          M, Ns, x.values/indices, the four edge_index tensors,
                          valid view / point ids.
  conv_<F>_<H>_<C>_<g>.npz one GATv2Conv call inside the reference wrapper code
                          (generate_node_features -> conv -> extract_target_node_features)
                          for (F,H,C) in (2,4,1) (32,4,8) (64,4,16) (1024,4,256):
                          node features, edge_index, params, out, dOut, grads.
  conv_identity_mean.npz  att = 0 known answer: the reference's PyG-free
                          SparseMat.mean (sparse_utils.py:414-419) of XL, + bias.
  net_small.npz           2-block reduced-width net (view 64, global 128), reference
                          init (seed 0): state_dict, outputs, parameter grads of a
                          fixed linear loss.
  net_learning12.npz / net_optim9.npz  full-width nets (12 / 9 blocks), weights
                          from oracle/weights.py, outputs only (fp64 and fp32 runs).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import refimport  # noqa: E402
from gasfm_amd import synthetic  # noqa: E402  (input generation only)
from oracle.pyg_gatv2 import GATv2Conv as OracleGATv2Conv  # noqa: E402
from oracle.weights import deterministic_state_dict, tensor_for  # noqa: E402

torch.set_grad_enabled(True)


def conf_dict(num_layers, view, glob):
    return refimport.DictConf({"dataset": {"calibrated": True}, "model": {
        "type": "graph_attn_sfm.GraphAttnSfMNet", "n_heads": 4, "stateful_global_features": True,
        "global2view_and_global2scenepoint_enabled": False, "n_feat_proj": 32, "n_feat_scenepoint": 64,
        "n_feat_view": view, "n_feat_global": glob, "num_layers": num_layers,
        "n_hidden_layers_scenepoint_update": 0, "n_hidden_layers_view_update": 0,
        "n_hidden_layers_global_update": 0, "n_hidden_layers_proj_update": 0, "use_norm_proj_update": True,
        "add_residual_skipconn_proj_update": True, "add_skipconn_from_init_projfeat": True,
        "pos_emb_n_freq": 0, "depth_head": {"enabled": False},
        "view_head": {"enabled": True, "n_hidden_layers": 2, "rot_representation": "quat"},
        "scenepoint_head": {"enabled": True, "n_hidden_layers": 2}}})


def build_scene(ref):
    sc = synthetic.config1()
    M = torch.from_numpy(sc.dense_M())
    Ns = torch.from_numpy(sc.Ns())
    Ps = torch.from_numpy(sc.Ps_gt())
    data = ref.SceneData.SceneData(M, Ns, Ps, "synthetic_config1", calibrated=True)
    return sc, data


def to_double_scene(data):
    data.x.values = data.x.values.double()
    return data


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v))
                                 for k, v in arrays.items()})
    print("wrote", path, sum(np.asarray(v).size if not torch.is_tensor(v) else v.numel() for v in arrays.values()))


def scene_fixture(data, M, Ns):
    gw = data.graph_wrappers
    save("scene_config1.npz", M=M, Ns=Ns, values=data.x.values.float(), indices=data.x.indices,
         cam_per_pts=data.x.cam_per_pts, pts_per_cam=data.x.pts_per_cam,
         p2v_edge_index=gw["proj2view"].edge_index, p2s_edge_index=gw["proj2scenepoint"].edge_index,
         v2g_edge_index=gw["view2global"].edge_index, s2g_edge_index=gw["scenepoint2global"].edge_index,
         valid_views=gw["view2global"].valid_indices[0], valid_pts=gw["scenepoint2global"].valid_indices[1])


def conv_fixture(wrapper, F_in, H, C, tag, src_feats, x_agg, seed):
    torch.manual_seed(seed)
    conv = OracleGATv2Conv(F_in, C, heads=H, add_self_loops=False).double()
    big = F_in * H * C > 100_000
    with torch.no_grad():  # non-trivial biases / att so every term is exercised
        conv.lin_l.bias.uniform_(-0.2, 0.2)
        conv.lin_r.bias.uniform_(-0.2, 0.2)
        conv.bias.uniform_(-0.2, 0.2)
        if big:  # regenerable weights (oracle.weights) instead of storing 2 x 8 MB matrices
            for k in ("lin_l.weight", "lin_r.weight"):
                w = torch.from_numpy(tensor_for(f"conv_{tag}.{k}", tuple(conv.get_parameter(k).shape)))
                conv.get_parameter(k).copy_(w)
    x = wrapper.generate_node_features(src_feats, x_agg=x_agg).detach().double().requires_grad_(True)
    out_all = conv(x, wrapper.edge_index)
    out = wrapper.extract_target_node_features(out_all).reshape(-1, H * C)
    g = torch.randn(out.shape, dtype=torch.float64)
    (out * g).sum().backward()
    name = f"conv_{F_in}_{H}_{C}_{tag}.npz"
    arrays = dict(x=x, edge_index=wrapper.edge_index, num_targets=out.shape[0], lin_l_b=conv.lin_l.bias,
                  lin_r_b=conv.lin_r.bias, att=conv.att, bias=conv.bias, out=out, gout=g, dx=x.grad,
                  d_lin_l_b=conv.lin_l.bias.grad, d_lin_r_b=conv.lin_r.bias.grad, d_att=conv.att.grad,
                  d_bias=conv.bias.grad)
    if big:  # weight grads as checksums: dW @ r for a stored random r
        r = torch.randn(F_in, dtype=torch.float64)
        arrays.update(weights_key=f"conv_{tag}", r=r, d_lin_l_w_r=conv.lin_l.weight.grad @ r,
                      d_lin_r_w_r=conv.lin_r.weight.grad @ r)
    else:
        arrays.update(lin_l_w=conv.lin_l.weight, lin_r_w=conv.lin_r.weight, d_lin_l_w=conv.lin_l.weight.grad,
                      d_lin_r_w=conv.lin_r.weight.grad)
    save(name, **arrays)
    return conv


def identity_mean_fixture(ref, data):
    """att = 0 -> uniform alpha -> out = mean of XL over the segment + bias (PyG-free known answer)."""
    torch.manual_seed(5)
    F_in, H, C = 32, 4, 8
    E = data.x.values.shape[0]
    feats = torch.randn(E, F_in, dtype=torch.float64)
    Wl = torch.randn(H * C, F_in, dtype=torch.float64) * 0.2
    bl = torch.randn(H * C, dtype=torch.float64) * 0.1
    bias = torch.randn(H * C, dtype=torch.float64) * 0.1
    XL = feats @ Wl.T + bl
    sm = ref.sparse_utils.SparseMat(XL, data.x.indices, data.x.cam_per_pts, data.x.pts_per_cam,
                                    (data.x.shape[0], data.x.shape[1], H * C))
    torch.set_default_dtype(torch.float64)  # SparseMat.sum allocates with the default dtype
    try:
        pt_mean = sm.mean(dim=0) + bias   # reference SparseMat.mean over cameras -> per point
        cam_mean = sm.mean(dim=1) + bias  # per camera
    finally:
        torch.set_default_dtype(torch.float32)
    save("conv_identity_mean.npz", feats=feats, lin_l_w=Wl, lin_l_b=bl, bias=bias, pt_out=pt_mean,
         cam_out=cam_mean, indices=data.x.indices)


def net_run(ref, data, conf, sd=None, dtype=torch.float64, grads=False, seed=0):
    torch.manual_seed(seed)
    net = ref.graph_attn_sfm.GraphAttnSfMNet(conf).to(dtype)
    if sd is not None:
        net.load_state_dict(sd)  # after .to(dtype): fp64 weights stay fp64
    d = data
    d.x.values = d.x.values.to(dtype)
    pred = net(d)
    out = {"Ps_norm": pred["Ps_norm"], "pts3D": pred["pts3D"]}
    if grads:
        g = torch.Generator().manual_seed(7)
        cP = torch.randn(pred["Ps_norm"].shape, generator=g, dtype=dtype)
        cX = torch.randn(pred["pts3D"].shape, generator=g, dtype=dtype)
        loss = (pred["Ps_norm"] * cP).sum() + (pred["pts3D"] * cX).sum()
        loss.backward()
        out["cP"], out["cX"] = cP, cX
        out["grads"] = {k: p.grad for k, p in net.named_parameters()}
    return net, out


def main():
    ref = refimport.load(OracleGATv2Conv)
    sc, data = build_scene(ref)
    scene_fixture(data, torch.from_numpy(sc.dense_M()), torch.from_numpy(sc.Ns()))
    gw = data.graph_wrappers
    x_coo = data.x.to_torch_hybrid_sparse_coo()
    m, n = data.x.shape[0], data.x.shape[1]
    E = data.x.values.shape[0]
    torch.manual_seed(1)

    # (2,4,1): block-0 style point direction, zero target features
    xs2 = torch.sparse_coo_tensor(x_coo.indices(), torch.randn(E, 2, dtype=torch.float64), (m, n, 2)).coalesce()
    conv_fixture(gw["proj2scenepoint"], 2, 4, 1, "p2s", xs2, None, seed=11)
    conv_fixture(gw["proj2view"], 2, 4, 1, "p2v", xs2, None, seed=12)
    # (32,4,8): blocks >= 1, both directions, stateful target features
    xs32 = torch.sparse_coo_tensor(x_coo.indices(), torch.randn(E, 32, dtype=torch.float64), (m, n, 32)).coalesce()
    conv_fixture(gw["proj2scenepoint"], 32, 4, 8, "p2s", xs32, torch.randn(n, 32, dtype=torch.float64), seed=13)
    conv_fixture(gw["proj2view"], 32, 4, 8, "p2v", xs32, torch.randn(m, 32, dtype=torch.float64), seed=14)
    # (64,4,16): scenepoint -> global over the valid points
    v = gw["scenepoint2global"].valid_indices
    pf = torch.randn(1, n, 64, dtype=torch.float64)
    xs64 = torch.sparse_coo_tensor(v, pf[v[0], v[1], :], (1, n, 64)).coalesce()
    conv_fixture(gw["scenepoint2global"], 64, 4, 16, "s2g", xs64, torch.randn(1, 64, dtype=torch.float64), seed=15)
    # (1024,4,256): view -> global over the valid views
    v = gw["view2global"].valid_indices
    vf = torch.randn(m, 1, 1024, dtype=torch.float64)
    xs1024 = torch.sparse_coo_tensor(v, vf[v[0], v[1], :], (m, 1, 1024)).coalesce()
    conv_fixture(gw["view2global"], 1024, 4, 256, "v2g", xs1024, torch.randn(1, 1024, dtype=torch.float64),
                 seed=16)
    identity_mean_fixture(ref, data)

    # reduced-width 2-block net, reference init, fp64 with grads
    conf_s = conf_dict(2, 64, 128)
    _, data = build_scene(ref)
    net, out = net_run(ref, data, conf_s, dtype=torch.float64, grads=True, seed=0)
    sd = {f"sd/{k}": v for k, v in net.state_dict().items()}
    gr = {f"grad/{k}": v for k, v in out["grads"].items()}
    save("net_small.npz", Ps_norm=out["Ps_norm"], pts3D=out["pts3D"], cP=out["cP"], cX=out["cX"], **sd, **gr)

    # full-width nets, deterministic weights, outputs in fp64 and fp32
    for tag, L in (("learning12", 12), ("optim9", 9)):
        conf_f = conf_dict(L, 1024, 2048)
        torch.manual_seed(0)
        template = ref.graph_attn_sfm.GraphAttnSfMNet(conf_f).state_dict()
        sdw = deterministic_state_dict(template, torch.float64)
        _, data = build_scene(ref)
        with torch.no_grad():
            _, o64 = net_run(ref, data, conf_f, sd=sdw, dtype=torch.float64)
        _, data = build_scene(ref)
        with torch.no_grad():
            _, o32 = net_run(ref, data, conf_f, sd={k: v.float() for k, v in sdw.items()}, dtype=torch.float32)
        save(f"net_{tag}.npz", Ps_norm=o64["Ps_norm"], pts3D=o64["pts3D"], Ps_norm_fp32=o32["Ps_norm"],
             pts3D_fp32=o32["pts3D"])


if __name__ == "__main__":
    main()
