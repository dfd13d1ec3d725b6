"""C-ABI library checks that need no GPU: load, exported symbols, host graph preprocessing."""
import os
import re

import numpy as np
import pytest
import torch

import gasfm_amd
from conftest import REPO, golden
from gasfm_amd import _native


def header_functions():
    text = open(os.path.join(REPO, "include", "gasfm.h")).read()
    return sorted(set(re.findall(r"\b(gasfm_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    lib = _native.lib()
    declared = header_functions()
    assert len(declared) >= 10
    for name in declared:
        assert hasattr(lib, name), f"{name} declared in include/gasfm.h but not exported"
    assert set(declared) == set(_native.exported_symbols())
    assert lib.gasfm_version() >= 1


def test_build_csr_matches_numpy_stable_sort():
    rng = np.random.default_rng(0)
    for n, E in ((1, 0), (1, 5), (50, 1000), (7, 3)):
        key = rng.integers(0, n, size=E).astype(np.int32)
        ptr, perm = _native.build_csr(key, n)
        ref_perm = np.argsort(key, kind="stable")
        np.testing.assert_array_equal(perm, ref_perm)
        np.testing.assert_array_equal(ptr, np.concatenate([[0], np.cumsum(np.bincount(key, minlength=n))]))


def test_build_csr_rejects_bad_keys():
    with pytest.raises(RuntimeError, match="outside"):
        _native.build_csr(np.array([0, 3], dtype=np.int32), 3)


def test_plan_work_splits_and_covers():
    rng = np.random.default_rng(1)
    lens = rng.integers(0, 40, size=100)
    lens[[3, 50]] = [1000, 257]
    ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    items, comb, n_slots = _native.plan_work(ptr, 32)
    covered = np.zeros(ptr[-1], dtype=np.int32)
    for s, b, e, slot in items:
        assert ptr[s] <= b <= e <= ptr[s + 1]
        assert e - b <= 32
        covered[b:e] += 1
        assert (slot >= 0) == (lens[s] > 32)
    assert (covered == 1).all()
    assert len(items) >= 100 and set(comb[:, 0]) == {i for i in range(100) if lens[i] > 32}
    assert comb[:, 2].sum() == n_slots
    # every segment, empty ones included, has exactly one item or one combine entry
    whole = {int(s) for s, b, e, slot in items if slot < 0}
    assert whole | set(comb[:, 0].tolist()) == set(range(100))


def test_plan_work_all_partial_slots():
    ptr = np.array([0, 3, 3, 10], dtype=np.int32)
    items, comb, n_slots = _native.plan_work(ptr, 4, all_partial=True)
    assert n_slots == 3 + 2  # one slot per segment + pieces of the split segment
    assert {int(i[3]) for i in items if i[0] != 2} == {0, 1}
    assert comb.tolist() == [[2, 3, 2, 1]]


def test_attn_plan_point_direction():
    s = golden("scene_config1.npz")
    idx = s["indices"]
    plan = gasfm_amd.AttnPlan.from_targets(idx[1], 200)
    assert plan.perm is not None
    perm = plan.perm.numpy()
    np.testing.assert_array_equal(idx[1][perm], np.sort(idx[1], kind="stable"))
    plan_c = gasfm_amd.AttnPlan.from_targets(idx[0], 10)
    assert plan_c.perm is None  # cam-major edges are already CSR


def test_state_dict_layout_matches_reference():
    f = golden("net_small.npz")
    ref_keys = {k[3:]: f[k].shape for k in f.files if k.startswith("sd/")}
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.conf.small_conf(2))
    ours = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    assert ours == {k: tuple(v) for k, v in ref_keys.items()}
    full = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf()).state_dict()
    assert len(full) == 886 and sum(v.numel() for v in full.values()) == 145_165_560
    assert sum(v.numel() for v in gasfm_amd.GraphAttnSfMNet(gasfm_amd.optim_conf()).state_dict().values()) \
        == 109_108_632


def test_compute_path_refuses_cpu_tensors():
    plan = gasfm_amd.AttnPlan.from_targets(np.array([0, 0, 1]), 2)
    XL = torch.randn(3, 32)
    with pytest.raises(TypeError, match="CUDA"):
        gasfm_amd.gat_attention(XL, torch.randn(2, 32), torch.randn(4, 8), torch.randn(32), plan, 4)


def test_conf_parser_roundtrip():
    text = """
    dataset { calibrated = true
      test_set = ["A" "B"] }
    model {
      type = "graph_attn_sfm.GraphAttnSfMNet"
      n_heads = 4
      view_head { enabled = true
        rot_representation = "quat" }
      depth_head.enabled = false
    }
    train.lr = 0.0001
    """
    c = gasfm_amd.Conf.parse_string(text)
    assert c.get_int("model.n_heads") == 4
    assert c.get_bool("model.view_head.enabled") is True
    assert c.get_bool("model.depth_head.enabled") is False
    assert c.get_string("model.view_head.rot_representation") == "quat"
    assert c.get("dataset.test_set") == ["A", "B"]
    assert abs(c.get_float("train.lr") - 1e-4) < 1e-12
    assert c.get_int("model.missing", default=None) is None


def test_device_plan_work_restatement_matches_host():
    """scene_device.plan_work_device (torch ops; runs on CPU tensors here) == gasfm_plan_work followed
    by attention._two_level, with the host scalars read by the function itself or passed in (from
    _piece_stats, or _piece_counts_host for host-known lengths)."""
    import torch
    from gasfm_amd.attention import _two_level
    from gasfm_amd.scene_device import _piece_counts_host, _piece_stats, plan_work_device
    rng = np.random.default_rng(0)
    n_two_level = 0
    for trial in range(160):
        N = int(rng.integers(0, 40))
        mp = int(rng.integers(1, 20))
        ap = bool(rng.integers(0, 2))
        ln = rng.integers(0, 3 if trial % 5 == 0 else (70 if trial % 3 else 400), size=N)
        ptr = np.concatenate([[0], np.cumsum(ln)]).astype(np.int32)
        items, comb, ns = _native.plan_work(ptr, mp, ap)
        top, l1 = _two_level(torch.from_numpy(comb.reshape(-1, 4)), ns)
        counts = _piece_counts_host([int(v) for v in ln], mp)
        assert counts == _piece_stats(torch.from_numpy(ln.astype(np.int64)), mp)[3].tolist()
        for cts in (None, counts):
            items2, top2, l12, ns2 = plan_work_device(torch.from_numpy(ptr), mp, ap, cts)
            assert ns == ns2
            np.testing.assert_array_equal(items.reshape(-1, 4), items2.numpy().reshape(-1, 4))
            np.testing.assert_array_equal(top.numpy().reshape(-1, 4), top2.numpy().reshape(-1, 4))
            assert (l1 is None) == (l12 is None)
            if l1 is not None:
                np.testing.assert_array_equal(l1.numpy(), l12.numpy())
        n_two_level += l1 is not None
    assert n_two_level > 10


def test_lazy_graph_wrappers_and_scene_csr():
    """SceneData built on the device carries a graph-wrapper builder instead of the wrappers
    (scene_device.scene_from_dense_device): the builder runs once, on first access, and before a
    .to() copy; loss.scene_csr reads the scene-build arrays until then, the plans afterwards."""
    import torch
    from gasfm_amd import SceneData, synthetic
    from gasfm_amd.loss import scene_csr
    sc = synthetic.scaled_config4(0.002, seed=1)
    host = SceneData.from_synthetic(sc)
    gw = host.graph_wrappers
    calls = []
    d = SceneData.__new__(SceneData)
    d.__dict__.update({k: v for k, v in host.__dict__.items() if k != "graph_wrappers"})
    pv, ps = gw["proj2view"].plan, gw["proj2scenepoint"].plan
    perm = ps.perm if ps.perm is not None else torch.arange(ps.num_edges, dtype=torch.int32)
    d._scene_build = {"cam_ptr": pv.seg_ptr, "pt_ptr": ps.seg_ptr, "perm": perm, "pos": ps.pos,
                      "pt": host.x.indices[1].to(torch.int32)}
    d._lazy_graph = lambda: calls.append(1) or gw
    caches, cam_ptr, pt_ptr, pt_perm = scene_csr(d)
    assert calls == [] and cam_ptr is pv.seg_ptr and pt_ptr is ps.seg_ptr and pt_perm is perm
    caches["x"] = 1
    assert scene_csr(d)[0] is caches  # one cache per source
    assert d.graph_wrappers is gw and calls == [1]
    assert d.graph_wrappers is gw and calls == [1]  # built once
    assert scene_csr(d)[1] is pv.seg_ptr  # from the plans now
    d2 = SceneData.__new__(SceneData)
    d2.__dict__.update(d.__dict__)
    d2.__dict__.pop("graph_wrappers")
    d2._lazy_graph = lambda: calls.append(2) or gw
    moved = d2.to("cpu")
    assert calls == [1, 2] and "_scene_build" not in moved.__dict__ and "_lazy_graph" not in moved.__dict__
    try:
        SceneData.__new__(SceneData).graph_wrappers
        raise AssertionError("expected AttributeError")
    except AttributeError:
        pass


def test_binding_arity_matches_header():
    """Every ctypes signature in _native._SIGS has as many parameters as its declaration in
    include/gasfm.h (a short argtypes list fails only at call time, on the GPU)."""
    import re
    text = re.sub(r"/\*.*?\*/", "", open(os.path.join(REPO, "include", "gasfm.h")).read(), flags=re.S)
    bad = []
    for m in re.finditer(r"\b(gasfm_\w+)\s*\(([^;{]*?)\)\s*;", text):
        name, args = m.group(1), m.group(2).strip()
        if name not in _native._SIGS:
            continue
        n = 0 if args in ("", "void") else args.count(",") + 1
        if n != len(_native._SIGS[name][1]):
            bad.append((name, n, len(_native._SIGS[name][1])))
    assert not bad, bad


def test_param_list_cache_follows_the_module_tree():
    """GraphAttnSfMNet._param_list (the forward's deferred-gradient check) is a cached list: it must
    follow a parameter replaced deep in the tree and a dtype / device conversion that creates new
    Parameter objects (torch's overwrite-on-conversion mode)."""
    import gasfm_amd
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=2))
    same = lambda: len(net._param_list()) == len(list(net.parameters())) and all(
        p is q for p, q in zip(net._param_list(), net.parameters()))
    assert same()
    net.equivariant_blocks[0].skip_projection.lin_proj.weight = torch.nn.Parameter(torch.zeros(32, 2))
    assert same()
    prev = torch.__future__.get_overwrite_module_params_on_conversion()
    torch.__future__.set_overwrite_module_params_on_conversion(True)
    try:
        net.double()
        assert same()
    finally:
        torch.__future__.set_overwrite_module_params_on_conversion(prev)
