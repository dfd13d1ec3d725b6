"""Import the reference's own model/graph code from /root/reference/code (build container only).

Used ONLY by tests/golden/make_golden.py to generate fixtures (and by optional
container-only tests that skip when /root/reference is absent).  Nothing is
copied: the reference modules are imported in place, read-only, with
PYTHONDONTWRITEBYTECODE so no bytecode is written into the mount.

Third-party packages the reference imports but that are absent offline are
replaced by stubs: torch_geometric (-> oracle.pyg_gatv2.GATv2Conv, the PyG
restatement), pytorch3d.transforms (quaternion_to_matrix restated from its
published formula; only baseNet.py:48 uses it), pyhocon, cv2, cvxpy, dask,
torch.utils.tensorboard (unused on the forward path).
"""
import math
import os
import sys
import types

REF_CODE = "/root/reference/code"


def _quaternion_to_matrix(q):
    # pytorch3d.transforms.quaternion_to_matrix, real part first (published formula).
    import torch
    r, i, j, k = torch.unbind(q, -1)
    two_s = 2.0 / (q * q).sum(-1)
    o = torch.stack((
        1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
        two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
        two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j),
    ), -1)
    return o.reshape(q.shape[:-1] + (3, 3))


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def available():
    return os.path.isdir(os.path.join(REF_CODE, "models"))


def load(gatv2_cls=None):
    """Return a namespace with the reference modules (graph_attn_sfm, layers, SceneData, ...)."""
    if not available():
        raise RuntimeError("reference not present")
    sys.dont_write_bytecode = True
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(os.path.dirname(here))
    if repo not in sys.path:
        sys.path.insert(0, repo)
    if gatv2_cls is None:
        from oracle.pyg_gatv2 import GATv2Conv as gatv2_cls
    tg = _stub("torch_geometric")
    tg.nn = _stub("torch_geometric.nn", GATv2Conv=gatv2_cls)
    p3 = _stub("pytorch3d")
    p3.transforms = _stub("pytorch3d.transforms", quaternion_to_matrix=_quaternion_to_matrix,
                          axis_angle_to_matrix=None, rotation_6d_to_matrix=None)

    class _ConfigTree(dict):
        pass

    _stub("pyhocon", ConfigFactory=None, HOCONConverter=None, ConfigTree=_ConfigTree)
    for name in ("cv2", "cvxpy"):
        _stub(name)
    dask = _stub("dask")
    dask.array = _stub("dask.array")
    _stub("torch.utils.tensorboard", SummaryWriter=object)
    # The reference has no __init__.py; its top-level names collide with installed packages
    # (HuggingFace `datasets`), so register the three source dirs as namespace packages.
    for pkg in ("datasets", "models", "utils"):
        m = types.ModuleType(pkg)
        m.__path__ = [os.path.join(REF_CODE, pkg)]
        sys.modules[pkg] = m
    if REF_CODE not in sys.path:
        sys.path.insert(0, REF_CODE)
    import importlib
    ns = types.SimpleNamespace()
    ns.graph_attn_sfm = importlib.import_module("models.graph_attn_sfm")
    ns.layers = importlib.import_module("models.layers")
    ns.SceneData = importlib.import_module("datasets.SceneData")
    ns.dataset_utils = importlib.import_module("utils.dataset_utils")
    ns.sparse_utils = importlib.import_module("utils.sparse_utils")
    ns.loss_functions = importlib.import_module("loss_functions")
    return ns


class DictConf:
    """Minimal pyhocon-like accessor (get_int/get_bool/get_string with default=)."""
    _MISSING = object()

    def __init__(self, d):
        self.d = d

    def _get(self, key, default):
        cur = self.d
        for part in key.split("."):
            if not isinstance(cur, dict) or part not in cur:
                if default is self._MISSING:
                    raise KeyError(key)
                return default
            cur = cur[part]
        return cur

    def get_int(self, key, default=_MISSING):
        v = self._get(key, default)
        return None if v is None else int(v)

    def get_float(self, key, default=_MISSING):
        v = self._get(key, default)
        return None if v is None else float(v)

    def get_bool(self, key, default=_MISSING):
        v = self._get(key, default)
        return None if v is None else bool(v)

    def get_string(self, key, default=_MISSING):
        v = self._get(key, default)
        return None if v is None else str(v)
