"""gasfm_amd — MI355X-native GASFM graph-attention hot path.

Drop-in replacement for the reference's ``models.graph_attn_sfm.GraphAttnSfMNet``
(same constructor, forward(data) and state_dict) and for
``torch_geometric.nn.GATv2Conv`` as GASFM uses it, with the edge-softmax +
aggregation (and backward) in hand-written HIP for gfx950 (gasfm_amd/csrc).
"""
from .attention import AttnPlan, gat_attention  # noqa: F401
from .conf import Conf, learning_conf, optim_conf  # noqa: F401
from .gatv2 import GATv2Conv  # noqa: F401
from .loss import ESFMLoss  # noqa: F401
from .model import GraphAttnSfMNet  # noqa: F401
from .ba import euc_ba, proj_ba  # noqa: F401
from .outliers import OutlierInjector, inject_outliers  # noqa: F401
from .scene import AxialAggregationGraphWrapper, SceneData, SparseMat, M2sparse  # noqa: F401
from .optim import Adam  # noqa: F401
from .static_batch import StaticTrainer  # noqa: F401

__all__ = ["AttnPlan", "gat_attention", "Conf", "learning_conf", "optim_conf", "GATv2Conv", "ESFMLoss", "GraphAttnSfMNet",
           "AxialAggregationGraphWrapper", "SceneData", "SparseMat", "M2sparse",
           "OutlierInjector", "inject_outliers", "euc_ba", "proj_ba", "Adam", "StaticTrainer"]
