"""CPU oracle for the GASFM GAT stack — TEST INFRASTRUCTURE ONLY.

Nothing in ``gasfm_amd/`` may import this package. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it,
and only as the checker / the timed CPU baseline, never as a product path.

Contents
--------
pyg_gatv2     torch-CPU restatement of PyG ``GATv2Conv`` (the third-party op the
              reference calls at code/models/layers.py:329-335, 426-432,
              550-556, 566-572), in the PyG op sequence (both linears on all
              E+N rows, index_select, scatter-max, exp, scatter-sum, index_add).
gasfm_ref     functional fp64/fp32 restatement of ``GraphAttnSfMNet.forward``
              (code/models/graph_attn_sfm.py:117-185 and the layers it calls),
              driven directly by a reference-layout state_dict.
esfm_loss     dense fp64 restatement of ESFMLoss (code/loss_functions.py:85-123, including
              its gradient hook) and the same on the E observed pairs only.
scenes        synthetic scene generators for BASELINE configs 1 and 4 and the
              CPU graph build (M2sparse, dataset_utils.py:116-156).

Parity pinning: ``tests/golden/`` holds fixtures produced by importing the
reference's own model/graph code from /root/reference/code in the build
container (``tests/golden/make_golden.py``) with ``pyg_gatv2.GATv2Conv``
injected as ``torch_geometric.nn.GATv2Conv``.  PyG itself is absent offline, so
the PyG op is pinned by its published algorithm plus the PyG-free identities
listed in SURVEY.md §8(c) (att=0 -> SparseMat.mean, single-edge segments,
permutation invariance, empty segment -> bias); the rest of the model is
pinned against the reference's own code.
"""
