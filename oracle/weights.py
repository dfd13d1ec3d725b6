"""Deterministic per-key weights for reference-layout state_dicts — TEST INFRASTRUCTURE.

Lets fixtures of the full-width (145 M parameter) network be pinned without a
580 MB weight file: every tensor is drawn from numpy PCG64 seeded by the
crc32 of its state_dict key, so the same weights are regenerated anywhere.
Scales follow the usual inits (fan-in uniform for Linear, glorot for GATv2
att, ~1 for LayerNorm gains) so 12 blocks stay well conditioned.
"""
import math
import zlib

import numpy as np
import torch


def tensor_for(key, shape):
    rng = np.random.default_rng(zlib.crc32(key.encode()))
    u = rng.uniform(-1.0, 1.0, size=shape)
    if key.endswith(".att"):
        a = math.sqrt(6.0 / (shape[-2] + shape[-1]))
        return a * u
    if len(shape) == 2:  # Linear weight [out, in]
        return u / math.sqrt(shape[1])
    if key.endswith(".weight"):  # LayerNorm gain
        return 1.0 + 0.1 * u
    return 0.05 * u  # biases


def deterministic_state_dict(template, dtype=torch.float32):
    return {k: torch.from_numpy(tensor_for(k, tuple(v.shape))).to(dtype) for k, v in template.items()}


def probe_vector(key, n):
    """Regenerable U(-1, 1) vector r for gradient projections G @ r (fixtures of full-width nets)."""
    return np.random.default_rng(zlib.crc32(("probe/" + key).encode())).uniform(-1.0, 1.0, size=(n,))
