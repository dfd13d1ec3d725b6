"""Host side of gasfm_amd.optim.Adam (no GPU): the chunk table matches gasfm_adam_chunk's layout
(int32 tensor index, int32 reserved, int64 first value) and covers every value of every tensor once
in GASFM_ADAM_CHUNK steps; the unsupported options raise."""
import ctypes

import numpy as np
import pytest
import torch

from gasfm_amd import _native
from gasfm_amd.optim import Adam, _chunk_table


class _Chunk(ctypes.Structure):  # gasfm_adam_chunk (include/gasfm.h)
    _fields_ = [("tensor", ctypes.c_int32), ("reserved", ctypes.c_int32), ("begin", ctypes.c_int64)]


def test_chunk_table_layout_and_coverage():
    sizes = [1, 4096, 4097, 3 * 4096 + 5, 33]
    t = _chunk_table(sizes, torch.device("cpu"))
    assert t.dtype == torch.int64 and t.shape[1] == 2
    raw = t.numpy().tobytes()
    rows = (_Chunk * t.shape[0]).from_buffer_copy(raw)
    C = _native.ADAM_CHUNK
    seen = {i: [] for i in range(len(sizes))}
    for r in rows:
        assert r.reserved == 0
        seen[r.tensor].append(r.begin)
    for i, n in enumerate(sizes):
        assert seen[i] == list(range(0, n, C)), i
    assert t.shape[0] == sum(-(-n // C) for n in sizes)
    assert ctypes.sizeof(_Chunk) == 16


def test_adam_rejects_options():
    p = torch.zeros(3, requires_grad=True)
    with pytest.raises(NotImplementedError):
        Adam([p], amsgrad=True)
    with pytest.raises(ValueError):
        Adam([p], betas=(1.0, 0.999))
    with pytest.raises(ValueError):
        Adam([p], weight_decay=-1e-4)  # torch.optim.Adam rejects it too
    with pytest.raises(TypeError):
        Adam([p], lr=torch.tensor(1e-3))  # a Tensor lr would need a host read per step
