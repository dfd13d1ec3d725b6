"""Adam in one HIP launch per step (csrc/adam.hip), a drop-in for train.py's torch.optim.Adam.

train.py (:97-100) builds ``torch.optim.Adam(model.parameters(), lr=...)`` and steps it after every
batch.  torch's multi-tensor Adam walks the ~880 parameter tensors (145 M values of the learning
conf) in ~34 kernel launches and reaches ~2.9 TB/s: 1.39 ms of a 13.7 ms captured training step
(profiles/r5_train_step_breakdown_*.txt).  ``Adam`` keeps torch.optim.Adam's update, state names
(``exp_avg``, ``exp_avg_sq``, ``step``) and param-group options, and runs every tensor of a group
in ONE launch from a cached table of (p, grad, exp_avg, exp_avg_sq) pointers, rebuilt only when a
parameter's gradient tensor changes (e.g. static_batch.StaticTrainer's per-bucket gradients).
Supported: fp32 CUDA parameters, amsgrad=False, maximize=False; anything else raises (no fallback).
"""
import ctypes

import torch

from . import _native


class _Tensor(ctypes.Structure):
    _fields_ = [("p", ctypes.c_void_p), ("g", ctypes.c_void_p), ("m", ctypes.c_void_p), ("v", ctypes.c_void_p),
                ("numel", ctypes.c_int64)]


class _Chunk(ctypes.Structure):
    _fields_ = [("tensor", ctypes.c_int32), ("reserved", ctypes.c_int32), ("begin", ctypes.c_int64)]


def _device_table(rows, ctype, device):
    arr = (ctype * len(rows))(*rows)
    host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
    return host.to(device)


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False,
                 maximize=False):
        if amsgrad or maximize:
            raise NotImplementedError("gasfm_amd.optim.Adam: amsgrad / maximize are not supported")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"gasfm_amd.optim.Adam: lr={lr}, betas={betas}, eps={eps}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._tables = {}

    def _build(self, ps, grads):
        """Validate the group, create missing state, build the device pointer tables."""
        for p, g in zip(ps, grads):
            if g is None:
                raise RuntimeError("gasfm_amd.optim.Adam: every parameter of a group needs a gradient "
                                   "(or none of them)")
            if not p.is_cuda or p.dtype != torch.float32 or g.dtype != torch.float32 or g.is_sparse:
                raise TypeError("gasfm_amd.optim.Adam: fp32 dense CUDA parameters and gradients only")
            if not (p.is_contiguous() and g.is_contiguous()):
                raise TypeError("gasfm_amd.optim.Adam: contiguous parameters and gradients only")
        steps = {int(self.state[p]["step"]) for p in ps if self.state[p]}
        if len(steps) > 1:
            raise RuntimeError("gasfm_amd.optim.Adam: the parameters of a group are at different steps")
        step = torch.tensor(float(steps.pop() if steps else 0))  # ONE step counter shared by the group
        tensors, chunks = [], []
        for i, (p, g) in enumerate(zip(ps, grads)):
            st = self.state[p]
            if "exp_avg" not in st:
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            st["step"] = step
            tensors.append(_Tensor(p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                                   p.numel()))
            chunks.extend(_Chunk(i, 0, b) for b in range(0, p.numel(), _native.ADAM_CHUNK))
        dev = ps[0].device
        # the entry holds the tensors whose pointers it stores, so the key's ids stay theirs
        keep = (list(ps), list(grads), [self.state[p]["exp_avg"] for p in ps], [self.state[p]["exp_avg_sq"] for p in ps])
        return (_device_table(tensors, _Tensor, dev), _device_table(chunks, _Chunk, dev), len(chunks), step, keep)

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._tables.clear()  # the moment buffers were replaced

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            ps = group["params"]
            grads = [p.grad for p in ps]
            if all(g is None for g in grads):
                continue
            # one dict lookup per step: the table of this exact set of (param, grad, moment) tensors
            key = (gi, tuple(map(id, ps)), tuple(map(id, grads)))
            t = self._tables.get(key)
            if t is None:
                t = self._build(ps, grads)
                if len(self._tables) > 64:
                    self._tables.clear()
                self._tables[key] = t
            tensors, chunks, n, step, _ = t
            step += 1  # in place: every parameter's state["step"]
            b1, b2 = group["betas"]
            _native.adam_step(tensors, chunks, n, group["lr"], b1, b2, group["eps"], group["weight_decay"],
                              int(step), ps[0])
        return loss
