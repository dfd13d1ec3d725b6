"""Adam in one HIP launch per step (csrc/adam.hip), a drop-in for train.py's torch.optim.Adam.

train.py (:97-100) builds ``torch.optim.Adam(model.parameters(), lr=...)`` and steps it after every
batch.  torch's multi-tensor Adam walks the ~880 parameter tensors (145 M values of the learning
conf) in ~34 kernel launches and reaches ~2.9 TB/s: 1.39 ms of a 13.7 ms captured training step
(profiles/r5_train_step_breakdown_*.txt).  ``Adam`` keeps torch.optim.Adam's update, state names
(``exp_avg``, ``exp_avg_sq``, ``step``) and param-group options, and runs every tensor of a group
in ONE launch from a cached table of (p, grad, exp_avg, exp_avg_sq) pointers; when the gradient tensors
are new ones (zero_grad(set_to_none=True) between steps, or StaticTrainer's per-bucket gradients) only
their pointer column is rewritten (one small host-to-device copy).
Supported: fp32 CUDA parameters, amsgrad=False, maximize=False, a float lr (a Tensor lr raises: it
would need a host read per step); anything else raises (no fallback).  Parameters whose .grad is None
are skipped, as torch.optim.Adam skips them (frozen or unused parameters keep their state).
"""
import numpy as np
import torch

from . import _native


def _chunk_table(sizes, device):
    """gasfm_adam_chunk rows (tensor index, first value) for tensors of these sizes, on the device."""
    t = np.concatenate([np.stack([np.full(-(-n // _native.ADAM_CHUNK), i, np.int64),
                                  np.arange(0, n, _native.ADAM_CHUNK, dtype=np.int64)], 1) for i, n in enumerate(sizes)])
    rows = np.zeros((t.shape[0], 2), dtype=np.int64)  # (int32 tensor | int32 reserved), int64 begin
    rows[:, 0] = t[:, 0]
    rows[:, 1] = t[:, 1]
    return torch.from_numpy(rows).to(device)


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False,
                 maximize=False):
        if amsgrad or maximize:
            raise NotImplementedError("gasfm_amd.optim.Adam: amsgrad / maximize are not supported")
        if torch.is_tensor(lr):
            raise TypeError("gasfm_amd.optim.Adam: a Tensor lr is not supported (pass a float)")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"gasfm_amd.optim.Adam: lr={lr}, betas={betas}, eps={eps}")
        if not 0.0 <= weight_decay:
            raise ValueError(f"gasfm_amd.optim.Adam: invalid weight_decay value: {weight_decay}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._tables = {}

    def _build(self, ps, grads):
        """Validate the group, create missing state, build the device tables: gasfm_adam_tensor rows as
        int64 [n, 5] (p, g, m, v, numel) and the chunk table.  A later step whose gradient tensors are
        other tensors (p.grad = None between steps) only rewrites column 1 (``_regrad``)."""
        for p, g in zip(ps, grads):
            if not p.is_cuda or p.dtype != torch.float32 or p.is_sparse:
                raise TypeError("gasfm_amd.optim.Adam: fp32 dense CUDA parameters only")
            if not p.is_contiguous():
                raise TypeError("gasfm_amd.optim.Adam: contiguous parameters only")
        steps = {int(self.state[p]["step"]) for p in ps if self.state[p]}
        if len(steps) > 1:
            raise RuntimeError("gasfm_amd.optim.Adam: the parameters of a group are at different steps")
        step = torch.tensor(float(steps.pop() if steps else 0))  # ONE step counter shared by the group
        rows = []
        for p, g in zip(ps, grads):
            st = self.state[p]
            if "exp_avg" not in st:
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            st["step"] = step
            rows.append([p.data_ptr(), 0, st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(), p.numel()])
        dev = ps[0].device
        tensors = torch.tensor(rows, dtype=torch.int64).to(dev)
        chunks = _chunk_table([p.numel() for p in ps], dev)
        # the entry holds the tensors whose pointers it stores, so their ids stay theirs
        keep = (list(ps), [self.state[p]["exp_avg"] for p in ps], [self.state[p]["exp_avg_sq"] for p in ps])
        return {"tensors": tensors, "chunks": chunks, "n": chunks.shape[0], "step": step, "keep": keep,
                "grads": None}

    @staticmethod
    def _regrad(t, grads):
        """Point the table at this step's gradient tensors (one host-to-device copy of n pointers)."""
        for g in grads:
            if g is None or g.dtype != torch.float32 or g.is_sparse or not g.is_contiguous():
                raise TypeError("gasfm_amd.optim.Adam: dense contiguous fp32 gradients for every parameter")
        ptrs = torch.tensor([g.data_ptr() for g in grads], dtype=torch.int64)
        t["tensors"][:, 1].copy_(ptrs.pin_memory().to(t["tensors"].device, non_blocking=True))
        t["grads"] = list(grads)  # keeps them alive, and their ids for the next comparison

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
            if torch.is_tensor(group["lr"]):
                raise TypeError("gasfm_amd.optim.Adam: a Tensor lr is not supported (pass a float)")
            live = [p for p in group["params"] if p.grad is not None]  # torch skips grad-less params
            if not live:
                continue
            key = (gi, tuple(map(id, live)))
            tabs = self._tables.get(key)
            if tabs is None:
                # another subset of this group has gradients now: its cached tables' shared step
                # counters no longer describe every member, so they go; torch keeps one counter per
                # parameter, so the parameters are split by their current step (one launch each)
                for k in [k for k in self._tables if k[0] == gi]:
                    del self._tables[k]
                by_step = {}
                for p in live:
                    by_step.setdefault(int(self.state[p]["step"]) if self.state[p] else 0, []).append(p)
                tabs = [self._build(ps, [p.grad for p in ps]) for ps in by_step.values()]
                self._tables[key] = tabs
            for t in tabs:
                ps = t["keep"][0]
                grads = [p.grad for p in ps]
                if t["grads"] is None or any(a is not b for a, b in zip(grads, t["grads"])):
                    self._regrad(t, grads)
                t["step"] += 1  # in place: every parameter's state["step"]
                b1, b2 = group["betas"]
                _native.adam_step(t["tensors"], t["chunks"], t["n"], group["lr"], b1, b2, group["eps"],
                                  group["weight_decay"], int(t["step"]), ps[0])
                # the kernel wrote p in place behind autograd's back: bump the version counters, as an
                # in-place torch op would (version-keyed caches -- e.g. dense.weight_shadow's bf16
                # shadows -- see it)
                torch.autograd.graph.increment_version(ps)
        return loss
