"""Whole-step HIP graph capture: one graph launch per forward+backward.

A GASFM step issues ~2,700 kernel launches (12 blocks of attention, edge, node and dense
camera/global work, forward and backward).  Issued eagerly through Python and autograd, the
host needs ~47 ms per step to enqueue them, as long as the GPU needs to run them at config 4,
and far longer than the GPU needs at the per-rank size of an 8-GPU run (measured by
tools/step_overhead.py).  Capturing the step once (torch.cuda.CUDAGraph = hipGraph on ROCm)
and replaying it removes the host cost and the per-launch gaps.

Requirements, all met by the GASFM path: fixed shapes per scene (plans are built once and
cached), no host synchronisation inside forward/backward (plan building happens in the warm-up
steps), every HIP kernel launched on torch's current stream (libgasfm's launches take
torch.cuda.current_stream()), and RCCL collectives captured by torch's ProcessGroupNCCL.

Usage::

    def fwd_bwd():                 # returns the loss; leaves gradients in p.grad
        loss = loss_fn(model(data))
        loss.backward()
        return loss
    step = CapturedStep(fwd_bwd, params=model.parameters())
    loss = step()                  # replays the graph; p.grad holds this step's gradients

After each replay every parameter's ``.grad`` is (re)set to the tensor the graph writes, so
``optimizer.zero_grad()`` between steps is harmless; a replay does not accumulate into an
existing gradient (each replay's gradients are that step's alone, as after zero_grad + backward).
"""
import contextlib
import gc

import torch


@contextlib.contextmanager
def gc_paused():
    """Python's cyclic garbage collector off for the duration (a stream capture).  A collection
    that runs mid-capture finalises whatever cyclic garbage is pending, e.g. an earlier step's
    CUDAGraph, whose hipGraphExecDestroy on the capturing thread is refused under
    capture_error_mode="thread_local" and aborts the process from the destructor (seen once in
    the GPU suite, round 6).  torch.cuda.graph collects before it begins capturing; this keeps
    the collector from running again until the capture has ended."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def retire_collectives():
    """Block until ProcessGroupNCCL's watchdog has retired every collective issued so far.

    The watchdog thread keeps each eager collective's Work on a list and polls its end event
    (hipEventQuery, every 100 ms) until it sees it complete.  A camera-sharded step issues
    asynchronous all-reduces (distributed.AsyncGradReducer) on the process group's internal RCCL
    stream; inside the capture that same stream joins the graph.  A watchdog poll of a warm-up
    Work's end event -- recorded on that stream before the capture -- that lands while the
    stream is capturing fails, and the watchdog rethrows it (SIGABRT from
    ProcessGroupNCCL.cpp's Watchdog::run).  Whether a poll hit that window was timing: ~1 capture
    in 10.  After torch.cuda.synchronize() every Work has completed, so the watchdog empties its
    list on its next poll; ``_wait_for_pending_works`` returns once the list is empty.  Works
    created during a capture are never listed, so nothing is polled until the capture ends."""
    dist = torch.distributed
    if not (dist.is_available() and dist.is_initialized()):
        return
    for pg in _process_groups():
        try:
            nccl = dist.get_backend(pg) == "nccl"
        except (RuntimeError, ValueError):
            nccl = False
        if nccl:
            wait = getattr(pg, "_wait_for_pending_works", None)
            if wait is None:
                raise RuntimeError(
                    f"torch {torch.__version__}: ProcessGroup._wait_for_pending_works is missing; without it "
                    "a capture can race ProcessGroupNCCL's watchdog (graph_step.retire_collectives)")
            wait()


def _process_groups():
    """Every process group torch.distributed has created (private c10d state: checked here, so a
    torch upgrade that renames it fails loudly instead of skipping the retire step)."""
    from torch.distributed import distributed_c10d as c10d
    world = getattr(c10d, "_world", None)
    pg_map = getattr(world, "pg_map", None)
    if pg_map is None:
        raise RuntimeError(f"torch {torch.__version__}: distributed_c10d._world.pg_map is missing "
                           "(graph_step.retire_collectives needs the process-group list)")
    return list(pg_map.keys())


def private_api_ok():
    """The private torch.distributed symbols retire_collectives relies on exist in this torch."""
    from torch.distributed import distributed_c10d as c10d
    pg_cls = getattr(torch._C._distributed_c10d, "ProcessGroup", None)
    return (getattr(getattr(c10d, "_world", None), "pg_map", None) is not None and pg_cls is not None
            and hasattr(pg_cls, "_wait_for_pending_works"))


def _grad_mismatch(params, ref_grads, rtol):
    for i, (p, r) in enumerate(zip(params, ref_grads)):
        g = p.grad
        if (g is None) != (r is None):
            return f"parameter {i}: gradient presence differs"
        if g is None:
            continue
        err = float((g.double() - r.double()).abs().max()) if g.numel() else 0.0
        scale = float(r.double().abs().max()) if r.numel() else 0.0
        if not err <= rtol * max(1.0, scale):
            return f"parameter {i} {tuple(g.shape)}: max |diff| {err:.3g} vs max |ref| {scale:.3g}"
    return None


class CapturedStep:
    """fn captured once and replayed per call.

    agree: for multi-process runs, a callable mapping this rank's bool to the AND over all
    ranks (one collective outside the graph).  Capture success and the replay check are agreed
    before any rank replays, so either every rank replays (and runs the captured collectives)
    or every rank runs eagerly: a rank-local fallback would leave the ranks running different
    collective sequences.
    """

    def __init__(self, fn, params, warmup=3, check=True, rtol=1e-5, agree=None, pool=None):
        """pool: a torch.cuda.graph_pool_handle() shared with other CapturedSteps that are never
        replayed concurrently (static_batch.StaticTrainer: one graph per bucket)."""
        self.fn = fn
        self.pool = pool
        self.params = list(params)
        self.graph = None
        self.static_out = None
        self.fallback_reason = None
        self._agree = agree or (lambda ok: ok)
        self._capture(warmup, check, rtol)

    def _zero(self):
        for p in self.params:
            p.grad = None

    def _capture(self, warmup, check, rtol):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # lazy initialisation (plans, workspaces, BLAS handles) off-capture
            for _ in range(max(1, warmup)):
                self._zero()
                ref = self.fn().detach().clone()
            ref_grads = [p.grad.detach().clone() if p.grad is not None else None for p in self.params] \
                if check else None
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        retire_collectives()
        self._zero()
        g = torch.cuda.CUDAGraph()
        ok = True
        try:
            # thread_local: unsafe calls (host syncs, event queries) are refused on this thread
            # while it captures.  ProcessGroupNCCL's watchdog thread queries nothing during the
            # capture: every warm-up collective was retired from its list above, and collectives
            # issued while capturing are never put on it (they belong to the graph).
            with gc_paused(), torch.cuda.graph(g, pool=self.pool, capture_error_mode="thread_local"):  # records only
                out = self.fn()
        except RuntimeError as e:  # capture unsupported for some op
            self.fallback_reason = f"capture failed: {e}"
            ok = False
        torch.cuda.synchronize()
        if not self._agree(ok):
            self.fallback_reason = self.fallback_reason or "capture failed on another rank"
            self._zero()
            return
        g.replay()
        torch.cuda.synchronize()
        if check:
            a, b = float(out.detach().double()), float(ref.double())
            ok = abs(a - b) <= rtol * max(1.0, abs(b))
            if not ok:
                self.fallback_reason = f"replayed loss {a!r} != eager loss {b!r}"
            else:  # the gradients too: a replay can be wrong where the loss is right
                bad = _grad_mismatch(self.params, ref_grads, rtol)
                if bad is not None:
                    ok = False
                    self.fallback_reason = f"replayed gradient != eager gradient ({bad})"
            del ref_grads
        if not self._agree(ok):
            self.fallback_reason = self.fallback_reason or "replay check failed on another rank"
            self._zero()
            return
        # detached: the captured autograd graph is not kept alive between replays
        self.graph, self.static_out = g, out.detach()
        # the .grad tensors the captured backward writes into: re-attached after every replay, so
        # an optimizer.zero_grad() (set_to_none=True by default, train.py:66) between steps cannot
        # leave the replayed gradients in tensors no parameter references
        self.static_grads = [p.grad for p in self.params]

    @property
    def captured(self):
        return self.graph is not None

    def __call__(self):
        if self.graph is None:
            self._zero()
            return self.fn()
        self.graph.replay()
        for p, g in zip(self.params, self.static_grads):
            p.grad = g
        return self.static_out
