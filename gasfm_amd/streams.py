"""Point side of a block on a second HIP stream, concurrent with the camera side.

After a block's two attentions, its scene-point work (PointTailFn + PointHubFn: 200k-row
LN/MFMA kernels) and its camera work (ViewTailFn + ViewHubFn: the 1000x1024 hipBLASLt GEMMs
and column-split kernels) are independent until the global update.  Run back to back on one
stream they add up; a ``SideSection`` runs the point kernels on a second stream, forward and
backward, so the two halves overlap (on their own streams in eager mode; as parallel branches
of the replayed hipGraph, which the HIP runtime executes on parallel streams).

Protocol (one SideSection per block):
  forward   fork() right after the attention (the side stream waits for it), then the camera
            work is enqueued on torch's stream and the point work inside ``launches()`` on the
            side stream; join() before the global update (torch's stream waits for the side).
  backward  autograd runs PointHubFn first (it is created last), which fork()s (the side stream
            waits for the global/epilogue backward), then PointTailFn continues on the side
            stream (its only gradient comes from the hub); DualAttentionFn.backward join()s
            before it reads the point-side gradient.
Allocation safety: every tensor is allocated on torch's current stream, so two rules apply.
(1) Every tensor a side-stream kernel touches is kept referenced (``keep``) until the join,
after which torch's stream is ordered behind the side stream: the caching allocator cannot
hand its memory to a torch-stream kernel while the side stream still uses it.  (2) Every
buffer a side-stream kernel writes is allocated BEFORE the fork (``alloc``/``bufs``): memory
allocated later may have been freed by torch-stream work enqueued after the fork and still
pending (a camera-side scratch buffer, say), which the side stream does not wait for.  Weight-gradient partials must be
deferred to the batched end-of-backward colsum (``_native.param_colsum``), which runs on
torch's stream after every join; sections are only used when they are.
"""
import os

import torch

from . import _native

_SIDE = {}

# Off by default: measured on MI355X (tools/ab_side.sh, hipGraph replay) config 4 37.66 ms with the
# side stream vs 37.43 ms without, the 1/8 proxy 11.80 vs 11.22 ms -- the 200k-row point kernels
# already fill the chip, so the overlap buys nothing.  env GASFM_SIDE_STREAM=1 turns it on.
enabled = os.environ.get("GASFM_SIDE_STREAM", "0") == "1"


def side_stream(device):
    s = _SIDE.get(device)
    if s is None:
        s = _SIDE[device] = torch.cuda.Stream(device)
    return s


class SideSection:
    def __init__(self, device):
        self.side = side_stream(device)
        self.keep = []
        self.bufs = {}   # side-stream buffers allocated before a fork (see point_block._take)
        self.forked = False

    def alloc(self, key, shape, like):
        self.bufs[key] = torch.empty(shape, dtype=torch.float32, device=like.device)

    def fork(self):
        self.side.wait_stream(torch.cuda.current_stream(self.side.device))
        self.forked = True

    def launches(self, *tensors):
        """Context for the side-stream launches; ``tensors`` stay referenced until join()."""
        self.keep.extend(t for t in tensors if t is not None)
        return _native.launching_on(self.side)

    def join(self):
        if self.forked:
            torch.cuda.current_stream(self.side.device).wait_stream(self.side)
            self.forked = False
        self.keep.clear()
        self.bufs.clear()


def section_for(device, deferring):
    """A SideSection when the point side may run concurrently (CUDA, deferred weight sums)."""
    if not (enabled and deferring and device.type == "cuda"):
        return None
    return SideSection(device)
