"""Data-parallel gradient reduction over RCCL (xGMI), overlapped with backward.

The reference trains in one process (train.py:677);
this module adds data parallelism the MI355X way: one process per GPU,
``torch.distributed`` with the ``nccl`` backend (= RCCL on ROCm), gradients
bucketed (~25 MB fp32) in reverse registration order — the order the fused
backward (unet_model.UNet._bwd) produces them — and each bucket all-reduced
the moment its last gradient is written, while the backward of the blocks
below keeps the compute stream busy.

Mechanics: every parameter's ``.grad`` is a view into its bucket's flat fp32
buffer, so the weight-gradient kernels write straight into the buffer that
RCCL reduces (no pack/unpack copies).  c10d enqueues the collective on its
own stream behind the work already queued on the compute stream (the event
fence), and ``finish()`` makes the compute stream wait for every bucket
before the optimizer reads the gradients.

BatchNorm running statistics stay per replica (the reference has no
SyncBN; DDP-without-SyncBN semantics: every rank normalises with its own
shard's batch statistics).  Parameters are broadcast from rank 0 once at
construction.
"""
import contextlib

import torch
import torch.distributed as dist


class GradBucketReducer:
    def __init__(self, params, bucket_bytes=25 * 1024 * 1024, group=None, average=True):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.world = dist.get_world_size(group)
        self.average = average
        self.buckets = []          # list of (flat tensor, [params])
        self.where = {}            # id(param) -> bucket index
        cur, cur_bytes = [], 0
        for p in reversed(self.params):
            cur.append(p)
            cur_bytes += p.numel() * 4
            if cur_bytes >= bucket_bytes:
                self.buckets.append(cur)
                cur, cur_bytes = [], 0
        if cur:
            self.buckets.append(cur)
        self.flats = []
        for bi, plist in enumerate(self.buckets):
            n = sum(p.numel() for p in plist)
            self.flats.append(torch.zeros(n, dtype=torch.float32, device=plist[0].device))
            for p in plist:
                self.where[id(p)] = bi
        self._pending = None
        self._handles = []
        self._sync = True
        self._unused = {}          # id(param) -> unreported AND zero slot on the last eager step (finish())
        self._used = set()         # id(param) of unreported parameters once seen non-zero (kept for good)
        with torch.no_grad():
            for p in self.params:
                dist.broadcast(p.data, src=0, group=group)

    def _bind(self):
        """Point every .grad at its slot of the flat bucket buffer.

        torch semantics are kept: a gradient accumulates until it is reset.
        A parameter whose ``.grad`` is None (``zero_grad(set_to_none=True)``)
        gets its slot zeroed; one already bound keeps its contents (gradient
        accumulation over micro-batches, train.py:401-411); a foreign tensor
        is copied into the slot."""
        for bi, plist in enumerate(self.buckets):
            flat = self.flats[bi]
            fresh = all(p.grad is None for p in plist)
            if fresh:
                flat.zero_()  # one launch per bucket after zero_grad(set_to_none=True)
            off = 0
            for p in plist:
                n = p.numel()
                view = flat[off:off + n].view(p.shape)
                # keep the parameter's memory layout (channels_last weights)
                if p.dim() == 4 and not p.is_contiguous():
                    view = flat[off:off + n].view(p.shape[0], p.shape[2], p.shape[3],
                                                  p.shape[1]).permute(0, 3, 1, 2)
                if p.grad is None:
                    if not fresh:
                        view.zero_()
                    p.grad = view
                elif p.grad.data_ptr() != view.data_ptr():
                    view.copy_(p.grad)
                    p.grad = view
                off += n

    def zero_grad(self):
        """Zero every bucket in place (the bound .grad views included): one HIP
        fill per bucket on the GPU (vu_zero), torch on CPU (gloo tests)."""
        for flat in self.flats:
            if flat.is_cuda:
                from . import kernels as K
                K.call("vu_zero", K.ptr(flat), 0, 1, flat.numel(), K.dcode(flat.dtype), K.stream())
            else:
                flat.zero_()

    @contextlib.contextmanager
    def no_sync(self):
        """Micro-batches run inside accumulate their gradients locally (no
        collective); the next synchronised backward all-reduces the sum --
        DDP's ``no_sync`` for the reference's grad-accumulation x2
        (train.py:401,406)."""
        old = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = old

    def prepare(self):
        """Call before the forward of every micro-batch (inside or outside
        ``no_sync``): binds the gradient views; arms the bucket counters only
        when this backward is to be reduced."""
        self._bind()
        self._handles = []
        if self._sync:
            self._pending = [len(b) for b in self.buckets]
            self._seen = set()
        else:
            self._pending = None

    def grad_ready(self, params):
        """Engine callback: these parameters' gradients are final for this step."""
        if self._pending is None:
            return
        for p in params:
            bi = self.where.get(id(p))
            if bi is None or id(p) in self._seen:
                continue
            self._seen.add(id(p))
            self._pending[bi] -= 1
            if self._pending[bi] == 0:
                self._launch(bi)

    def _launch(self, bi):
        flat = self.flats[bi]
        if self.average and dist.get_backend(self.group) == "nccl":
            h = dist.all_reduce(flat, op=dist.ReduceOp.AVG, group=self.group, async_op=True)
            self._handles.append((h, None))
        else:
            h = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            self._handles.append((h, flat if self.average else None))

    def finish(self):
        """Launch any bucket the engine did not report, then fence on all of
        them (a no-op after a ``no_sync`` micro-batch).

        A parameter the engine never reported during a synchronised backward
        AND whose reduced gradient slot is exactly zero on every rank received
        no gradient this step (UNetResNet's z_initial when use_bottleneck is
        False): its ``.grad`` is reset to None afterwards -- torch semantics,
        so the optimizer skips it (no AdamW state, no weight decay) as it
        would without the reducer.  A non-zero slot is kept: a backward path
        that forgot to report a parameter only delays its bucket, it never
        drops a real gradient.  Only "used" is cached: a parameter found zero
        is re-tested (one host read) on every later eager step until its slot
        is non-zero once, so a gradient that first arrives on step k > 1
        (zero-initialised downstream weight, a dead ReLU, a branch warming up)
        is kept from step k on.  While a graph is being captured
        the last eager observation decides."""
        if not self._sync:
            return
        unseen = []
        if self._pending is not None:
            if self._seen:
                unseen = [p for p in self.params if id(p) not in self._seen]
            for bi, left in enumerate(self._pending):
                if left > 0:
                    self._pending[bi] = 0
                    self._launch(bi)
        for h, flat in self._handles:
            h.wait()
            if flat is not None:
                flat.div_(self.world)
        self._handles = []
        self._pending = None
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        for p in unseen:
            if id(p) in self._used:
                continue
            if capturing or p.grad is None:
                if self._unused.get(id(p)):
                    p.grad = None
                continue
            if bool(torch.count_nonzero(p.grad).item() == 0):
                self._unused[id(p)] = True
                p.grad = None
            else:
                self._used.add(id(p))
                self._unused.pop(id(p), None)


def attach(model, **kw):
    """Create a reducer for ``model`` and wire the fused backward's grad_ready hook."""
    red = GradBucketReducer(model.parameters(), **kw)
    model.grad_ready = red.grad_ready
    return red
