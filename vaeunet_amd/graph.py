"""Whole training step as one HIP graph (launch reduction).

The reference's step (train.py:381-411) is ~300 (U-Net) to ~600 (VAE-U-Net)
kernel launches; issued from Python each one costs tens of microseconds of
host time, which for the VAE-U-Net exceeds the GPU time of the step.
``GraphedTrainStep`` captures forward + loss + backward + clip_grad_norm_ +
AdamW once (``torch.cuda.CUDAGraph`` over HIP graphs) and replays it:

* static inputs: the caller's ``forward_backward`` closure reads fixed
  tensors (copy each new batch into them before ``step()``);
* persistent ``.grad`` buffers: zero-initialised before capture, the
  backward accumulates into them and the capturable AdamW kernel
  (``vu_mt_adamw_dev``) clears them after use, so every replay sees zeros;
* the step count lives on the device (one per parameter group) and the
  AdamW bias corrections are derived from it in the kernel (same double
  arithmetic as the eager path);
* the derived bf16 weight images are rebuilt in place by one prebuilt
  permute launch at the start of each replay (``engine.StaticRefresh``);
* the multi-tensor tables of the clip and AdamW launches are uploaded once,
  before capture.

The learning rate, betas, eps, weight decay and max_norm are frozen at
capture (rebuild the object to change them).

Data parallel (``reducer``, vaeunet_amd.parallel): the gradient buffers are
the reducer's bucket views, and the bucketed all-reduces the fused backward
launches (RCCL, c10d's ``nccl`` backend) are captured with the step: each
collective's fork from and join to the compute stream become graph edges,
so a replay overlaps the buckets with the backward exactly as the eager step
does.  Only RCCL collectives are capturable (gloo runs on the host).
"""
import gc
import weakref

import torch
from torch.autograd.graph import increment_version

from . import _lib
from . import engine as E
from .optim import FusedAdamW, _Table, clip_grad_norm_


class GraphedTrainStep:
    """forward_backward(): runs the forward, the loss and ``loss.backward()``
    on static inputs and returns the loss tensor."""

    def __init__(self, forward_backward, optimizer, max_norm=None, warmup=2, reducer=None):
        if not isinstance(optimizer, FusedAdamW):
            raise TypeError("GraphedTrainStep needs vaeunet_amd.optim.FusedAdamW")
        if reducer is not None:
            import torch.distributed as dist
            if dist.get_backend(reducer.group) != "nccl":
                raise RuntimeError("GraphedTrainStep: only RCCL (nccl backend) collectives can be captured")
            inner = forward_backward

            def forward_backward():
                reducer.prepare()
                loss = inner()
                reducer.finish()
                return loss
        self.reducer = reducer
        self.fb = forward_backward
        self.opt = optimizer
        self.max_norm = max_norm
        every = [p for g in optimizer.param_groups for p in g["params"] if p.requires_grad]
        # eager warm-up: builds the weight images, optimizer state and every
        # workspace the step touches
        for _ in range(max(1, warmup)):
            self.fb()
            if max_norm is not None:
                clip_grad_norm_([p for p in every if p.grad is not None], max_norm)
            optimizer.step()
            optimizer.zero_grad(set_to_none=True)
        # only the parameters the step gives a gradient (those AdamW holds state
        # for): an unused one (UNetResNet's z_initial when use_bottleneck is
        # False) keeps .grad None, so torch's AdamW would leave it untouched too
        params = [p for p in every if len(optimizer.state.get(p, {})) > 0]
        if not params:
            raise RuntimeError("GraphedTrainStep: no parameter received a gradient in the warm-up")
        self.params = params
        keep = set(id(p) for p in params)
        dev = params[0].device
        # persistent zero gradients (the backward accumulates into them; the
        # capturable AdamW clears them after use): the reducer's bucket views
        # when data parallel
        if reducer is not None:
            reducer.zero_grad()
            reducer._bind()
            for p in params:
                if p.grad is None:
                    raise RuntimeError("GraphedTrainStep: a parameter outside the reducer's buckets")
        else:
            for p in params:
                p.grad = torch.zeros_like(p)
        self.grads = [p.grad for p in params]
        self.clip_tab = _Table([(p.grad, p.grad, None, None, 0.0, 1.0) for p in params], dev)
        self.norm = torch.empty(2, dtype=torch.float32, device=dev)
        self.ws = torch.empty(max(1, self.clip_tab.nchunks), dtype=torch.float64, device=dev)
        self.groups = []
        for group in optimizer.param_groups:
            rows, step0 = [], 0.0
            for p in group["params"]:
                if id(p) not in keep:
                    continue
                st = optimizer.state[p]
                rows.append((p, p.grad, st["exp_avg"], st["exp_avg_sq"], 0.0, 1.0))
                step0 = float(st["step"])
            if rows:
                step = torch.full((1,), step0, dtype=torch.float32, device=dev)
                self.groups.append((group, _Table(rows, dev), step))
        # images, then capture
        self._synced = True
        # weak: no optimizer <-> graph cycle, so a dropped GraphedTrainStep (and
        # its CUDAGraph) is freed at once, never by a cyclic GC pass that could
        # run while another graph is being captured
        optimizer._vu_graph = weakref.ref(self)
        self.moments = [t for _, tab, _ in self.groups for r in tab.keep for t in (r[2], r[3])]
        self.refresh = E.StaticRefresh(params)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        E._STATIC_REFRESH = self.refresh
        gc_was = gc.isenabled()
        gc.collect()
        gc.disable()   # no collector pass (and no foreign graph destructor) mid-capture
        try:
            with torch.cuda.graph(self.graph):
                self.loss = self.fb()
                self._tail()
        finally:
            E._STATIC_REFRESH = None
            if gc_was:
                gc.enable()
        torch.cuda.synchronize()

    def _tail(self):
        s = _lib.stream()
        coef = None
        if self.max_norm is not None:
            t = self.clip_tab
            _lib.call("vu_mt_grad_norm", t.ptr(), t.n, t.nchunks, float(self.max_norm), _lib.ptr(self.norm[0:1]),
                      _lib.ptr(self.norm[1:2]), _lib.ptr(self.ws), s)
            # the clip coefficient is applied as AdamW reads each gradient
            # (the gradients are cleared after use, so nothing else sees them
            # scaled): the same bits as clip_grad_norm_'s in-place scaling, one
            # pass over the gradients fewer (round 6)
            coef = _lib.ptr(self.norm[1:2])
        for group, t, step in self.groups:
            b1, b2 = group["betas"]
            _lib.call("vu_mt_adamw_dev_scaled", t.ptr(), t.n, t.nchunks, float(group["lr"]),
                      float(group["weight_decay"]), float(b1), float(b2), float(group["eps"]), _lib.ptr(step), 1,
                      coef, s)

    def step(self):
        """Replay one training step; returns the (static) loss tensor.

        The replay updates the parameters and moments in place behind
        autograd's back: their version counters are bumped as torch's in-place
        ops do, so an eager forward after it (validation, inference helpers)
        rebuilds its derived weight images instead of reusing the ones the
        replay started from."""
        self.graph.replay()
        increment_version(self.params)
        increment_version(self.moments)
        self._synced = False
        return self.loss

    @property
    def grad_norm(self):
        """Total gradient norm of the last replay (device tensor)."""
        return self.norm[0]

    def sync_optimizer_state(self):
        """Write the device step counts back into the optimizer's state (for
        checkpoints: train.py:542-565 saves optimizer.state_dict(), and before
        any eager ``optimizer.step()`` after replays).  One host sync."""
        for group, tab, step in self.groups:
            v = float(step.item())
            for r in tab.keep:
                self.opt.state[r[0]]["step"] = torch.tensor(v, dtype=torch.float32)
        self._synced = True

    def load_optimizer_steps(self):
        """The optimizer's (host) step counts -> the device counters the replays
        read: after an eager ``optimizer.step()`` between replays (called by
        FusedAdamW.step itself)."""
        for group, tab, step in self.groups:
            step.fill_(float(self.opt.state[tab.keep[0][0]]["step"]))
        # the eager step consumed the captured gradient buffers without clearing
        # them (and zero_grad may have unbound them): clear and rebind
        with torch.no_grad():
            for p, g in zip(self.params, self.grads):
                g.zero_()
                p.grad = g
        self._synced = True
