"""Optimizer tail of the training step as multi-tensor HIP launches.

Drop-ins for the two calls of the reference's optimizer step
(train.py:406-411, optimizer built at train.py:334):

* ``clip_grad_norm_(params, max_norm)`` == ``torch.nn.utils.clip_grad_norm_``
  (norm_type 2): total norm over all grads (fp64 accumulation), grads scaled
  in place by ``min(1, max_norm / (norm + 1e-6))``, the norm returned as a
  0-dim device tensor.  No host synchronisation.
* ``FusedAdamW`` == ``torch.optim.AdamW`` (decoupled weight decay, amsgrad
  off): same constructor, ``param_groups``, ``state`` keys (``step`` as a CPU
  float32 tensor, ``exp_avg``, ``exp_avg_sq``) and update order as torch's
  foreach implementation, so state dicts move between the two and
  ``GradScaler`` drives it unchanged.

Each is one table upload plus one to three launches for ALL parameters
(include/vaeunet.h, vu_mt_*), instead of a dozen foreach launches.
"""
import ctypes as C

import torch
from torch.autograd.graph import increment_version

from . import _lib

_CHUNK = None


def _chunk():
    global _CHUNK
    if _CHUNK is None:
        _CHUNK = int(_lib.query("vu_mt_chunk_elems"))
    return _CHUNK


def _is_dense(t):
    """Non-overlapping and dense: the elements fill numel() consecutive slots
    of storage in some dimension order (contiguous, channels_last, ...)."""
    if t.numel() <= 1:
        return True
    dims = sorted((st, sz) for st, sz in zip(t.stride(), t.size()) if sz != 1)
    expect = 1
    for st, sz in dims:
        if st != expect:
            return False
        expect *= sz
    return True


def _dense_like(t, ref):
    """``t`` with ``ref``'s strides (the kernels walk the flat storage)."""
    if t.stride() == ref.stride() and _is_dense(t):
        return t
    out = torch.empty_like(ref)
    out.copy_(t)
    return out


class _Table:
    """Device copy of a VuMtEntry array (uploaded asynchronously from pinned
    memory; the caching host allocator keeps the staging block alive until
    the copy has run)."""

    def __init__(self, rows, device):
        ch = _chunk()
        n = len(rows)
        arr = (_lib.VuMtEntry * n)()
        c0 = 0
        for i, (p, g, m, v, step_size, bc2s) in enumerate(rows):
            e = arr[i]
            e.param = p.data_ptr()
            e.grad = g.data_ptr()
            e.exp_avg = m.data_ptr() if m is not None else None
            e.exp_avg_sq = v.data_ptr() if v is not None else None
            e.numel = p.numel()
            e.chunk0 = c0
            e.step_size = step_size
            e.bc2_sqrt = bc2s
            c0 += -(-p.numel() // ch)
        self.n = n
        self.nchunks = c0
        host = torch.frombuffer(bytearray(arr), dtype=torch.uint8).pin_memory()
        self.dev = host.to(device, non_blocking=True)
        self.keep = rows  # the tensors must outlive the launches queued on them

    def ptr(self):
        return C.c_void_p(self.dev.data_ptr())


def _check(t, what):
    if not t.is_cuda:
        raise RuntimeError(f"vaeunet_amd.optim: {what} must be a GPU tensor (no CPU path)")
    if t.dtype != torch.float32:
        raise RuntimeError(f"vaeunet_amd.optim: {what} must be float32, got {t.dtype}")


@torch.no_grad()
def clip_grad_norm_(parameters, max_norm, norm_type=2.0, error_if_nonfinite=False, foreach=None):
    """torch.nn.utils.clip_grad_norm_ for fp32 GPU grads (norm_type 2)."""
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    grads = [p.grad for p in parameters if p.grad is not None]
    if float(norm_type) != 2.0:
        raise NotImplementedError("vaeunet_amd.optim.clip_grad_norm_: only norm_type=2")
    if not grads:
        return torch.tensor(0.0)
    dev = grads[0].device
    rows = []
    for g in grads:
        _check(g, "grad")
        if not _is_dense(g):
            raise RuntimeError("vaeunet_amd.optim.clip_grad_norm_: grads must be dense")
        rows.append((g, g, None, None, 0.0, 1.0))
    tab = _Table(rows, dev)
    out = torch.empty(2, dtype=torch.float32, device=dev)  # norm, coef
    ws = torch.empty(tab.nchunks, dtype=torch.float64, device=dev)
    s = _lib.stream()
    _lib.call("vu_mt_grad_norm", tab.ptr(), tab.n, tab.nchunks, float(max_norm), _lib.ptr(out[0:1]),
              _lib.ptr(out[1:2]), _lib.ptr(ws), s)
    _lib.call("vu_mt_scale_grads", tab.ptr(), tab.n, tab.nchunks, _lib.ptr(out[1:2]), s)
    increment_version(grads)  # written in place behind autograd's back
    total = out[0]
    if error_if_nonfinite and not torch.isfinite(total):
        raise RuntimeError(f"The total norm of order {norm_type} for gradients from `parameters` "
                           "is non-finite, so it cannot be clipped.")
    return total


class FusedAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW with one multi-tensor HIP launch per parameter group."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 amsgrad=False, *, maximize=False, foreach=None, capturable=False,
                 differentiable=False, fused=None):
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameters: {betas}")
        if not 0.0 <= weight_decay:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if amsgrad or maximize or capturable or differentiable:
            raise NotImplementedError("FusedAdamW: amsgrad / maximize / capturable / differentiable")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad,
                        maximize=maximize, foreach=foreach, capturable=capturable,
                        differentiable=differentiable, fused=fused)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        ref = getattr(self, "_vu_graph", None)  # weakref to a GraphedTrainStep replaying this optimizer
        graph = ref() if ref is not None else None
        if graph is not None and not graph._synced:
            graph.sync_optimizer_state()  # its replays advanced the step count on the device
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            lr = float(group["lr"])
            rows = []
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdamW does not support sparse gradients")
                _check(p, "param")
                _check(p.grad, "grad")
                if not _is_dense(p):
                    raise RuntimeError("FusedAdamW: parameters must be dense")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                m = _dense_like(st["exp_avg"], p)
                v = _dense_like(st["exp_avg_sq"], p)
                if m is not st["exp_avg"]:
                    st["exp_avg"] = m
                if v is not st["exp_avg_sq"]:
                    st["exp_avg_sq"] = v
                st["step"] += 1
                step = float(st["step"].item()) if st["step"].device.type == "cpu" else float(st["step"])
                bc1 = 1 - beta1 ** step
                bc2 = 1 - beta2 ** step
                rows.append((p, _dense_like(p.grad, p), m, v, lr / bc1, bc2 ** 0.5))
            if not rows:
                continue
            tab = _Table(rows, rows[0][0].device)
            _lib.call("vu_mt_adamw", tab.ptr(), tab.n, tab.nchunks,
                      1.0 - lr * float(group["weight_decay"]), 1.0 - beta1, float(beta2),
                      1.0 - beta2, float(group["eps"]), None, _lib.stream())
            # the kernel updated params and moments in place: bump their
            # version counters like torch's in-place ops do (derived caches,
            # e.g. the engine's bf16 weight layouts, key on them)
            increment_version([r[k] for r in rows for k in (0, 2, 3)])
        if graph is not None:
            graph.load_optimizer_steps()  # later replays continue from this step
        return loss
