"""autograd.Function adapters between torch's autograd and the fused engine.

``BlockFn`` runs one block (forward sequence of HIP launches) and keeps the
saved activations on the ctx; its backward runs the block's backward
sequence.  Parameters are passed to ``apply`` only so that autograd knows the
output depends on them; their gradients are written in place by the engine
(see engine.py) and ``None`` is returned for them.
"""
import torch

from . import engine as E


class Runner:
    """fwd(inputs) -> (out, state); bwd(state, dout) -> tuple(grad per input)."""

    def __init__(self, fwd, bwd):
        self.fwd, self.bwd = fwd, bwd


class BlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, runner, n_in, *args):
        inputs = args[:n_in]
        out, state = runner.fwd(inputs)
        ctx.runner, ctx.state = runner, state
        ctx.n_params = len(args) - n_in
        ctx.in_meta = [(t.requires_grad, t.dtype, t.shape) if torch.is_tensor(t) else None
                       for t in inputs]
        ctx.mark_non_differentiable(*[o for o in (out if isinstance(out, tuple) else (out,))
                                      if not o.is_floating_point()])
        return out

    @staticmethod
    def backward(ctx, *douts):
        grads = ctx.runner.bwd(ctx.state, douts if len(douts) > 1 else douts[0])
        E.join_side()   # weight gradients forked onto the side stream are complete after this point
        ctx.state = None
        return (None, None) + tuple(grads) + (None,) * ctx.n_params


def run_block(module, fwd, bwd, inputs):
    params = [p for p in module.parameters() if p.requires_grad]
    needs_graph = torch.is_grad_enabled() and (
        any(p.requires_grad for p in params) or
        any(torch.is_tensor(t) and t.requires_grad for t in inputs))
    if not needs_graph:
        out, _ = fwd(inputs)
        return out
    return BlockFn.apply(Runner(fwd, bwd), len(inputs), *inputs, *params)


def act_grad(M, dout):
    """Incoming gradient -> NHWC storage of the mode's dtype."""
    return E.to_act(M, dout)
