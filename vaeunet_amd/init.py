"""Seeded, version-stable parameter initialisation.

The golden fixtures (tests/golden) and the benchmark need the same weights
on every machine without shipping a 125 MB state_dict.  torch's own RNG
stream is not guaranteed stable across versions, so weights are drawn from
numpy's PCG64 in state_dict order:

* conv / conv-transpose weights: U(-b, b), b = 1/sqrt(prod(shape[1:]))
* BatchNorm weight: 1 + 0.1*U(-1, 1); BatchNorm bias: 0.1*U(-1, 1)
* every other float parameter (conv biases): 0.05*U(-1, 1)
* buffers (running_mean / running_var / num_batches_tracked) keep their
  constructor values.
"""
import numpy as np
import torch


def seeded_state(named_shapes, seed=0):
    """Return {name: np.float32 array} for (name, shape, kind) triples.

    ``kind`` is one of "weight", "bn_weight", "bn_bias", "bias".
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for name, shape, kind in named_shapes:
        n = int(np.prod(shape)) if len(shape) else 1
        u = rng.uniform(-1.0, 1.0, size=n).astype(np.float32).reshape(shape)
        if kind == "weight":
            fan = int(np.prod(shape[1:])) if len(shape) > 1 else 1
            out[name] = u * np.float32(1.0 / np.sqrt(fan))
        elif kind == "bn_weight":
            out[name] = np.float32(1.0) + np.float32(0.1) * u
        elif kind == "bn_bias":
            out[name] = np.float32(0.1) * u
        else:
            out[name] = np.float32(0.05) * u
    return out


def _param_kinds(module):
    kinds = []
    for mname, m in module.named_modules():
        for pname, p in m.named_parameters(recurse=False):
            full = f"{mname}.{pname}" if mname else pname
            is_bn = isinstance(m, torch.nn.modules.batchnorm._BatchNorm)
            if is_bn:
                kind = "bn_weight" if pname == "weight" else "bn_bias"
            elif pname == "weight" and p.dim() > 1:
                kind = "weight"
            else:
                kind = "bias"
            kinds.append((full, tuple(p.shape), kind))
    return kinds


@torch.no_grad()
def seeded_init_(module, seed=0):
    """Overwrite every parameter of ``module`` in place from PCG64(seed)."""
    kinds = _param_kinds(module)
    vals = seeded_state(kinds, seed)
    params = dict(module.named_parameters())
    for name, _, _ in kinds:
        p = params[name]
        p.copy_(torch.from_numpy(vals[name]).to(device=p.device, dtype=p.dtype))
    return module
