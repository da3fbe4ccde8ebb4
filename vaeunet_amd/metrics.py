"""Hard-threshold segmentation metric (drop-in for the reference's
utils/metrics.py:8-47: ``dice_score``, ``multiclass_dice_score``,
``dice_loss``).

``dice_score`` thresholds the RAW tensors at 0.5 (logits, not probabilities:
metrics.py:18-19) and takes global sums; ``reduce_batch_first`` only changes
the view the reference sums over, never the sums, so it does not change the
value.  The counts are exact integers on the device (csrc/loss.hip
``vu_dice_score``) and the reference's ``denominator.item() == 0`` branch is a
device-side select, so no host synchronisation happens.
"""
import torch

from ._lib import ptr, call, query, stream
from .loss import _dense_pair


def dice_score(input, target, reduce_batch_first=False, epsilon=1e-6):
    """Dice of (input > 0.5) vs (target > 0.5) (metrics.py:8-35); 0-dim fp32
    tensor on the input's device."""
    if input.shape != target.shape:
        raise ValueError(f'Shape mismatch in dice_score: input {input.shape} vs target {target.shape}')
    x, t = _dense_pair(input, target)
    score = torch.empty((), dtype=torch.float32, device=x.device)
    ws = torch.empty(query("vu_loss_workspace_bytes") // 8 + 1, dtype=torch.float64, device=x.device)
    call("vu_dice_score", ptr(x), ptr(t), x.numel(), float(epsilon), ptr(score), None, ptr(ws),
         stream())
    return score


def multiclass_dice_score(input, target, reduce_batch_first=False, epsilon=1e-6):
    """metrics.py:38-41 (the class flatten does not change the global sums)."""
    return dice_score(input.flatten(0, 1), target.flatten(0, 1), reduce_batch_first, epsilon)


def dice_loss(input, target, multiclass=False):
    """1 - dice (metrics.py:44-47)."""
    fn = multiclass_dice_score if multiclass else dice_score
    return 1 - fn(input, target, reduce_batch_first=True)
