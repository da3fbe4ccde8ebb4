"""On-disk checkpoint format of the reference.

* ``save_checkpoint`` writes the nested dict of train.py:542-565
  (``epoch``, ``model_state_dict``, ``optimizer_state_dict``,
  ``scheduler_state_dict``, ``best_val_score``, ``amp_scaler``,
  ``global_step``, ``params``) with ``torch.save``; the analysis scripts read
  it back with ``checkpoint['model_state_dict']`` (visualize_vae.py:1236-1237,
  analyze_model.py:1308-1309).
* ``load_checkpoint`` accepts that nested dict or a raw state_dict (train.py's
  ``--load`` path pops ``mask_values``, train.py:698-703), always with
  ``torch.load(..., weights_only=True)`` (nothing executable is unpickled).

The drop-in modules keep the reference's state_dict keys, so checkpoints move
between the reference and this package in both directions.  Derived kernel
weight images are keyed on the parameter version, so ``load_state_dict``
(an in-place copy) invalidates them; ``FusedAdamW`` keeps torch.optim.AdamW's
state layout, so optimizer states are interchangeable too.
"""
import torch


def checkpoint_dict(model, optimizer=None, scheduler=None, grad_scaler=None, epoch=0, best_val_score=float("-inf"),
                    global_step=0, params=None):
    """The train.py:542-565 checkpoint dictionary."""
    return {
        "epoch": epoch,
        "model_state_dict": model.state_dict(),
        "optimizer_state_dict": optimizer.state_dict() if optimizer is not None else None,
        "scheduler_state_dict": scheduler.state_dict() if scheduler is not None else None,
        "best_val_score": best_val_score,
        "amp_scaler": grad_scaler.state_dict() if grad_scaler is not None else None,
        "global_step": global_step,
        "params": dict(params or {}),
    }


def save_checkpoint(path, model, optimizer=None, scheduler=None, grad_scaler=None, epoch=0, best_val_score=float("-inf"),
                    global_step=0, params=None):
    ck = checkpoint_dict(model, optimizer, scheduler, grad_scaler, epoch, best_val_score, global_step, params)
    torch.save(ck, path)
    return ck


def load_checkpoint(path, model, optimizer=None, scheduler=None, grad_scaler=None, map_location=None,
                    strict=True):
    """Load a train.py checkpoint (nested dict) or a raw state_dict into
    ``model`` (and optimizer / scheduler / scaler when given and present).
    Returns the checkpoint dict (a raw state_dict is wrapped as
    ``{'model_state_dict': ...}``)."""
    ck = torch.load(path, map_location=map_location, weights_only=True)
    if not (isinstance(ck, dict) and "model_state_dict" in ck):
        ck = {"model_state_dict": ck}
    sd = dict(ck["model_state_dict"])
    sd.pop("mask_values", None)
    model.load_state_dict(sd, strict=strict)
    if optimizer is not None and ck.get("optimizer_state_dict"):
        optimizer.load_state_dict(ck["optimizer_state_dict"])
    if scheduler is not None and ck.get("scheduler_state_dict"):
        scheduler.load_state_dict(ck["scheduler_state_dict"])
    if grad_scaler is not None and ck.get("amp_scaler"):
        grad_scaler.load_state_dict(ck["amp_scaler"])
    return ck
