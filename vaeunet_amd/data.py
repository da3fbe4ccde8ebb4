"""Reader for the reference's IDRiD patch cache.

The reference slices every training image into overlapping patches and
caches each one with ``torch.save({'image': [3,P,P] f32, 'mask': [1,P,P] f32,
'coords': (y, x), 'has_lesion': bool})`` (utils/data_loading.py:302-446); its
``__getitem__`` reads one file (603-616), a 6-worker DataLoader collates a
batch on the host (train.py:111-134, 239-248) and the training loop copies
it to the device as channels_last (train.py:382-383).

``PatchCache`` reads the same files (``torch.load(weights_only=True)``: no
code is unpickled) with a thread pool, stages each batch in pinned host
memory, copies it to the GPU on a side stream (overlapping the step that is
running) and applies the GEOMETRIC part of the reference's training
augmentation (utils/data_loading.py:116-120: HorizontalFlip, VerticalFlip,
RandomRotate90, each p = 0.5, applied to image and mask alike) on the device
in one gather launch per tensor (``vu_gather_affine``).  The photometric and
elastic transforms (CLAHE, gamma, colour jitter, affine, noise, blur, grid
distortion; :121-178) come from albumentations, which is absent here: out of
scope.  Normalize(mean=0, std=1) of train.py:37 is the identity.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

from . import kernels as K
from ._lib import F32

CL = torch.channels_last


def load_patch(path):
    """One cache record (utils/data_loading.py:605-612)."""
    return torch.load(path, map_location="cpu", weights_only=True)


def _flip_rot_map(P, hflip, vflip, k):
    """Integer map (y, x) of the SOURCE pixel for output (i, j) after
    HorizontalFlip -> VerticalFlip -> rot90(k) (numpy's counter-clockwise
    rot90, as albumentations), square P x P."""
    # start from the identity output->source map and undo the ops last-first
    # rot90 (CCW) once: out[i][j] = in[j][P-1-i]
    ay, by, cy = 1, 0, 0     # y_src = ay*i + by*j + cy
    ax, bx, cx = 0, 1, 0     # x_src = ax*i + bx*j + cx
    for _ in range(k % 4):
        # out[i][j] = prev[j][P-1-i]: substitute (i, j) -> (j, P-1-i) into prev's map
        ay, by, cy, ax, bx, cx = -by, ay, cy + by * (P - 1), -bx, ax, cx + bx * (P - 1)
    if vflip:
        ay, by, cy = -ay, -by, (P - 1) - cy
    if hflip:
        ax, bx, cx = -ax, -bx, (P - 1) - cx
    return [ay, by, cy, ax, bx, cx]


class PatchCache:
    """Iterate the cached patches in batches on ``device``.

    paths: cache files (or a directory holding them); yields dicts with
    ``image`` [B, 3, P, P] and ``mask`` [B, 1, P, P] (fp32, channels_last, on
    the device), ``img_id`` and ``coords``.  ``augment`` enables the
    flip/rotate augmentation (seeded: ``seed``)."""

    def __init__(self, paths, batch_size, device="cuda", augment=False, shuffle=False, seed=0, workers=6,
                 drop_last=False):
        if isinstance(paths, (str, os.PathLike)) and os.path.isdir(paths):
            paths = sorted(os.path.join(paths, f) for f in os.listdir(paths))
        self.paths = list(paths)
        self.batch_size = batch_size
        self.device = torch.device(device)
        self.augment = augment
        self.shuffle = shuffle
        self.rng = np.random.Generator(np.random.PCG64(seed))
        self.pool = ThreadPoolExecutor(max_workers=workers)        # file reads
        self.batch_pool = ThreadPoolExecutor(max_workers=1)        # batch assembly (prefetch 1)
        self.drop_last = drop_last
        self.stream = torch.cuda.Stream(device=self.device) if self.device.type == "cuda" else None

    def __len__(self):
        n = len(self.paths)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def _host_batch(self, idx):
        recs = list(self.pool.map(lambda i: load_patch(self.paths[i]), idx))
        img = torch.stack([r["image"] for r in recs]).float()
        msk = torch.stack([r["mask"] for r in recs]).float()
        ids = [os.path.basename(self.paths[i]).rsplit("_", 1)[0] for i in idx]
        return img.pin_memory(), msk.pin_memory(), ids, [tuple(r.get("coords", (0, 0))) for r in recs]

    def _to_device(self, host):
        img, msk, ids, coords = host
        with torch.cuda.stream(self.stream):
            dimg = img.to(self.device, non_blocking=True).contiguous(memory_format=CL)
            dmsk = msk.to(self.device, non_blocking=True).contiguous(memory_format=CL)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return dimg, dmsk, ids, coords, ev

    def augment_batch(self, img, msk, flags=None):
        """Flip / rot90 per sample (flags: [(hflip, vflip, k)] or drawn)."""
        B, _, H, W = img.shape
        if H != W:
            raise ValueError("rot90 augmentation needs square patches")
        if flags is None:
            flags = []
            for _ in range(B):
                hf = self.rng.random() < 0.5
                vf = self.rng.random() < 0.5
                k = int(self.rng.integers(0, 4)) if self.rng.random() < 0.5 else 0
                flags.append((hf, vf, k))
        m = torch.tensor([_flip_rot_map(H, *f) for f in flags], dtype=torch.int32).to(img.device)
        outs = []
        for t in (img, msk):
            o = K.empty_act(B, t.shape[1], H, W, torch.float32, t.device)
            K.call("vu_gather_affine", K.ptr(t), B, H, W, t.shape[1], K.ptr(m), K.ptr(o), H, W, F32, K.stream())
            outs.append(o)
        return outs[0], outs[1], flags

    def __iter__(self):
        order = np.arange(len(self.paths))
        if self.shuffle:
            self.rng.shuffle(order)
        batches = [order[i:i + self.batch_size] for i in range(0, len(order), self.batch_size)]
        if self.drop_last and batches and len(batches[-1]) < self.batch_size:
            batches.pop()
        nxt = self.batch_pool.submit(self._host_batch, batches[0]) if batches else None
        for bi in range(len(batches)):
            host = nxt.result()
            nxt = self.batch_pool.submit(self._host_batch, batches[bi + 1]) if bi + 1 < len(batches) else None
            img, msk, ids, coords, ev = self._to_device(host)
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            img.record_stream(cur)   # allocated on the copy stream, used (and freed) on this one
            msk.record_stream(cur)
            if self.augment:
                img, msk, _ = self.augment_batch(img, msk)
            yield {"image": img, "mask": msk, "img_id": ids, "coords": coords}
