"""The reference's IDRiD patch cache: producer and reader.

Producer (``IDRIDDataset``, ``precompute_all_patches``): the reference's
``utils/data_loading.py:42-446`` in patch mode.  Each image / lesion mask pair
is loaded and scaled with PIL exactly as the reference does (``load_image``
:18-28, ``preprocess`` :580-601: bicubic image, nearest mask, /255, mask > 0),
then every stride-P/2 window is decided in ONE device launch per image
(``vu_patch_stats``: black-pixel and lesion-pixel counts of every window, the
reference's per-window Python loop with ``is_valid_patch`` :287-300 and
``has_lesion`` :381), and the kept windows are written in the reference's
record format and file names (:383-389), with the train split's
positive/negative balancing and deletion of the unselected negatives
(:404-446; ``random.shuffle`` of the global generator, or a given one).
Full-image mode (``patch_size=None``: fundus detection with cv2,
:223-285, 448-578) is not built: cv2 is absent here, so it cannot be pinned.

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
import logging
import os
import random
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np
import torch

from . import kernels as K
from ._lib import F32

CL = torch.channels_last


# ----------------------------------------------------------------------------
# producer
# ----------------------------------------------------------------------------
def load_image(filename):
    """utils/data_loading.py:18-28: open with PIL and force 3-channel RGB."""
    from PIL import Image
    return Image.open(filename).convert("RGB")


def preprocess(pil_img, scale, is_mask):
    """utils/data_loading.py:580-601: resize to int(scale * size) (nearest for
    masks, bicubic for images); mask -> {0, 1} float32 [H, W], image ->
    float32 [3, H, W] in [0, 1]."""
    from PIL import Image
    w, h = pil_img.size
    nw, nh = int(scale * w), int(scale * h)
    if nw < 1 or nh < 1:
        raise ValueError(f"Image {pil_img} scaled too small => {nw}x{nh}.")
    arr = np.asarray(pil_img.resize((nw, nh), resample=Image.NEAREST if is_mask else Image.BICUBIC))
    if is_mask:
        return ((arr[..., 0] if arr.ndim == 3 else arr) > 0).astype(np.float32)
    if arr.ndim == 2:
        arr = np.stack([arr] * 3, axis=-1)
    return (arr.astype(np.float32) / 255.0).transpose(2, 0, 1)


def window_stats(img, mask, patch, stride, device):
    """(ny, nx, black counts, lesion counts) of every stride-spaced window of
    img [C, H, W] / mask [1 or C', H, W] (CPU float32): one vu_patch_stats
    launch; the counts come back as int64 numpy arrays [ny * nx]."""
    _, h, w = img.shape
    ny = (h - patch) // stride + 1 if h >= patch else 0
    nx = (w - patch) // stride + 1 if w >= patch else 0
    if ny == 0 or nx == 0:
        return ny, nx, np.zeros(0, np.int64), np.zeros(0, np.int64)
    dimg = img.to(device, dtype=torch.float32).contiguous()
    dmsk = mask[0].to(device, dtype=torch.float32).contiguous()
    out = torch.empty(2, ny * nx, dtype=torch.int32, device=device)
    with torch.cuda.device(device):
        K.call("vu_patch_stats", K.ptr(dimg), img.shape[0], h, w, K.ptr(dmsk), patch, stride, ny, nx,
               K.ptr(out[0]), K.ptr(out[1]), K.stream())
    cnt = out.cpu().numpy().astype(np.int64)   # one D2H of 8 B per window
    return ny, nx, cnt[0], cnt[1]


def black_ratio_ok(black, patch, threshold):
    """is_valid_patch's test (data_loading.py:296-299): the fp32 mean of the
    per-pixel black flags (count / P^2, rounded to float32) <= threshold."""
    return float(np.float32(black) / np.float32(patch * patch)) <= threshold


def precompute_all_patches(ids, images_dir, masks_dir, patches_dir, split, scale, patch_size, lesion_type,
                           skip_border_check=False, rng=None, device="cuda"):
    """utils/data_loading.py:302-446 (patch mode): writes the cache files into
    ``patches_dir`` and returns the patch index [(img_id, path, has_lesion)]
    in the reference's order (positives in scan order, then the selected
    negatives for 'train'; every patch for 'val' / 'test')."""
    images_dir, masks_dir, patches_dir = Path(images_dir), Path(masks_dir), Path(patches_dir)
    rng = random if rng is None else rng
    threshold = 0.5 if split == "test" else 0.1
    positive_count, negative_paths, patch_index = 0, [], []
    stride = patch_size // 2
    for img_id in ids:
        img_file = images_dir / f"{img_id}.jpg"
        mask_file = masks_dir / lesion_type / f"{img_id}_{lesion_type}.tif"
        img_pil = load_image(img_file).convert("RGB")
        mask_pil = load_image(mask_file).convert("L")
        if img_pil.size != mask_pil.size:
            logging.warning(f"Mismatch in size for {img_file} vs {mask_file}; skipping.")
            continue
        img = torch.as_tensor(preprocess(img_pil, scale, False), dtype=torch.float32)
        msk = torch.as_tensor(preprocess(mask_pil, scale, True), dtype=torch.float32)
        if msk.dim() == 2:
            msk = msk.unsqueeze(0)
        if img.dim() == 2:
            img = img.unsqueeze(0)
        _, h, w = img.shape
        if h < patch_size or w < patch_size:
            logging.warning(f"{img_id}: scaled to {h}x{w} < patch_size={patch_size}; skipping.")
            continue
        ny, nx, black, lesion = window_stats(img, msk, patch_size, stride, device)
        count = 0
        for wi in range(ny * nx):
            y, x = (wi // nx) * stride, (wi % nx) * stride
            if not skip_border_check and img.shape[0] > 0 and not black_ratio_ok(black[wi], patch_size, threshold):
                continue
            has = bool(lesion[wi] > 0)
            path = patches_dir / f"{img_id}_{count}"
            torch.save({"image": img[:, y:y + patch_size, x:x + patch_size].contiguous(),
                        "mask": msk[:, y:y + patch_size, x:x + patch_size].contiguous(),
                        "coords": (y, x),
                        "has_lesion": torch.tensor(has)}, path)
            if has:
                positive_count += 1
                patch_index.append((img_id, str(path), True))
            else:
                negative_paths.append((img_id, str(path)))
            count += 1
    logging.info(f"Found {positive_count} positive patches and {len(negative_paths)} negative patches")
    if split == "train":
        rng.shuffle(negative_paths)
        patch_index += [(i, p, False) for i, p in negative_paths[:positive_count]]
        for _, p in negative_paths[positive_count:]:
            try:
                os.remove(p)
            except OSError as e:
                logging.warning(f"Error removing {p}: {e}")
        return patch_index
    index = patch_index + [(i, p, False) for i, p in negative_paths]
    if split == "test" and not index and positive_count == 0:
        index = [(i, p, False) for i, p in negative_paths[:min(10, len(negative_paths))]]
    return index


class IDRIDDataset(torch.utils.data.Dataset):
    """utils/data_loading.py:42-180 + 603-636 in patch mode: same constructor
    (plus ``ids`` to fix the image order — the reference takes
    ``os.listdir`` order —, ``rng`` for the balancing shuffle and the device
    of the window statistics), same cache directory
    (``base_dir/patches/split/lesion_type``, cleared first), same
    ``patch_indices`` and ``__getitem__`` records.  ``transform`` is None:
    the photometric augmentations are albumentations (absent); the geometric
    flips / rot90 run on the device in ``PatchCache(augment=True)``."""

    def __init__(self, base_dir, split="train", scale=0.25, patch_size=None, lesion_type="EX", max_images=None,
                 skip_border_check=False, ids=None, rng=None, device="cuda"):
        super().__init__()
        if patch_size is None:
            raise NotImplementedError("full-image mode needs cv2 fundus detection (data_loading.py:223-285), "
                                      "absent here: use patch_size")
        self.scale, self.split, self.patch_size = scale, split, patch_size
        self.base_dir = Path(base_dir)
        self.images_dir = self.base_dir / "imgs" / split
        self.masks_dir = self.base_dir / "masks" / split
        self.lesion_type = self.class_dir = lesion_type
        self.skip_border_check = skip_border_check
        self.is_full_image = False
        self.transform = None
        if ids is None:
            ids = [os.path.splitext(f)[0] for f in os.listdir(self.images_dir) if f.endswith(".jpg")]
            if max_images is not None:
                ids = ids[:max_images]
        ids = [i for i in ids if (self.masks_dir / lesion_type / f"{i}_{lesion_type}.tif").exists()]
        if not ids:
            raise RuntimeError(f"No valid image-mask pairs found in {self.images_dir} and {self.masks_dir}")
        self.ids = ids
        self.stride = patch_size // 2
        self.patches_dir = self.base_dir / "patches" / split / lesion_type
        if self.patches_dir.exists():
            import shutil
            shutil.rmtree(self.patches_dir)
        self.patches_dir.mkdir(parents=True, exist_ok=True)
        self.patch_indices = precompute_all_patches(ids, self.images_dir, self.masks_dir, self.patches_dir, split,
                                                    scale, patch_size, lesion_type, skip_border_check, rng, device)

    def __len__(self):
        return len(self.patch_indices)

    def __getitem__(self, idx):
        img_id, path, _ = self.patch_indices[idx]
        rec = load_patch(path)
        return {"image": rec["image"], "mask": rec["mask"], "img_id": img_id}

    def paths(self):
        """The cache files in index order (feed to PatchCache)."""
        return [p for _, p, _ in self.patch_indices]


# ----------------------------------------------------------------------------
# reader
# ----------------------------------------------------------------------------


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
