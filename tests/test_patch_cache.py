"""Patch-cache producer (vaeunet_amd.data.IDRIDDataset / precompute_all_patches)
against the reference's own IDRIDDataset.precompute_all_patches
(utils/data_loading.py:302-446), recorded by oracle/gen_golden.py on synthetic
JPEG / TIF files (tests/golden/patch_cache.npz holds the file bytes and the
reference's patch index, record coords / has_lesion / content checksums and
the files it left on disk after balancing).

CPU (not gpu): the oracle's window statistics and the host-side slicing,
naming, record format and balancing reproduce the fixture.  GPU: the same with
the device statistics kernel (vu_patch_stats), then the reader (PatchCache)
batches the produced files."""
import os
import random
import zlib

import numpy as np
import pytest
import torch

from golden_util import load

SPLITS = ("train", "val", "test")


def _materialise(rec, root):
    for i, f in enumerate(rec["files"]):
        p = os.path.join(root, str(f))
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "wb") as fh:
            fh.write(rec[f"file{i}"].tobytes())


def _check_split(rec, split, index, patches_dir):
    assert [os.path.basename(p) for _, p, _ in index] == [str(n) for n in rec[f"{split}.index_names"]]
    assert [bool(h) for _, _, h in index] == [bool(h) for h in rec[f"{split}.index_lesion"]]
    for k, (_, p, _) in enumerate(index):
        r = torch.load(p, weights_only=True)
        assert set(r) == {"image", "mask", "coords", "has_lesion"}
        assert tuple(r["coords"]) == tuple(int(v) for v in rec[f"{split}.coords"][k])
        assert r["has_lesion"].dtype == torch.bool and bool(r["has_lesion"]) == bool(rec[f"{split}.has_lesion"][k])
        assert r["image"].dtype == torch.float32 and r["image"].is_contiguous()
        assert float(r["image"].double().sum()) == float(rec[f"{split}.image_sum"][k])
        assert float(r["mask"].double().sum()) == float(rec[f"{split}.mask_sum"][k])
        crc = zlib.crc32(r["image"].numpy().tobytes()) ^ (zlib.crc32(r["mask"].numpy().tobytes()) << 1)
        assert crc == int(rec[f"{split}.crc"][k])
    assert sorted(os.listdir(patches_dir)) == [str(n) for n in rec[f"{split}.on_disk"]]


def _run(rec, root, device):
    from vaeunet_amd.data import IDRIDDataset
    out = {}
    for split in SPLITS:
        random.seed(int(rec["cfg.seed"]))
        ds = IDRIDDataset(root, split=split, scale=float(rec["cfg.scale"]), patch_size=int(rec["cfg.patch"]),
                          lesion_type=str(rec["cfg.lesion"]), ids=[str(i) for i in rec[f"{split}.ids"]],
                          device=device)
        _check_split(rec, split, ds.patch_indices, ds.patches_dir)
        out[split] = ds
    return out


def test_oracle_window_stats_and_host_logic_match_reference(tmp_path, monkeypatch):
    from oracle import cpu_ref as R
    import vaeunet_amd.data as D
    rec = load("patch_cache")
    _materialise(rec, tmp_path)

    def oracle_stats(img, mask, patch, stride, device):
        return R.patch_window_stats(img.numpy(), mask.numpy(), patch, stride)
    monkeypatch.setattr(D, "window_stats", oracle_stats)   # test-only: no device here
    ds = _run(rec, str(tmp_path), "cpu")
    assert len(ds["train"]) == 2 * int(np.sum(rec["train.index_lesion"]))   # balanced
    item = ds["val"][0]
    assert item["image"].shape == (3, 64, 64) and item["mask"].shape == (1, 64, 64)


def test_full_image_mode_refused():
    from vaeunet_amd.data import IDRIDDataset
    with pytest.raises(NotImplementedError):
        IDRIDDataset("/nonexistent", patch_size=None)


@pytest.mark.gpu
def test_device_producer_matches_reference_and_reader_batches(tmp_path):
    from vaeunet_amd.data import PatchCache
    rec = load("patch_cache")
    _materialise(rec, tmp_path)
    ds = _run(rec, str(tmp_path), "cuda")
    paths = ds["test"].paths()
    pc = PatchCache(paths, batch_size=8, device="cuda")
    seen = 0
    for b in pc:
        for k in range(b["image"].shape[0]):
            r = torch.load(paths[seen + k], weights_only=True)
            assert torch.equal(b["image"][k].cpu(), r["image"])
            assert torch.equal(b["mask"][k].cpu(), r["mask"])
            assert tuple(b["coords"][k]) == tuple(r["coords"])
        seen += b["image"].shape[0]
    assert seen == len(paths)


@pytest.mark.gpu
def test_device_window_stats_match_oracle_ragged():
    """Non-square, odd-sized image, odd patch and stride, 1- and 3-channel."""
    from oracle import cpu_ref as R
    from vaeunet_amd.data import window_stats
    g = torch.Generator().manual_seed(9)
    for C, H, W, P, st in ((3, 77, 131, 21, 10), (1, 40, 40, 40, 20), (3, 300, 97, 33, 16)):
        img = (torch.randint(0, 256, (C, H, W), generator=g).float() / 255.0)
        msk = (torch.rand(1, H, W, generator=g) < 0.02).float()
        got = window_stats(img, msk, P, st, "cuda")
        ref = R.patch_window_stats(img.numpy(), msk.numpy(), P, st)
        assert got[0] == ref[0] and got[1] == ref[1]
        np.testing.assert_array_equal(got[2], ref[2])
        np.testing.assert_array_equal(got[3], ref[3])
