"""Patch-cache reader (vaeunet_amd/data.py) on the GPU: files in the
reference's cache format (utils/data_loading.py:381-388) come back as the
same batches on the device, and the device flip/rot90 augmentation equals
torch.flip / torch.rot90 on the same flags (image and mask alike)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _write_cache(tmp_path, n=7, P=16):
    g = torch.Generator().manual_seed(4)
    recs = []
    for i in range(n):
        img = torch.rand(3, P, P, generator=g)
        msk = (torch.rand(1, P, P, generator=g) < 0.1).float()
        rec = {"image": img.contiguous(), "mask": msk.contiguous(), "coords": (i, 2 * i),
               "has_lesion": torch.any(msk > 0.5)}
        torch.save(rec, tmp_path / f"IDRiD_{i:02d}_{i}")
        recs.append(rec)
    return recs


def test_patch_cache_batches(tmp_path):
    from vaeunet_amd.data import PatchCache
    recs = _write_cache(tmp_path)
    pc = PatchCache(str(tmp_path), batch_size=3, device="cuda")
    seen = 0
    for b in pc:
        n = b["image"].shape[0]
        assert b["image"].is_cuda and b["image"].is_contiguous(memory_format=torch.channels_last)
        for k in range(n):
            r = recs[seen + k]
            assert torch.equal(b["image"][k].cpu(), r["image"])
            assert torch.equal(b["mask"][k].cpu(), r["mask"])
            assert b["coords"][k] == r["coords"]
        seen += n
    assert seen == len(recs) and len(pc) == 3


def test_device_flip_rot90_matches_torch(tmp_path):
    from vaeunet_amd.data import PatchCache
    _write_cache(tmp_path, n=16)
    pc = PatchCache(str(tmp_path), batch_size=16, device="cuda")
    b = next(iter(pc))
    flags = [(h, v, k) for h in (0, 1) for v in (0, 1) for k in range(4)][:16]
    img, msk, _ = pc.augment_batch(b["image"], b["mask"], flags)
    for i, (h, v, k) in enumerate(flags):
        for src, got in ((b["image"][i], img[i]), (b["mask"][i], msk[i])):
            ref = src
            if h:
                ref = torch.flip(ref, (2,))
            if v:
                ref = torch.flip(ref, (1,))
            ref = torch.rot90(ref, k, (1, 2))
            assert torch.equal(got.cpu(), ref.cpu()), (h, v, k)
