"""On-disk formats, CPU side: the train.py:542-565
checkpoint dict round trip and raw state_dict loading (train.py:698-703), and
the flip/rot90 index maps of the patch-cache augmentation against numpy."""
import warnings

import numpy as np
import torch

from vaeunet_amd import UNet, UNetResNet
from vaeunet_amd.checkpoint import save_checkpoint, load_checkpoint
from vaeunet_amd.data import _flip_rot_map
from vaeunet_amd.init import seeded_init_


def test_checkpoint_dict_round_trip(tmp_path):
    m = seeded_init_(UNet(3, 1), 1)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=1e-5)
    for p in m.parameters():
        p.grad = torch.ones_like(p) * 1e-3
    opt.step()
    scaler = torch.amp.GradScaler("cpu", enabled=False)
    path = tmp_path / "best_model.pth"
    save_checkpoint(path, m, opt, None, scaler, epoch=3, best_val_score=0.5, global_step=7,
                    params={"model_type": "basic", "seed": 42})
    raw = torch.load(path, weights_only=True)
    assert set(raw) == {"epoch", "model_state_dict", "optimizer_state_dict", "scheduler_state_dict",
                        "best_val_score", "amp_scaler", "global_step", "params"}
    assert raw["epoch"] == 3 and raw["global_step"] == 7 and raw["params"]["seed"] == 42
    m2 = seeded_init_(UNet(3, 1), 2)
    opt2 = torch.optim.AdamW(m2.parameters(), lr=1e-4, weight_decay=1e-5)
    ck = load_checkpoint(path, m2, opt2)
    assert ck["best_val_score"] == 0.5
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k
    sa, sb = opt.state_dict()["state"], opt2.state_dict()["state"]
    assert sa.keys() == sb.keys() and all(torch.equal(sa[i]["exp_avg"], sb[i]["exp_avg"]) for i in sa)


def test_raw_state_dict_with_mask_values(tmp_path):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        m = seeded_init_(UNetResNet(3, 1, pretrained=False), 3)
        m2 = UNetResNet(3, 1, pretrained=False)
    sd = dict(m.state_dict())
    sd["mask_values"] = [0, 1]
    path = tmp_path / "raw.pth"
    torch.save(sd, path)
    load_checkpoint(path, m2)
    for k, v in m.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k]), k


def test_flip_rot90_maps_match_numpy():
    for P in (4, 7):
        img = np.arange(P * P).reshape(P, P)
        for hf in (0, 1):
            for vf in (0, 1):
                for k in range(4):
                    ref = img
                    if hf:
                        ref = ref[:, ::-1]
                    if vf:
                        ref = ref[::-1, :]
                    ref = np.rot90(ref, k)
                    m = _flip_rot_map(P, hf, vf, k)
                    out = np.array([[img[m[0] * i + m[1] * j + m[2], m[3] * i + m[4] * j + m[5]]
                                     for j in range(P)] for i in range(P)])
                    assert np.array_equal(out, ref), (P, hf, vf, k)
