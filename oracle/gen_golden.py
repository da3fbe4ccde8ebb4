"""Golden-vector generator — TEST INFRASTRUCTURE, runs only in the build container.

Imports the reference (``/root/reference``, read-only) and records small
input/output/gradient fixtures under ``tests/golden/*.npz``.  Nothing here
ships to the GPU box as code: only the ``.npz`` data travels.  The reference
modules imported are

* ``unet.unet_parts``  (AttentionGate 7-30, DoubleConv 32-49, Down 51-63,
  Up 65-95, OutConv 97-103)
* ``unet.unet_model.UNet`` (6-36)
* ``utils.loss``  (dice_loss 6-28, CombinedLoss 44-63, KLAnnealer 114-145,
  kl_with_free_bits 148-170)
* ``utils.metrics.dice_score`` (8-35)
* ``unet/unet_resnet.py``: ``timm`` (requirements.txt:2, timm~=1.0.13) is
  absent here, so the module cannot be imported.  ``DecoderBlock`` (31-101),
  ``AttentionGate`` (6-29) and ``UNetResNet`` (103-279) are compiled from the
  reference file's AST *without* the ``import timm`` line.  For
  ``UNetResNet`` the name ``timm`` is bound to a TEST DOUBLE whose
  ``create_model`` returns a module that ignores its input and returns five
  fixed, seeded feature maps (leaf parameters, so their gradients are
  recorded) with ``feature_info.channels() == [64, 64, 128, 256, 512]``; it
  restates nothing of timm.  ``torch.randn_like`` is patched to return a
  fixture ``eps`` during those runs.  This pins everything after the encoder
  (heads 140-147, reparameterize 191-194, injection modes 157-175/210-234,
  DecoderBlocks, final conv + interpolate 237-238); the ResNet34 encoder's
  own arithmetic stays parity-unpinned.

The train-step golden restates ``train.py:381-411`` (the reference's own
``train.py`` needs wandb/torchvision and cannot be imported) using the
reference's own model and loss objects and ``torch.optim.AdamW`` exactly as
``train.py:334`` configures it.

Usage:  python oracle/gen_golden.py   (writes tests/golden/*.npz)
"""
import ast
import os
import sys

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)
sys.path.insert(0, REF)

from vaeunet_amd.init import seeded_init_  # noqa: E402
sys.path.insert(0, os.path.join(REPO, "tests"))
from golden_util import (_rand, seed_vae_tail, vae_feature, vae_feature_shapes,  # noqa: E402
                         vae_eps, vae_target, pyramid_encoder, seed_bn_stats, infer_inputs,
                         INFER_SEED, INFER_GEN, INFER_PATCH)
from unet.unet_parts import AttentionGate, DoubleConv, Down, Up, OutConv  # noqa: E402
from unet.unet_model import UNet  # noqa: E402
from utils.loss import dice_loss, CombinedLoss, KLAnnealer, kl_with_free_bits  # noqa: E402
from utils.metrics import dice_score  # noqa: E402

torch.set_num_threads(8)
torch.use_deterministic_algorithms(True)


def _t(a, cl=False):
    t = torch.from_numpy(np.ascontiguousarray(a))
    return t.to(memory_format=torch.channels_last) if cl and t.dim() == 4 else t


def _np(t):
    return t.detach().contiguous().cpu().numpy().copy()


def _load_decoder_block():
    """Compile DecoderBlock/AttentionGate from unet/unet_resnet.py without `import timm`."""
    path = os.path.join(REF, "unet", "unet_resnet.py")
    src = open(path).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, ast.ClassDef)
            and n.name in ("AttentionGate", "DecoderBlock")]
    mod = ast.Module(body=keep, type_ignores=[])
    ns = {"torch": torch, "nn": nn, "F": F}
    exec(compile(mod, path, "exec"), ns)
    return ns["DecoderBlock"]


class _FeatureInfo:
    def channels(self):
        return [64, 64, 128, 256, 512]


class FixedFeatures(nn.Module):
    """Test double standing in for ``timm.create_model(..., features_only=True)``:
    returns five seeded feature maps, whatever the input."""

    def __init__(self, shapes, seed):
        super().__init__()
        self.f = nn.ParameterList([nn.Parameter(torch.from_numpy(vae_feature(shape, seed, i)))
                                   for i, shape in enumerate(shapes)])
        self.feature_info = _FeatureInfo()

    def forward(self, x):
        return [f for f in self.f]


def _load_unet_resnet(stub_factory):
    path = os.path.join(REF, "unet", "unet_resnet.py")
    tree = ast.parse(open(path).read())
    keep = [n for n in tree.body if isinstance(n, ast.ClassDef)]
    mod = ast.Module(body=keep, type_ignores=[])

    class _TimmDouble:
        @staticmethod
        def create_model(backbone, pretrained=False, features_only=True, in_chans=3, **kw):
            return stub_factory()

    ns = {"torch": torch, "nn": nn, "F": F, "timm": _TimmDouble}
    exec(compile(mod, path, "exec"), ns)
    return ns["UNetResNet"]


def gen_vae(mode, B=2, S=256, seed=300):
    """UNetResNet train-step fixture (fp64 reference run) with a fixed-feature
    encoder double and a fixture eps; fixtures regenerable from seeds
    (features, target, eps, parameters) are NOT stored, only outputs."""
    shapes = vae_feature_shapes(B, S)
    UNetResNet = _load_unet_resnet(lambda: FixedFeatures(shapes, seed))
    torch.manual_seed(0)
    model = UNetResNet(3, 1, pretrained=False, latent_injection=mode)
    seed_vae_tail(model, seed)
    model = model.double().train()
    eps = vae_eps(B, seed).astype(np.float64)
    target = vae_target(B, S, seed).astype(np.float64)
    x = torch.zeros(B, 3, S, S, dtype=torch.float64)
    real = torch.randn_like
    torch.randn_like = lambda t, **kw: torch.from_numpy(eps).to(t.dtype)
    try:
        out, mu, logvar = model(x)
    finally:
        torch.randn_like = real
    crit = CombinedLoss()
    loss = crit(out, torch.from_numpy(target)) + 1e-3 * kl_with_free_bits(mu, logvar, free_bits=1e-3)
    loss.backward()
    rec = {"out": _np(out).astype(np.float32), "mu": _np(mu), "logvar": _np(logvar),
           "loss": np.float64(loss.item()), "B": np.int64(B), "S": np.int64(S), "seed": np.int64(seed)}
    names, norms, heads = [], [], []
    for k, p in model.named_parameters():
        if k.startswith("encoder."):
            continue
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        names.append(k)
        norms.append(float(g.norm()))
        heads.append(_np(g).reshape(-1)[:16])
    rec["names"] = np.array(names)
    rec["gnorm"] = np.array(norms, np.float64)
    rec["ghead"] = np.stack([np.pad(h, (0, 16 - len(h))) for h in heads])
    rec["fgnorm"] = np.array([float(f.grad.norm()) if f.grad is not None else 0.0
                              for f in model.encoder.f], np.float64)
    rec["fghead"] = np.stack([_np(f.grad).reshape(-1)[:16] if f.grad is not None else np.zeros(16)
                              for f in model.encoder.f])
    for k, b in model.named_buffers():
        if "running" in k:
            rec[f"buf.{k}"] = _np(b)
    np.savez_compressed(os.path.join(OUT, f"vae_{mode}_{S}.npz"), **rec)
    print(f"vae_{mode}_{S}: loss {loss.item():.6f} |mu| {float(mu.abs().mean()):.4f}")


def record_module(name, module, inputs, seed, cl=True):
    """Forward (train mode) + backward with a seeded grad_output."""
    seeded_init_(module, seed)
    module.train()
    state = {k: _np(v) for k, v in module.state_dict().items()
             if v.dtype.is_floating_point}
    ins = [_t(a, cl).requires_grad_(True) for a in inputs]
    if cl:
        module = module.to(memory_format=torch.channels_last)
    out = module(*ins)
    gout = _rand(seed + 1000, tuple(out.shape))
    out.backward(_t(gout, cl))
    rec = {"out": _np(out), "gout": gout}
    for i, (a, t) in enumerate(zip(inputs, ins)):
        rec[f"in{i}"] = a
        rec[f"gin{i}"] = _np(t.grad) if t.grad is not None else np.zeros_like(a)
    for k, v in state.items():
        rec[f"p0.{k}"] = v
    for k, p in module.named_parameters():
        rec[f"grad.{k}"] = _np(p.grad)
    for k, b in module.named_buffers():
        rec[f"buf.{k}"] = _np(b)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **rec)
    print(f"{name}: out {tuple(out.shape)}  |out|={float(out.detach().abs().mean()):.4f}")


def gen_parts():
    record_module("doubleconv_8_16", DoubleConv(8, 16), [_rand(1, (2, 8, 16, 16))], 11)
    record_module("doubleconv_3_16_mid8", DoubleConv(3, 16, 8), [_rand(2, (2, 3, 12, 12))], 12)
    record_module("down_16_32", Down(16, 32), [_rand(3, (2, 16, 16, 16))], 13)
    record_module("down_odd_16_32", Down(16, 32), [_rand(4, (2, 16, 11, 9))], 14)
    record_module("up_64_32_convT", Up(64, 32, bilinear=False),
                  [_rand(5, (2, 64, 4, 4)), _rand(6, (2, 32, 8, 8))], 15)
    record_module("up_64_32_bilinear", Up(64, 32, bilinear=True),
                  [_rand(7, (2, 32, 4, 4)), _rand(8, (2, 32, 8, 8))], 16)
    record_module("up_odd_64_32_convT", Up(64, 32, bilinear=False),
                  [_rand(9, (2, 64, 4, 4)), _rand(10, (2, 32, 9, 10))], 17)
    record_module("up_odd_64_32_bilinear", Up(64, 32, bilinear=True),
                  [_rand(18, (2, 32, 5, 4)), _rand(19, (2, 32, 11, 9))], 20)
    record_module("attention_32_32_16", AttentionGate(32, 32, 16),
                  [_rand(21, (2, 32, 8, 8)), _rand(22, (2, 32, 8, 8))], 23)
    record_module("outconv_16_2", OutConv(16, 2), [_rand(24, (2, 16, 8, 8))], 25)
    DecoderBlock = _load_decoder_block()
    record_module("decoder_64_32_48", DecoderBlock(64, 32, 48, 8, True, True, True),
                  [_rand(26, (2, 64, 4, 4)), _rand(27, (2, 32, 8, 8)),
                   _rand(28, (2, 8, 1, 1))], 29)
    record_module("decoder_noattn_64_32_48", DecoderBlock(64, 32, 48, 8, False, True, False),
                  [_rand(30, (2, 64, 4, 4)), _rand(31, (2, 32, 8, 8)),
                   _rand(32, (2, 8, 1, 1))], 33)


def gen_losses():
    rec = {}
    cases = {
        "a": (_rand(40, (2, 1, 16, 16), -4, 4), (_rand(41, (2, 1, 16, 16), 0, 1) < 0.1)),
        "b": (_rand(42, (3, 1, 8, 8), -9, 9), (_rand(43, (3, 1, 8, 8), 0, 1) < 0.5)),
        "empty": (_rand(44, (2, 1, 8, 8), -8, -2), np.zeros((2, 1, 8, 8), bool)),
        "c2": (_rand(45, (2, 2, 8, 8), -3, 3), (_rand(46, (2, 2, 8, 8), 0, 1) < 0.2)),
    }
    crit = CombinedLoss()
    for k, (lg, tg) in cases.items():
        tg = tg.astype(np.float32)
        x = _t(lg).requires_grad_(True)
        loss = crit(x, _t(tg))
        loss.backward()
        rec[f"{k}.logits"], rec[f"{k}.target"] = lg, tg
        rec[f"{k}.loss"] = np.float32(loss.item())
        rec[f"{k}.grad"] = _np(x.grad)
        rec[f"{k}.dice_loss"] = np.float32(dice_loss(_t(lg), _t(tg)).item())
        rec[f"{k}.bce"] = np.float32(F.binary_cross_entropy_with_logits(_t(lg), _t(tg)).item())
        rec[f"{k}.dice_score"] = np.float32(dice_score(_t(lg), _t(tg)).item())
    # KL with free bits: include exact ties with free_bits and clamp saturation.
    mu = _rand(50, (4, 8), -2, 2)
    lv = _rand(51, (4, 8), -3, 3)
    mu[0, 0], lv[0, 0] = 0.0, 0.0           # kl == 0  -> below free bits
    mu[1, 1], lv[1, 1] = 30.0, 0.0          # kl = 450 -> clamped at 100
    lv[2, 2] = 6.0                          # large logvar
    for fb in (1e-3, 1e-4, 0.0, 0.5):
        m = _t(mu).requires_grad_(True)
        v = _t(lv).requires_grad_(True)
        kl = kl_with_free_bits(m, v, free_bits=fb)
        kl.backward()
        tag = f"kl_fb{fb:g}"
        rec[f"{tag}.value"] = np.float32(kl.item())
        rec[f"{tag}.gmu"] = _np(m.grad)
        rec[f"{tag}.glogvar"] = _np(v.grad)
    rec["kl.mu"], rec["kl.logvar"] = mu, lv
    ann = KLAnnealer(kl_start=0.0, kl_end=1e-3, warmup_epochs=20)
    rec["annealer"] = np.array([ann.get_weight(e) for e in range(0, 25)], np.float64)
    np.savez_compressed(os.path.join(OUT, "losses.npz"), **rec)
    print("losses: ok")


def _grad_summary(model, rec, prefix):
    names, norms, heads = [], [], []
    for k, p in model.named_parameters():
        names.append(k)
        norms.append(float(p.grad.double().norm()))
        heads.append(_np(p.grad).reshape(-1)[:16])
    rec[f"{prefix}names"] = np.array(names)
    rec[f"{prefix}gnorm"] = np.array(norms, np.float64)
    rec[f"{prefix}ghead"] = np.stack([np.pad(h, (0, 16 - len(h))) for h in heads])


def gen_unet(n_classes, bilinear, tag, batch=2, size=64, steps=1):
    """Tiny-config train step (train.py:381-411) on the reference UNet."""
    torch.manual_seed(0)
    model = UNet(3, n_classes, bilinear=bilinear)
    seeded_init_(model, 0)
    model = model.to(memory_format=torch.channels_last).train()
    x = _rand(100, (batch, 3, size, size), 0.0, 1.0)
    m = (_rand(101, (batch, 1, size, size), 0, 1) < 0.05).astype(np.float32)
    if n_classes == 2:
        target = np.concatenate([1.0 - m, m], axis=1).astype(np.float32)
    else:
        target = m
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-5)
    crit = CombinedLoss()
    rec = {"x": x, "target": target}
    xs = _t(x, cl=True)
    logits = model(xs)
    # dice_loss does .view(-1): channels_last output with C>1 cannot be viewed
    # (SURVEY appendix); the C=2 golden uses contiguous logits.
    lg = logits.contiguous() if n_classes > 1 else logits
    loss = crit(lg, _t(target))
    loss.backward()
    rec["logits"] = _np(logits)
    rec["argmax"] = _np(logits.argmax(1)) if n_classes > 1 else _np(logits > 0)
    rec["loss"] = np.float32(loss.item())
    _grad_summary(model, rec, "")
    total = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    rec["total_norm"] = np.float32(total.item())
    opt.step()
    opt.zero_grad(set_to_none=True)
    for k, v in model.state_dict().items():
        if "running" in k or "num_batches" in k:
            rec[f"buf.{k}"] = _np(v)
    heads = [(_np(p).reshape(-1)[:16]) for _, p in model.named_parameters()]
    rec["p1head"] = np.stack([np.pad(h, (0, 16 - len(h))) for h in heads])
    # second forward (after the update) in eval mode: running-stat path
    model.eval()
    with torch.no_grad():
        rec["eval_logits"] = _np(model(xs))
    np.savez_compressed(os.path.join(OUT, f"{tag}.npz"), **rec)
    print(f"{tag}: loss {rec['loss']:.6f} total_norm {rec['total_norm']:.6f}")


def _load_visualize_fns():
    """predict_full_image (61-87), calculate_uncertainty_metrics (90-117),
    predict_with_patches (243-415) compiled from visualize_vae.py's AST (the
    module itself imports matplotlib/psutil/timm-dependent code)."""
    import logging
    import math
    path = os.path.join(REF, "visualize_vae.py")
    tree = ast.parse(open(path).read())
    want = ("predict_full_image", "calculate_uncertainty_metrics", "predict_with_patches")
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in want]
    ns = {"torch": torch, "F": F, "math": math, "logging": logging, "np": np}
    exec(compile(ast.Module(body=keep, type_ignores=[]), path, "exec"), ns)
    return [ns[k] for k in want]


def gen_inference():
    """Inference sampling path fixtures from the reference's
    own functions: utils/vae_utils.generate_predictions / encode_images and
    visualize_vae.predict_full_image / predict_with_patches /
    calculate_uncertainty_metrics, on the reference UNetResNet with an
    input-dependent encoder TEST DOUBLE (golden_util.pyramid_encoder) and
    seeded eval-mode BatchNorm statistics; randn_like patched to fixture eps."""
    from utils.vae_utils import generate_predictions, encode_images
    predict_full_image, calculate_uncertainty_metrics, predict_with_patches = _load_visualize_fns()
    UNetResNet = _load_unet_resnet(lambda: pyramid_encoder(INFER_SEED))
    torch.manual_seed(0)
    model = UNetResNet(3, 1, pretrained=False, latent_injection="all")
    seed_vae_tail(model, INFER_SEED)
    seed_bn_stats(model, INFER_SEED + 50)
    model.eval()
    inp = infer_inputs()
    rec = {}
    imgs = torch.from_numpy(inp["gen_images"])
    mu, lv = encode_images(model, imgs)
    rec["enc_mu"], rec["enc_logvar"] = _np(mu), _np(lv)
    draws = iter([torch.from_numpy(e) for e in inp["gen_eps"]])
    real = torch.randn_like
    torch.randn_like = lambda t, **kw: next(draws).to(t.dtype)
    try:
        rec["gen_out"] = _np(generate_predictions(model, imgs, temperature=INFER_GEN["temperature"],
                                                  num_samples=INFER_GEN["samples"]))
    finally:
        torch.randn_like = real
    rec["full_out"] = _np(predict_full_image(model, torch.from_numpy(inp["full_img"]),
                                             torch.from_numpy(inp["full_z"])))
    rec["patch_out"] = _np(predict_with_patches(model, torch.from_numpy(inp["patch_img"]),
                                                torch.from_numpy(inp["patch_z"]), INFER_PATCH["patch"], None,
                                                INFER_PATCH["batch"]))
    unc = calculate_uncertainty_metrics(torch.from_numpy(inp["segs"]))
    for k, v in unc.items():
        rec[f"unc_{k}"] = _np(v)
    np.savez_compressed(os.path.join(OUT, "inference.npz"), **rec)
    print("inference:", {k: v.shape for k, v in rec.items()})


PATCH_CFG = {"patch": 64, "scale": 0.25, "seed": 1234, "lesion": "EX"}


def _synthetic_idrid(root, seed=5):
    """Small fundus-like JPEG images + TIF lesion masks in the reference's
    directory layout (imgs/<split>/*.jpg, masks/<split>/EX/*_EX.tif): a bright
    textured disc on a black background (border rejection), lesion blobs,
    plus one image too small for the patch and one with a mismatched mask
    (both skipped by the reference)."""
    from PIL import Image
    rng = np.random.Generator(np.random.PCG64(seed))
    layout = {"train": 4, "val": 2, "test": 2}
    for split, n in layout.items():
        os.makedirs(os.path.join(root, "imgs", split), exist_ok=True)
        os.makedirs(os.path.join(root, "masks", split, "EX"), exist_ok=True)
        for i in range(n + 1):
            H, W = (720, 1040) if i < n else ((200, 200) if split != "train" else (720, 1040))
            yy, xx = np.mgrid[0:H, 0:W]
            cy, cx = H / 2 + rng.uniform(-30, 30), W / 2 + rng.uniform(-60, 60)
            r = min(H, W) * rng.uniform(0.42, 0.5)
            disc = ((yy - cy) ** 2 + (xx - cx) ** 2) < r * r
            base = np.stack([rng.uniform(120, 200), rng.uniform(40, 90), rng.uniform(10, 40)])
            tex = rng.normal(0, 12, (H // 8 + 1, W // 8 + 1, 3)).repeat(8, 0).repeat(8, 1)[:H, :W]
            img = np.clip(base[None, None, :] + tex, 0, 255) * disc[..., None]
            # a few dark-but-not-black pixels around the 0.1 mean threshold
            img[:, :40] = np.array([25, 26, 26])[None, None, :] * (rng.random((H, 40, 1)) < 0.5)
            m = np.zeros((H, W), np.uint8)
            for _ in range(int(rng.integers(2, 6))):
                ly, lx = rng.integers(0, H), rng.integers(0, W)
                rr = rng.uniform(6, 30)
                m[((yy - ly) ** 2 + (xx - lx) ** 2) < rr * rr] = 255
            name = f"IDRiD_{split}_{i:02d}"
            Image.fromarray(img.astype(np.uint8)).save(os.path.join(root, "imgs", split, name + ".jpg"), quality=92)
            if split == "train" and i == n:
                m = m[:, :-8]    # mismatched mask size: skipped
            Image.fromarray(m).save(os.path.join(root, "masks", split, "EX", f"{name}_EX.tif"))
    return layout


def _load_idrid_slicer():
    """IDRIDDataset.is_valid_patch (287-300), precompute_all_patches (302-446)
    and preprocess (580-601) plus load_image (18-28), compiled from
    utils/data_loading.py's AST (the module imports albumentations and cv2 at
    the top, both absent; none of these methods touches them) onto a bare
    class: the reference's own slicing, border rejection, record format and
    positive/negative balancing."""
    import logging
    import random
    from pathlib import Path
    from PIL import Image
    path = os.path.join(REF, "utils", "data_loading.py")
    tree = ast.parse(open(path).read())
    fns = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "load_image"]
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "IDRIDDataset")
    want = ("is_valid_patch", "precompute_all_patches", "preprocess")
    body = [n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name in want]
    slicer = ast.copy_location(ast.ClassDef(name="IDRIDSlicer", bases=[], keywords=[], body=body,
                                            decorator_list=[]), cls)
    mod = ast.fix_missing_locations(ast.Module(body=fns + [slicer], type_ignores=[]))
    ns = {"torch": torch, "np": np, "Image": Image, "logging": logging, "os": os, "random": random,
          "Path": Path, "tqdm": lambda it, **kw: it}
    exec(compile(mod, path, "exec"), ns)
    return ns["IDRIDSlicer"]


def gen_patch_cache():
    """Patch-cache producer fixture: the reference's own
    precompute_all_patches run on synthetic images; stores the input FILES
    (bytes) and, per split, the resulting patch index and every kept record's
    coords / has_lesion / content checksums, and the files left on disk."""
    import random
    import tempfile
    import zlib
    from pathlib import Path
    Slicer = _load_idrid_slicer()
    rec = {}
    with tempfile.TemporaryDirectory() as root:
        layout = _synthetic_idrid(root)
        files = []
        for dp, _, fs in os.walk(root):
            for f in sorted(fs):
                files.append(os.path.relpath(os.path.join(dp, f), root))
        files.sort()
        rec["files"] = np.array(files)
        for i, f in enumerate(files):
            rec[f"file{i}"] = np.frombuffer(open(os.path.join(root, f), "rb").read(), np.uint8)
        P, lt = PATCH_CFG["patch"], PATCH_CFG["lesion"]
        for split in layout:
            s = Slicer.__new__(Slicer)
            s.split, s.scale, s.patch_size, s.lesion_type = split, PATCH_CFG["scale"], P, lt
            s.is_full_image, s.skip_border_check, s.stride = False, False, P // 2
            s.images_dir = Path(root) / "imgs" / split
            s.masks_dir = Path(root) / "masks" / split
            s.ids = sorted(os.path.splitext(f)[0] for f in os.listdir(s.images_dir) if f.endswith(".jpg"))
            s.patches_dir = Path(root) / "patches" / split / lt
            s.patches_dir.mkdir(parents=True, exist_ok=True)
            random.seed(PATCH_CFG["seed"])
            s.precompute_all_patches()
            rec[f"{split}.ids"] = np.array(s.ids)
            rec[f"{split}.index_names"] = np.array([os.path.basename(p) for _, p, _ in s.patch_indices])
            rec[f"{split}.index_lesion"] = np.array([bool(h) for _, _, h in s.patch_indices])
            coords, has, isum, msum, crc = [], [], [], [], []
            for _, p, _ in s.patch_indices:
                r = torch.load(p, weights_only=True)
                coords.append(tuple(r["coords"]))
                has.append(bool(r["has_lesion"]))
                isum.append(float(r["image"].double().sum()))
                msum.append(float(r["mask"].double().sum()))
                crc.append(zlib.crc32(r["image"].numpy().tobytes()) ^ (zlib.crc32(r["mask"].numpy().tobytes()) << 1))
            rec[f"{split}.coords"] = np.array(coords, np.int64).reshape(-1, 2)
            rec[f"{split}.has_lesion"] = np.array(has)
            rec[f"{split}.image_sum"] = np.array(isum)
            rec[f"{split}.mask_sum"] = np.array(msum)
            rec[f"{split}.crc"] = np.array(crc, np.int64)
            rec[f"{split}.on_disk"] = np.array(sorted(os.listdir(s.patches_dir)))
            print(f"patch_cache {split}: {len(s.patch_indices)} patches "
                  f"({int(np.sum(rec[split + '.index_lesion']))} positive), {len(rec[split + '.on_disk'])} on disk")
    for k, v in PATCH_CFG.items():
        rec[f"cfg.{k}"] = np.array(v)
    np.savez_compressed(os.path.join(OUT, "patch_cache.npz"), **rec)


def gen_decoder_spatial():
    """DecoderBlock with the reference's spatial z [B, L, h, w] (not constant)."""
    DecoderBlock = _load_decoder_block()
    record_module("decoder_zspatial_64_32_48", DecoderBlock(64, 32, 48, 8, True, True, True),
                  [_rand(34, (2, 64, 4, 4)), _rand(35, (2, 32, 8, 8)), _rand(36, (2, 8, 3, 3))], 37)


if __name__ == "__main__":
    # python oracle/gen_golden.py [parts losses unet vae decoder_spatial]  (default: all)
    os.makedirs(OUT, exist_ok=True)
    what = set(sys.argv[1:]) or {"parts", "losses", "unet", "vae", "decoder_spatial", "inference", "patch_cache"}
    if "parts" in what:
        gen_parts()
    if "losses" in what:
        gen_losses()
    if "unet" in what:
        gen_unet(1, False, "unet_c1_64")
        gen_unet(2, False, "unet_c2_64")
        gen_unet(1, True, "unet_c1_bilinear_64")
    if "decoder_spatial" in what:
        gen_decoder_spatial()
    if "vae" in what:
        for mode in ("all", "none", "first", "bottleneck"):
            gen_vae(mode)
    if "inference" in what:
        gen_inference()
    if "patch_cache" in what:
        gen_patch_cache()
