"""Host-side checks that need no GPU: drop-in surface (names, signatures,
state_dict keys and shapes), the C-ABI library exports, init determinism."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from golden_util import load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_unet_state_dict_matches_reference_keys():
    from vaeunet_amd import UNet
    for tag, nc, bil in [("unet_c1_64", 1, False), ("unet_c2_64", 2, False),
                         ("unet_c1_bilinear_64", 1, True)]:
        rec = load(tag)
        m = UNet(3, nc, bilinear=bil)
        names = [k for k, _ in m.named_parameters()]
        assert names == list(rec["names"])
    m = UNet(3, 2)
    assert len(m.state_dict()) == 202
    assert sum(p.numel() for p in m.parameters()) == 31389230
    assert sum(p.numel() for p in UNet(3, 2, bilinear=True).parameters()) == 17614574


def test_block_state_dicts_match_reference():
    import vaeunet_amd.unet_parts as P
    from vaeunet_amd.unet_resnet import DecoderBlock
    cases = {"doubleconv_8_16": P.DoubleConv(8, 16), "down_16_32": P.Down(16, 32),
             "up_64_32_convT": P.Up(64, 32, False), "up_64_32_bilinear": P.Up(64, 32, True),
             "attention_32_32_16": P.AttentionGate(32, 32, 16), "outconv_16_2": P.OutConv(16, 2),
             "decoder_64_32_48": DecoderBlock(64, 32, 48, 8, True, True, True),
             "decoder_noattn_64_32_48": DecoderBlock(64, 32, 48, 8, False, True, False)}
    for name, mod in cases.items():
        rec = load(name)
        ref = {k[3:]: v.shape for k, v in rec.items() if k.startswith("p0.")}
        mine = {k: tuple(v.shape) for k, v in mod.state_dict().items() if v.is_floating_point()}
        assert mine == {k: tuple(s) for k, s in ref.items()}, name


def test_unet_resnet_surface():
    from vaeunet_amd import UNetResNet
    m = UNetResNet(3, 1, pretrained=False)
    assert len(m.state_dict()) == 389
    assert sum(p.numel() for p in m.parameters()) == 30455789
    assert m.encoder.feature_info.channels() == [64, 64, 128, 256, 512]
    for attr in ("encoder", "mu_head", "logvar_head", "z_initial", "decoder_blocks", "final_conv",
                 "use_bottleneck", "use_skip", "use_attention", "latent_injection", "latent_dim",
                 "reparameterize", "encode", "decode"):
        assert hasattr(m, attr)
    assert not UNetResNet(3, 1, pretrained=False, latent_injection="none").use_bottleneck
    assert UNetResNet(3, 1, pretrained=False, latent_injection="bogus").latent_injection == "all"


def test_kl_annealer_matches_reference():
    from vaeunet_amd.loss import KLAnnealer
    rec = load("losses")
    a = KLAnnealer(kl_start=0.0, kl_end=1e-3, warmup_epochs=20)
    np.testing.assert_allclose([a.get_weight(e) for e in range(25)], rec["annealer"], rtol=1e-12)
    assert KLAnnealer(strategy="constant", kl_end=0.3).get_weight(3) == 0.3


def test_seeded_init_is_deterministic():
    from vaeunet_amd import UNet
    from vaeunet_amd.init import seeded_init_
    a = seeded_init_(UNet(3, 1), 5).state_dict()
    b = seeded_init_(UNet(3, 1), 5).state_dict()
    assert all(torch.equal(a[k], b[k]) for k in a)


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "vaeunet.h")).read()
    return sorted(set(re.findall(r"\b(vu_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from vaeunet_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    declared = _declared_symbols()
    assert declared, "no declarations parsed"
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    # every symbol the Python binding uses is declared in the header
    undeclared = [s for s in _lib.exported_symbols() if s not in declared]
    assert not undeclared, undeclared
    _lib.lib()  # resolves every signature


def test_abi_struct_sizes_match_the_binding():
    """The ctypes mirrors of the C-ABI descriptors have the compiled sizes (a
    field added on one side only would shift every later field)."""
    from vaeunet_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    out = (ctypes.c_int64 * 9)()
    lib.vu_abi_struct_sizes(out)
    mine = [ctypes.sizeof(c) for c in (_lib.VuGather, _lib.VuGemmFwd, _lib.VuGemmWgrad, _lib.VuConvFp8,
                                       _lib.VuPermJob, _lib.VuMtEntry, _lib.VuLatentJob, _lib.VuLatentHeads,
                                       _lib.VuZbJob)]
    assert list(out) == mine, (list(out), mine)


def test_product_path_has_no_oracle_or_fallback():
    pkg = os.path.join(ROOT, "vaeunet_amd")
    for fn in os.listdir(pkg):
        if fn.endswith(".py"):
            txt = open(os.path.join(pkg, fn)).read()
            assert "oracle" not in txt.replace("oracle/", "").replace("the oracle", ""), fn


def test_optim_dense_layout_check():
    """Host logic of the multi-tensor optimizer: which layouts walk as flat storage."""
    from vaeunet_amd.optim import _is_dense, FusedAdamW
    assert _is_dense(torch.empty(4, 3, 5, 5))
    assert _is_dense(torch.empty(4, 3, 5, 5).contiguous(memory_format=torch.channels_last))
    assert _is_dense(torch.empty(7))
    assert not _is_dense(torch.empty(4, 6)[:, :3])
    assert not _is_dense(torch.empty(4, 6).t()[::2])
    with pytest.raises(NotImplementedError):
        FusedAdamW([torch.nn.Parameter(torch.zeros(3))], amsgrad=True)
    opt = FusedAdamW([torch.nn.Parameter(torch.zeros(3))], lr=1e-4, weight_decay=1e-5)
    assert opt.param_groups[0]["betas"] == (0.9, 0.999) and opt.param_groups[0]["eps"] == 1e-8
