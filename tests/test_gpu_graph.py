"""The captured-HIP-graph training step (vaeunet_amd/graph.py) against the
same steps run eagerly: identical kernels, so parameters and losses agree."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _setup(vae):
    from vaeunet_amd import UNet, UNetResNet
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
    from vaeunet_amd.optim import FusedAdamW
    torch.manual_seed(0)
    model = UNetResNet(3, 1, pretrained=False) if vae else UNet(3, 2)
    model = seeded_init_(model, 0).to(DEV).to(memory_format=torch.channels_last).train()
    opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-2)
    crit = CombinedLoss()
    g = torch.Generator().manual_seed(3)
    S = 64
    x = torch.rand(2, 3, S, S, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    if vae:
        t = (torch.rand(2, 1, S, S, generator=g) > 0.5).float().to(DEV)
        model.eps_override = torch.randn(2, model.latent_dim, generator=g).to(DEV)
    else:
        lab = torch.randint(0, 2, (2, S, S), generator=g)
        t = torch.nn.functional.one_hot(lab, 2).permute(0, 3, 1, 2).float().to(DEV)

    def fwd_bwd():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if vae:
                lg, mu, lv = model(x)
                loss = crit(lg, t) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
            else:
                loss = crit(model(x), t)
        loss.backward()
        return loss
    return model, opt, fwd_bwd


@pytest.mark.parametrize("vae", [False, True])
def test_graph_replay_matches_eager(vae):
    from vaeunet_amd.graph import GraphedTrainStep
    from vaeunet_amd.optim import clip_grad_norm_
    # eager: warmup 2 + 3 steps
    m1, o1, fb1 = _setup(vae)
    losses1 = []
    for i in range(5):
        loss = fb1()
        clip_grad_norm_(m1.parameters(), 1.0)
        o1.step()
        o1.zero_grad(set_to_none=True)
        if i >= 2:
            losses1.append(float(loss.detach()))
    # graph: the same 2 warm-up steps run eagerly inside, then 3 replays
    m2, o2, fb2 = _setup(vae)
    gs = GraphedTrainStep(fb2, o2, max_norm=1.0, warmup=2)
    losses2 = [float(gs.step().detach()) for _ in range(3)]
    torch.cuda.synchronize()
    for a, b in zip(losses1, losses2):
        assert abs(a - b) <= 1e-6 * max(1.0, abs(a)), (losses1, losses2)
    for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        torch.testing.assert_close(p2, p1, rtol=1e-6, atol=1e-7, msg=f"param {n}")
    gs.sync_optimizer_state()
    p0 = next(m2.parameters())
    assert float(o2.state[p0]["step"]) == 5.0


@pytest.mark.parametrize("vae", [False, True])
def test_eager_forward_after_replays_sees_updated_weights(vae):
    """Replays update the parameters behind autograd; the version bump in
    GraphedTrainStep.step() makes an eager (eval) forward afterwards rebuild its
    weight images: it must equal the same forward of the eagerly trained model."""
    from vaeunet_amd.graph import GraphedTrainStep
    from vaeunet_amd.optim import clip_grad_norm_
    m1, o1, fb1 = _setup(vae)
    for _ in range(4):
        fb1()
        clip_grad_norm_(m1.parameters(), 1.0)
        o1.step()
        o1.zero_grad(set_to_none=True)
    m2, o2, fb2 = _setup(vae)
    gs = GraphedTrainStep(fb2, o2, max_norm=1.0, warmup=2)
    for _ in range(2):
        gs.step()
    g = torch.Generator().manual_seed(11)
    xe = torch.rand(2, 3, 64, 64, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    outs = []
    for m in (m1, m2):
        m.eval()
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            o = m(xe)
        outs.append((o[0] if vae else o).float())
    torch.testing.assert_close(outs[1], outs[0], rtol=1e-5, atol=1e-5)
    # an eager optimizer step between replays continues the count and the graph
    # resumes from it
    m2.train()
    fb2()
    clip_grad_norm_([p for p in m2.parameters() if p.grad is not None], 1.0)
    o2.step()
    assert float(o2.state[next(m2.parameters())]["step"]) == 5.0
    gs.step()
    gs.sync_optimizer_state()
    assert float(o2.state[next(m2.parameters())]["step"]) == 6.0


def test_graph_with_unused_parameter():
    """latent_injection='none': UNetResNet's z_initial gets no gradient (use_bottleneck
    False); the graph leaves it out (no AdamW state, .grad None, no weight decay)
    exactly as torch's AdamW does."""
    from vaeunet_amd import UNetResNet
    from vaeunet_amd.graph import GraphedTrainStep
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
    from vaeunet_amd.optim import FusedAdamW
    model = seeded_init_(UNetResNet(3, 1, pretrained=False, latent_injection="none"), 0)
    model = model.to(DEV).to(memory_format=torch.channels_last).train()
    assert not model.use_bottleneck
    z0 = {n: p.detach().clone() for n, p in model.named_parameters() if n.startswith("z_initial")}
    opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-2)
    crit = CombinedLoss()
    g = torch.Generator().manual_seed(5)
    x = torch.rand(2, 3, 64, 64, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    t = (torch.rand(2, 1, 64, 64, generator=g) > 0.5).float().to(DEV)

    def fb():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lg, mu, lv = model(x)
            loss = crit(lg, t) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
        loss.backward()
        return loss
    gs = GraphedTrainStep(fb, opt, max_norm=1.0, warmup=1)
    losses = [float(gs.step()) for _ in range(3)]
    assert all(torch.isfinite(torch.tensor(losses)))
    for n, p in model.named_parameters():
        if n.startswith("z_initial"):
            assert p.grad is None
            torch.testing.assert_close(p.detach(), z0[n], rtol=0, atol=0)
