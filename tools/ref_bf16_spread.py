"""The reference's own CPU-bf16 per-parameter BatchNorm-affine gradient drift
against its fp32 path, for the bench input and two copies perturbed below bf16
resolution (2^-12, 2^-10 relative): the spread the config-3 bf16 test's
ensemble yardstick is built from (profiles/r5_ref_bf16_spread.log).  CPU only;
test infrastructure (imports oracle/)."""
import sys, time, torch
import os
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
torch.set_num_threads(8)
from oracle import cpu_ref as R
from vaeunet_amd import UNetResNet
from vaeunet_amd.init import seeded_init_
B,S=8,512
g = torch.Generator().manual_seed(1000)
x = torch.rand(B, 3, S, S, generator=g)
m = (torch.rand(B, 1, S, S, generator=g) < 0.0085).float()
eps = torch.randn(B, 32, generator=torch.Generator().manual_seed(77))
model = seeded_init_(UNetResNet(3, 1, pretrained=False), 0)
state = model.state_dict()
names=[k for k,p in model.named_parameters() if p.dim()==1]
def run(xx, ac):
    ref = R.UNetResNetRef(state)
    if ac:
        with torch.autocast("cpu", dtype=torch.bfloat16):
            lg, mu, lv = ref.forward(xx, eps, True)
            loss = R.combined_loss(lg.float(), m) + 1e-3 * R.kl_with_free_bits(mu.float(), lv.float(), 1e-3)
    else:
        lg, mu, lv = ref.forward(xx, eps, True)
        loss = R.combined_loss(lg, m) + 1e-3 * R.kl_with_free_bits(mu, lv, 1e-3)
    loss.backward()
    return {k: float(ref.p[k].grad.double().norm()) for k in names if ref.p[k].grad is not None}
t0=time.time()
g32=run(x,False); print('fp32', time.time()-t0, flush=True)
g16=run(x,True); print('bf16', time.time()-t0, flush=True)
r = torch.rand(x.shape, generator=torch.Generator().manual_seed(5))*2-1
outs=[]
for i,sc in enumerate([2**-12, 2**-10]):
    xp = x*(1+sc*r)
    outs.append(run(xp,True)); print('bf16 pert', sc, time.time()-t0, flush=True)
print("%-45s %8s %8s %8s"%("param","bf16","pert12","pert10"))
for k in names:
    if k not in g32 or not k.startswith("encoder"): continue
    ref=g32[k]
    print("%-45s %8.3f %8.3f %8.3f"%(k, abs(g16[k]-ref)/ref, abs(outs[0][k]-ref)/ref, abs(outs[1][k]-ref)/ref))
