"""Compare one eager vs one graphed Phase-6 micro-batch on the full bench model (no optimizer step)."""
import os, sys, random
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "robust-audio-deepfake-evolution_amd")); sys.path.insert(0, ROOT)
import numpy as np, torch
from radhip.build import apply_lora_to_wavlm, get_model, load_config
from radhip.train import Trainer, GraphedMicroStep
dev = torch.device("cuda", 0)
cfg = load_config("Phase6_Proposed.conf"); cfg["training_config"]["accumulation_steps"] = 100
torch.manual_seed(1234)
m = apply_lora_to_wavlm(get_model(cfg["model_config"], dev), cfg["training_config"])
m.wavlm_stream._core().config.layerdrop = 0.0
tr = Trainer(m, cfg, dev, total_steps=1000)
B = 8
rng = np.random.default_rng(0)
x = torch.from_numpy(np.clip(0.1 * rng.standard_normal((B, 64600)), -1, 1).astype(np.float32)).to(dev)
y = np.array([0, 1, 0, 0, 1, 0, 0, 0])
def snap():
    torch.cuda.synchronize()
    return tr.grads.flat.clone(), float(tr.loss_sum)
def eager(seed):
    np.random.seed(seed); random.seed(seed); torch.manual_seed(seed)
    lam, perm = tr.mixup_draw(B)
    xm = lam * x + (1 - lam) * x[torch.tensor(perm, device=dev)]
    tr.micro_step(xm, torch.from_numpy(y), lam, perm)
    return snap()
tr.grads.zero(); tr.loss_sum.zero_()
ge, le = eager(5)
print("eager loss", le, "grad norm", float(ge.norm()), "nan", bool(torch.isnan(ge).any()))
tr.grads.zero(); tr.loss_sum.zero_()
ge2, le2 = eager(5)
print("eager again loss", le2, "max|dg|", float((ge2 - ge).abs().max()), "rel", float((ge2-ge).norm()/ge.norm()))
g = GraphedMicroStep(tr, B)
g.capture()
tr.grads.zero(); tr.loss_sum.zero_()
np.random.seed(5); random.seed(5); torch.manual_seed(5)
lam, perm = tr.mixup_draw(B)
g.x.copy_(lam * x + (1 - lam) * x[torch.tensor(perm, device=dev)])
g.run(y, lam, perm)
gg, lg = snap()
print("graph loss", lg, "grad norm", float(gg.norm()), "nan", bool(torch.isnan(gg).any()),
      "rel vs eager", float((gg - ge).norm() / ge.norm()))
# per-parameter comparison
off = 0
bad = []
for n, p in m.named_parameters():
    if not p.requires_grad: continue
    k = p.numel(); a, b = ge[off:off+k], gg[off:off+k]; off += k
    r = float((a - b).norm() / (a.norm() + 1e-30))
    if r > 1e-2 or torch.isnan(b).any(): bad.append((n, r, float(a.norm()), float(b.norm())))
print("params off:", len(bad)); [print(" ", t) for t in bad[:30]]
