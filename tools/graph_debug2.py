"""Bisect graph-vs-eager gradient mismatches on the tiny golden model."""
import os, sys, random, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "robust-audio-deepfake-evolution_amd"), ROOT, os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import numpy as np, torch
from seeded import seeded_fill_
import models.DualStreamSEMamba as DS
from radhip.build import apply_lora_to_wavlm, load_config
from radhip.train import Trainer, GraphedMicroStep
dev = torch.device("cuda", 0)
g = dict(np.load(os.path.join(ROOT, "tests/golden/model_tiny.npz")))
def build(drop):
    class Args:
        emb_size, num_encoders, d_state, sinc_channels, wavlm_freeze_layers = 144, 2, 16, 70, -1
        wavlm_config = dict(json.loads(str(g["wavlm_config"])), hidden_dropout=drop, attention_dropout=drop,
                            activation_dropout=0.0, feat_proj_dropout=drop, layerdrop=0.0)
    torch.manual_seed(0)
    m = DS.Model(Args(), device=dev); seeded_fill_(m, seed=41); m = m.to(dev)
    m.fusion.dropout.p = drop; m.dropout.p = drop
    return m
def variant(drop, fgm, amp, lora_drop):
    cfg = load_config("Phase6_Proposed.conf")
    tc = cfg["training_config"]; tc["accumulation_steps"] = 100; tc["use_fgm"] = fgm; tc["lora_dropout"] = lora_drop
    res = {}
    for mode in ("eager", "eager2", "graph"):
        m = apply_lora_to_wavlm(build(drop), tc)
        tr = Trainer(m, cfg, dev, total_steps=1000, amp_dtype=torch.bfloat16 if amp else torch.float32)
        B = 4
        rng = np.random.default_rng(0)
        x = torch.from_numpy(np.clip(0.1 * rng.standard_normal((B, 64600)), -1, 1).astype(np.float32)).to(dev)
        y = np.array([0, 1, 0, 1])
        gs = GraphedMicroStep(tr, B) if mode == "graph" else None
        if gs: gs.capture()
        tr.grads.zero(); tr.loss_sum.zero_()
        np.random.seed(5); random.seed(5); torch.manual_seed(5)
        lam, perm = tr.mixup_draw(B)
        xm = lam * x + (1 - lam) * x[torch.tensor(perm, device=dev)]
        if gs:
            gs.x.copy_(xm); gs.run(y, lam, perm)
        else:
            tr.micro_step(xm, torch.from_numpy(y), lam, perm)
        torch.cuda.synchronize()
        res[mode] = ({n: p.grad.detach().clone() for n, p in m.named_parameters() if p.requires_grad}, float(tr.loss_sum))
    (ge, le), (gg, lg), (g2, l2) = res["eager"], res["graph"], res["eager2"]
    noise = {n: float((g2[n]-ge[n]).norm()/(ge[n].norm()+1e-30)) for n in ge}
    worst = sorted(((float((gg[n]-ge[n]).norm()/(ge[n].norm()+1e-30)), n) for n in ge), reverse=True)[:4]
    worst = [(a, b, round(noise[b], 5)) for a, b in worst]
    nans = sum(int(torch.isnan(gg[n]).any() or torch.isinf(gg[n]).any()) for n in gg)
    print(f"drop={drop} fgm={fgm} amp={amp} loradrop={lora_drop}: loss e {le:.6f} g {lg:.6f} nan-params {nans} worst {[(round(a,4), b[-40:], c) for a,b,c in worst]}", flush=True)
for drop in [0.0, 0.1]:
    for fgm in [False, True]:
        variant(drop, fgm, amp=False, lora_drop=0.0)
variant(0.1, True, amp=True, lora_drop=0.1)
variant(0.0, False, amp=True, lora_drop=0.0)
