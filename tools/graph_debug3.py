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
def build():
    class Args:
        emb_size, num_encoders, d_state, sinc_channels, wavlm_freeze_layers = 144, 2, 16, 70, -1
        wavlm_config = dict(json.loads(str(g["wavlm_config"])), hidden_dropout=0.0, attention_dropout=0.0,
                            activation_dropout=0.0, feat_proj_dropout=0.0, layerdrop=0.0, mask_time_prob=0.0)
    torch.manual_seed(0)
    m = DS.Model(Args(), device=dev); seeded_fill_(m, seed=41); m = m.to(dev)
    m.fusion.dropout.p = 0.0; m.dropout.p = 0.0
    return m
cfg = load_config("Phase6_Proposed.conf")
tc = cfg["training_config"]; tc["accumulation_steps"] = 100; tc["lora_dropout"] = 0.0
cfg["freq_aug"] = "False"
B = 4
rng = np.random.default_rng(0)
x = torch.from_numpy(np.clip(0.1 * rng.standard_normal((B, 64600)), -1, 1).astype(np.float32)).to(dev)
y = torch.tensor([0, 1, 0, 1], device=dev)
snaps = {}
for mode in ("eager", "graph"):
    m = apply_lora_to_wavlm(build(), tc)
    tr = Trainer(m, cfg, dev, total_steps=1000, amp_dtype=torch.float32)
    fp = [(n, p) for n, p in m.named_parameters() if "feature_projection" in n]
    S = []
    if mode == "graph":
        gs = GraphedMicroStep(tr, B); gs.capture()
        tr.grads.zero()
        gs.x.copy_(x); gs._stage(y.cpu().numpy(), 1.0, None)
        gs.graphs[0].replay(); torch.cuda.synchronize(); S.append(tr.grads.flat.clone())
        gs._fgm(); torch.cuda.synchronize(); S.append(torch.cat([p.detach().reshape(-1) for _, p in fp]).clone())
        gs.graphs[1].replay(); torch.cuda.synchronize(); S.append(tr.grads.flat.clone())
        gs._restore()
    else:
        tr.grads.zero()
        tr.train_mode()
        loss = tr._fwd_loss(x, y, y, 1.0); loss.backward(); torch.cuda.synchronize(); S.append(tr.grads.flat.clone())
        tr.fgm.attack(); torch.cuda.synchronize(); S.append(torch.cat([p.detach().reshape(-1) for _, p in fp]).clone())
        adv = tr._fwd_loss(x, y, y, 1.0); adv.backward(); torch.cuda.synchronize(); S.append(tr.grads.flat.clone())
        tr.fgm.restore()
    names = [(n, p.numel()) for n, p in m.named_parameters() if p.requires_grad]
    snaps[mode] = S
def cmp(a, b, label):
    off = 0; bad = []
    for n, k in names:
        da, db = a[off:off+k], b[off:off+k]; off += k
        r = float((da - db).norm() / (da.norm() + 1e-30))
        if r > 1e-4: bad.append((round(r, 4), n[-50:], float(da.norm()), float(db.norm())))
    print(label, "mismatched params:", len(bad)); [print("   ", t) for t in bad[:8]]
cmp(snaps["eager"][0], snaps["graph"][0], "clean grads")
d = (snaps["eager"][1] - snaps["graph"][1]).abs().max()
print("attacked params max diff", float(d))
cmp(snaps["eager"][2], snaps["graph"][2], "after adv grads")
