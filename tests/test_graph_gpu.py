"""HIP-graph micro-step == eager micro-step (same host draws, same dropout off)."""
import numpy as np
import pytest
import torch

from seeded import seeded_fill_

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(golden):
    import json
    import models.DualStreamSEMamba as DS
    g = golden("model_tiny.npz")

    class Args:
        emb_size, num_encoders, d_state, sinc_channels, wavlm_freeze_layers = 144, 2, 16, 70, -1
        wavlm_config = dict(json.loads(str(g["wavlm_config"])), hidden_dropout=0.0, attention_dropout=0.0,
                            activation_dropout=0.0, feat_proj_dropout=0.0, layerdrop=0.1)
    m = DS.Model(Args(), device=DEV)
    seeded_fill_(m, seed=41)
    m.fusion.dropout.p = 0.0
    m.dropout.p = 0.0
    return m.to(DEV)


@pytest.mark.parametrize("fgm", [True, False])
def test_graphed_micro_step_matches_eager(golden, fgm):
    import random
    from radhip.build import apply_lora_to_wavlm, load_config
    from radhip.train import GraphedMicroStep, Trainer
    cfg = load_config("Phase6_Proposed.conf")
    cfg["training_config"]["accumulation_steps"] = 2
    cfg["training_config"]["lora_dropout"] = 0.0
    cfg["training_config"]["use_fgm"] = fgm
    rng = np.random.default_rng(5)
    xs = [torch.from_numpy(np.clip(0.1 * rng.standard_normal((4, 64600)), -1, 1).astype(np.float32)).to(DEV)
          for _ in range(3)]
    ys = [np.array([0, 1, 0, 1]), np.array([1, 1, 0, 0]), np.array([0, 0, 1, 0])]
    results = []
    for graphed in (False, True):
        torch.manual_seed(0)
        m = apply_lora_to_wavlm(_model(golden), cfg["training_config"])
        tr = Trainer(m, cfg, DEV, total_steps=4, amp_dtype=torch.float32)
        g = GraphedMicroStep(tr, 4) if graphed else None
        if g is not None:
            g.capture()
        np.random.seed(11)
        random.seed(11)
        torch.manual_seed(11)
        for i, (x, y) in enumerate(zip(xs, ys)):
            lam, perm = tr.mixup_draw(4)
            xm = lam * x + (1 - lam) * x[torch.tensor(perm, device=DEV)]
            if g is not None:
                g.x.copy_(xm)
                g.run(y, lam, perm, last_in_epoch=(i == 2))
            else:
                tr.micro_step(xm, torch.from_numpy(y), lam, perm, last_in_epoch=(i == 2))
        torch.cuda.synchronize()
        results.append(({n: p.detach().clone() for n, p in m.named_parameters() if p.requires_grad},
                        tr.epoch_loss()))
    (pe, le), (pg, lg) = results
    assert lg == pytest.approx(le, rel=1e-4)
    for n in pe:
        torch.testing.assert_close(pg[n], pe[n], rtol=1e-4, atol=1e-6, msg=n)
