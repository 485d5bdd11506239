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


def _run(golden, fgm, graphed, accum, n_micro, xs, ys):
    import random
    from radhip.build import apply_lora_to_wavlm, load_config
    from radhip.train import GraphedMicroStep, Trainer
    cfg = load_config("Phase6_Proposed.conf")
    cfg["training_config"]["accumulation_steps"] = accum
    cfg["training_config"]["lora_dropout"] = 0.0
    cfg["training_config"]["lora_mode"] = "active"
    cfg["training_config"]["use_fgm"] = fgm
    torch.manual_seed(0)
    m = apply_lora_to_wavlm(_model(golden), cfg["training_config"])
    tr = Trainer(m, cfg, DEV, total_steps=4, amp_dtype=torch.float32)
    g = GraphedMicroStep(tr, 4) if graphed else None
    if g is not None:
        g.capture()
    np.random.seed(11)
    random.seed(11)
    torch.manual_seed(11)
    for i in range(n_micro):
        x, y = xs[i], ys[i]
        lam, perm = tr.mixup_draw(4)
        xm = lam * x + (1 - lam) * x[torch.tensor(perm, device=DEV)]
        last = i == n_micro - 1 and accum <= n_micro
        if g is not None:
            g.x.copy_(xm)
            g.run(y, lam, perm, last_in_epoch=last)
        else:
            tr.micro_step(xm, torch.from_numpy(y), lam, perm, last_in_epoch=last)
    torch.cuda.synchronize()
    return m, tr


def _inputs():
    rng = np.random.default_rng(5)
    xs = [torch.from_numpy(np.clip(0.1 * rng.standard_normal((4, 64600)), -1, 1).astype(np.float32)).to(DEV)
          for _ in range(3)]
    ys = [np.array([0, 1, 0, 1]), np.array([1, 1, 0, 0]), np.array([0, 0, 1, 0])]
    return xs, ys


@pytest.mark.parametrize("fgm", [True, False])
def test_graphed_micro_steps_accumulate_same_grads(golden, fgm):
    """Three graphed micro-batches (no optimizer step yet): the accumulated flat gradient and the loss
    equal the eager path's. Replays 2 and 3 guard against non-idempotent captured ops (memset nodes)."""
    xs, ys = _inputs()
    grads, losses, names = [], [], None
    for graphed in (False, True):
        m, tr = _run(golden, fgm, graphed, accum=100, n_micro=3, xs=xs, ys=ys)
        grads.append(tr.grads.flat.detach().clone())
        losses.append(float(tr.loss_sum.item()))
        names = [(n, p.numel()) for n, p in m.named_parameters() if p.requires_grad]
    assert losses[1] == pytest.approx(losses[0], rel=1e-5)
    off, bad = 0, []
    for n, k in names:
        a, b = grads[0][off:off + k], grads[1][off:off + k]
        off += k
        diff, ref = float((a - b).norm()), float(a.norm())
        # absolute floor: e.g. attention_pool.bias feeds a softmax over time, its gradient is
        # analytically zero and both paths return fp32 rounding noise
        if diff > 1e-4 * ref and diff > 1e-6:
            bad.append((n, diff, ref))
    assert not bad, bad


def test_graphed_optimizer_step_updates(golden):
    xs, ys = _inputs()
    m0, _ = _run(golden, True, False, accum=2, n_micro=2, xs=xs, ys=ys)
    m1, tr = _run(golden, True, True, accum=2, n_micro=2, xs=xs, ys=ys)
    p0 = dict(m0.named_parameters())
    moved = 0
    for n, p in m1.named_parameters():
        if p.requires_grad:
            assert torch.isfinite(p).all(), n
            # same update as eager within Adam's sensitivity to last-bit gradient noise
            torch.testing.assert_close(p, p0[n], rtol=1e-3, atol=2e-5, msg=n)
            moved += 1
    assert moved > 0 and np.isfinite(tr.epoch_loss())
