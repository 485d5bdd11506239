"""Focal loss (radhip.train.FocalLoss) = kornia.losses.FocalLoss(alpha, gamma, reduction='mean') as the
Phase-6 criterion (src/main.py:297-305; focal_alpha 0.9, focal_gamma 2.5 in Phase6_*.conf).

kornia is absent from the image and unpinned by the reference, so these pin the restated formula by
hand-computed values (pure-Python math, no torch) in both kornia conventions, plus its closed-form
limits: gamma = 0 and alpha = None is cross-entropy, the per-class weights, p -> 1 without NaN, and the
gradient against torch autograd of the same closed form."""
import math

import pytest
import torch

from radhip.train import FocalLoss, build_criterion

LOGITS = [[2.0, -1.0], [0.5, 0.3], [-1.0, 3.0], [0.0, 0.0]]
TARGET = [0, 1, 1, 0]


def _hand(alpha, gamma, mode):
    """Per-element restatement with math.* only."""
    tot = 0.0
    for (a, b), y in zip(LOGITS, TARGET):
        m = max(a, b)
        lse = m + math.log(math.exp(a - m) + math.exp(b - m))
        lp = (a if y == 0 else b) - lse
        p = math.exp(lp)
        if alpha is None:
            w = 1.0
        elif mode == "per_class":
            w = (1.0 - alpha) if y == 0 else alpha
        else:
            w = alpha
        tot += -w * (1.0 - p) ** gamma * lp
    n = len(TARGET)
    return tot / (2 * n) if mode == "per_class" else tot / n


@pytest.mark.parametrize("mode", ["per_class", "scalar"])
@pytest.mark.parametrize("alpha,gamma", [(0.9, 2.5), (0.25, 2.0), (0.5, 0.0)])
def test_focal_matches_hand_computed(mode, alpha, gamma):
    got = FocalLoss(alpha, gamma, mode)(torch.tensor(LOGITS), torch.tensor(TARGET))
    assert float(got) == pytest.approx(_hand(alpha, gamma, mode), rel=1e-6, abs=1e-9)


def test_phase6_value_pinned():
    """alpha 0.9, gamma 2.5, per-class (kornia >= 0.7): the number the Phase-6 criterion returns."""
    got = float(FocalLoss(0.9, 2.5)(torch.tensor(LOGITS), torch.tensor(TARGET)))
    assert got == pytest.approx(0.0216605, rel=1e-5)
    assert got == pytest.approx(_hand(0.9, 2.5, "per_class"), rel=1e-6)


def test_gamma0_no_alpha_is_cross_entropy():
    x, y = torch.tensor(LOGITS), torch.tensor(TARGET)
    ce = torch.nn.functional.cross_entropy(x, y)
    assert torch.allclose(FocalLoss(None, 0.0, "scalar")(x, y), ce, rtol=1e-6)
    assert torch.allclose(FocalLoss(None, 0.0, "per_class")(x, y), ce / 2, rtol=1e-6)   # mean over B*C


def test_per_class_weights():
    """Class 0 (spoof) is weighted 1 - alpha, class 1 (bona fide) alpha (kornia >= 0.7)."""
    x = torch.tensor([[0.3, -0.2]])
    f1 = FocalLoss(None, 2.0)
    for y, wgt in ((0, 0.1), (1, 0.9)):
        t = torch.tensor([y])
        assert float(FocalLoss(0.9, 2.0)(x, t)) == pytest.approx(wgt * float(f1(x, t)), rel=1e-6)


def test_confident_prediction_is_finite_and_zero():
    x = torch.tensor([[60.0, -60.0], [-80.0, 80.0]], requires_grad=True)
    y = torch.tensor([0, 1])
    loss = FocalLoss(0.9, 2.5)(x, y)
    loss.backward()
    assert float(loss) == 0.0 and torch.isfinite(x.grad).all()


def test_gradient_matches_closed_form():
    torch.manual_seed(0)
    x = torch.randn(16, 2, dtype=torch.float64, requires_grad=True)
    y = torch.randint(0, 2, (16,))
    FocalLoss(0.9, 2.5)(x.float(), y).backward()
    x2 = x.detach().clone().requires_grad_(True)
    lp = torch.log_softmax(x2, 1).gather(1, y[:, None]).squeeze(1)
    a = torch.where(y == 0, 0.1, 0.9).double()
    (-(a * (1 - lp.exp()) ** 2.5 * lp).sum() / 32).backward()
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-5, atol=1e-8)


def test_build_criterion_selection():
    """main.py:270-312: 'Focal' or use_focal_loss -> focal (alpha/gamma from training_config); else the
    class-weighted CE [0.1, 0.9] with label smoothing."""
    c = build_criterion({"loss": "Focal", "training_config": {"focal_alpha": 0.9, "focal_gamma": 2.5}}, "cpu")
    assert isinstance(c, FocalLoss) and (c.alpha, c.gamma, c.alpha_mode) == (0.9, 2.5, "per_class")
    c = build_criterion({"loss": "CCE", "training_config": {"use_focal_loss": True}}, "cpu")
    assert isinstance(c, FocalLoss) and (c.alpha, c.gamma) == (0.25, 2.0)
    c = build_criterion({"loss": "CCE", "training_config": {"label_smoothing": 0.1}}, "cpu")
    assert isinstance(c, torch.nn.CrossEntropyLoss) and c.label_smoothing == 0.1
    assert torch.equal(c.weight, torch.tensor([0.1, 0.9]))
    with pytest.raises(ValueError):
        FocalLoss(0.9, 2.5, "other")
