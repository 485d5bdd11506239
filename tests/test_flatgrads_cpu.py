"""FlatGrads (radhip/train.py): every .grad a view of one fp32 buffer; clip_norm_ equals
torch.nn.utils.clip_grad_norm_ (to fp32 summation order) whether it clips or not, and bound() notices a .grad that
was rebound elsewhere (the trainer then takes torch's per-tensor clip)."""
import torch

from radhip.train import FlatGrads


def _setup(scale):
    g = torch.Generator().manual_seed(7)
    ps = [torch.nn.Parameter(torch.randn(*s, generator=g)) for s in [(3,), (64, 9), (1,), (5, 7, 2)]]
    fg = FlatGrads(ps)
    for p in ps:
        p.grad.copy_(scale * torch.randn(p.shape, generator=g))
    return ps, fg


def test_clip_norm_matches_torch():
    for scale in (0.01, 10.0):            # below and above max_norm
        ps, fg = _setup(scale)
        ref = [p.grad.clone() for p in ps]
        qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
        for q, r in zip(qs, ref):
            q.grad = r.clone()
        n_ref = torch.nn.utils.clip_grad_norm_(qs, max_norm=3.0, foreach=False)
        assert fg.bound()
        n = fg.clip_norm_(3.0)
        assert abs(float(n) - float(n_ref)) <= 1e-6 * float(n_ref)
        for p, q in zip(ps, qs):
            assert torch.allclose(p.grad, q.grad, rtol=1e-6, atol=1e-7)


def test_bound_detects_rebinding():
    ps, fg = _setup(1.0)
    assert fg.bound()
    ps[1].grad = torch.zeros_like(ps[1])
    assert not fg.bound()
