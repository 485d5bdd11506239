"""radhip.optim.AdamW (csrc/optim.hip) against torch.optim.AdamW(fused=True) on the same tensors: two parameter
groups (different lr / weight decay), sizes below, at and above the 4096-element block and not a multiple of 4,
GradScaler's grad_scale (grads stored back unscaled) and found_inf (update skipped, step counts rolled back), and
the state_dict both ways. Tolerance: fp32 element math in a different operation order, 2e-6 of each tensor's
max-norm after four steps; step counts and the skipped step exact."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _params(seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    shapes = [(3,), (4096,), (4097,), (576, 144), (1, 144), (70, 1, 129)]
    return [torch.nn.Parameter(torch.randn(*s, generator=g).to(DEV)) for s in shapes]


def _groups(ps):
    return [{"params": ps[:3], "lr": 1e-3, "weight_decay": 1e-4}, {"params": ps[3:], "lr": 3e-4, "weight_decay": 0.0}]


def test_adamw_matches_torch_fused():
    from radhip.optim import AdamW
    a, b = _params(1), _params(1)
    oa = AdamW(_groups(a), betas=(0.9, 0.999), eps=1e-8)
    ob = torch.optim.AdamW(_groups(b), betas=(0.9, 0.999), eps=1e-8, fused=True)
    g = torch.Generator(device="cpu").manual_seed(2)
    for step in range(5):
        for pa, pb in zip(a, b):
            gr = torch.randn(pa.shape, generator=g).to(DEV)
            pa.grad, pb.grad = gr.clone(), gr.clone()
        scale = torch.full((), 1024.0, device=DEV) if step % 2 else None
        inf = torch.full((), 1.0 if step == 3 else 0.0, device=DEV) if step >= 2 else None
        if scale is not None:
            for pa, pb in zip(a, b):
                pa.grad.mul_(1024.0)
                pb.grad.mul_(1024.0)
        for o in (oa, ob):
            if scale is not None:
                o.grad_scale = scale
            if inf is not None:
                o.found_inf = inf
        before = [p.detach().clone() for p in a]
        oa.step()
        ob.step()
        for o in (oa, ob):
            for k in ("grad_scale", "found_inf"):
                if hasattr(o, k):
                    delattr(o, k)
        if step == 3:
            assert all(torch.equal(p, q) for p, q in zip(a, before)), "found_inf must skip the update"
        for pa, pb in zip(a, b):
            tol = 2e-6 * float(pb.detach().abs().max().clamp_min(1.0))
            assert float((pa - pb).abs().max()) <= tol
            assert float((pa.grad - pb.grad).abs().max()) <= 1e-6 * float(pb.grad.abs().max().clamp_min(1.0))
            sa, sb = oa.state[pa], ob.state[pb]
            assert float(sa["step"]) == float(sb["step"])
            for k in ("exp_avg", "exp_avg_sq"):
                assert float((sa[k] - sb[k]).abs().max()) <= 2e-6 * float(sb[k].abs().max().clamp_min(1e-30)) + 1e-30
    assert float(oa.state[a[0]]["step"]) == 4.0      # five steps, one skipped
    # state_dict both ways: a torch AdamW continues from ours and ours from torch's, identically to each other
    c = _params(3)
    oc_ = torch.optim.AdamW(_groups(c), fused=True)
    oc_.load_state_dict(oa.state_dict())
    d = _params(3)
    od = AdamW(_groups(d))
    od.load_state_dict(ob.state_dict())
    for p in c + d:
        p.grad = torch.ones_like(p)
    oc_.step()
    od.step()
    for pc, pd in zip(c, d):
        assert float((pc - pd).abs().max()) <= 2e-6 * float(pc.detach().abs().max().clamp_min(1.0))


def test_adamw_cpu_step_state_and_flags():
    """A state_dict whose step counts are CPU scalars (torch's non-fused AdamW, or a checkpoint loaded with
    map_location="cpu") steps on the device like torch's fused AdamW; the saved groups carry torch's fused flags, so
    torch's own AdamW resumed from them keeps the fused form (the one that takes GradScaler's arguments)."""
    from radhip.optim import AdamW
    a, b = _params(5), _params(5)
    ref = torch.optim.AdamW(_groups(a), foreach=False)          # non-fused: CPU step scalars
    for p in a:
        p.grad = torch.ones_like(p)
    ref.step()
    sd = ref.state_dict()
    assert not sd["state"][0]["step"].is_cuda
    o = AdamW(_groups(b))
    with torch.no_grad():
        for pa, pb in zip(a, b):
            pb.copy_(pa)
    o.load_state_dict(sd)
    for p in a + b:
        p.grad = torch.full_like(p, 0.5)
    ref.step()
    o.step()
    torch.cuda.synchronize()
    for pa, pb in zip(a, b):
        assert o.state[pb]["step"].is_cuda and float(o.state[pb]["step"]) == 2.0
        assert float((pa - pb).abs().max()) <= 2e-6 * float(pa.detach().abs().max().clamp_min(1.0))
    saved = o.state_dict()["param_groups"][0]
    assert saved["fused"] is True
    t = torch.optim.AdamW(_groups(_params(5)), fused=True)
    t.load_state_dict(o.state_dict())
    assert t.param_groups[0]["fused"] is True
