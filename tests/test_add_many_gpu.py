"""ops.add_many (csrc/layersum.hip rdx_add_f32_many): the window's per-pass gradient hand-over, dst += src over up
to 64 fp32 tensors per launch (or dst = src), against torch's _foreach_add_ / _foreach_copy_ (the same fp32 adds:
bit-exact)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _tensors(sizes, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return [torch.randn(n, generator=g).to(DEV) for n in sizes]


@pytest.mark.parametrize("copy", [False, True])
@pytest.mark.parametrize("sizes", [
    [1],
    [4096],
    [4097, 0, 3, 65536 + 17],                  # ragged, an empty tensor in the middle
    [0, 5],                                    # an empty first tensor
    [1024 * 512, 512, 512, 1024],              # feature_projection's four tensors
    [37 * k + 1 for k in range(150)],          # more than one launch (64 per launch)
])
def test_add_many_matches_foreach(sizes, copy):
    from radhip import ops
    dst = _tensors(sizes, 1)
    src = _tensors(sizes, 2)
    ref = [d.clone() for d in dst]
    if copy:
        torch._foreach_copy_(ref, src)
    else:
        torch._foreach_add_(ref, src)
    ops.add_many(dst, src, copy=copy)
    torch.cuda.synchronize()
    for a, b in zip(dst, ref):
        assert torch.equal(a, b)


def test_add_many_views_and_shapes():
    """Destinations are views of one flat buffer (the trainer's gradient buffer), sources 2-D tensors."""
    from radhip import ops
    flat = torch.randn(3 * 1000 + 7, device=DEV)
    views = [flat[:1000].view(10, 100), flat[1000:2003], flat[2003:].view(-1)]
    src = [torch.randn(10, 100, device=DEV), torch.randn(1003, device=DEV), torch.randn(flat.numel() - 2003, device=DEV)]
    want = flat.clone()
    want[:1000] += src[0].view(-1)
    want[1000:2003] += src[1]
    want[2003:] += src[2]
    ops.add_many(views, src)
    assert torch.equal(flat, want)


def test_add_many_rejects_bad_operands():
    from radhip import ops
    a = torch.zeros(8, device=DEV)
    with pytest.raises(ValueError):
        ops.add_many([a], [torch.zeros(8, device=DEV, dtype=torch.float16)])
    with pytest.raises(ValueError):
        ops.add_many([a], [torch.zeros(9, device=DEV)])
    with pytest.raises(ValueError):
        ops.add_many([torch.zeros(4, 4, device=DEV).t()], [torch.zeros(4, 4, device=DEV)])
    with pytest.raises(RuntimeError):
        ops.add_many([torch.zeros(8)], [torch.zeros(8)])
