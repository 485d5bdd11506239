"""The head linears' weight / bias gradients on csrc/wgrad.hip (radhip.ops.wgrad_acc, used by SideLinear's
backward) against a torch fp32 reference of the same bf16 operands: dW += dY^T X and db += sum(dY), accumulated
into existing fp32 buffers, at the PN-BiMamba / fusion / pooling shapes (token rows 1608, 3216, 6432; outputs
576 x 144, 41 x 288, 288 x 9, 144 x 1024, 1 x 144) and ragged, unaligned cases. Tolerance: fp32 sums of bf16
products in a different order, 1e-5 relative (max-norm); repeat launches bit-identical."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("M,N,K", [(1608, 576, 144), (3216, 41, 288), (3216, 288, 9), (1608, 144, 1024),
                                   (6432, 144, 576), (1608, 1, 144), (37, 3, 5), (1, 2, 144), (6432, 2, 144)])
@pytest.mark.parametrize("bias", [True, False])
def test_wgrad_acc_matches_fp32(M, N, K, bias):
    from radhip.ops import wgrad_acc
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    dy = torch.randn(M, N, generator=g).to(DEV).to(torch.bfloat16)
    x = torch.randn(M, K, generator=g).to(DEV).to(torch.bfloat16)
    dw0 = torch.randn(N, K, generator=g).to(DEV)
    db0 = torch.randn(N, generator=g).to(DEV)
    dw, db = dw0.clone(), db0.clone()
    wgrad_acc(dy, x, dw, db if bias else None)
    ref = dw0 + dy.double().t() @ x.double()
    scale = float((dy.double().t() @ x.double()).abs().max().clamp_min(1.0))
    assert float((dw.double() - ref).abs().max()) / scale < 1e-5
    if bias:
        refb = db0.double() + dy.double().sum(0)
        assert float((db.double() - refb).abs().max()) / float(dy.double().sum(0).abs().max().clamp_min(1.0)) < 1e-5
    else:
        assert torch.equal(db, db0)
    dw2, db2 = dw0.clone(), db0.clone()
    wgrad_acc(dy, x, dw2, db2 if bias else None)
    assert torch.equal(dw2, dw) and torch.equal(db2, db)


def test_wgrad_acc_strided_views():
    """Row views with a leading stride (the x_dbl / xz column slices of the Bi-Mamba) and an unaligned base."""
    from radhip.ops import wgrad_acc
    g = torch.Generator(device="cpu").manual_seed(5)
    big = torch.randn(3216, 50, generator=g).to(DEV).to(torch.bfloat16)
    dy = big[:, 9:50]                       # [3216, 41], ld 50, base offset 9 elements
    x = torch.randn(3216, 288, generator=g).to(DEV).to(torch.bfloat16)
    dw = torch.zeros(41, 288, device=DEV)
    wgrad_acc(dy, x, dw)
    ref = dy.double().t() @ x.double()
    assert float((dw.double() - ref).abs().max() / ref.abs().max()) < 1e-5
