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


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_wgrad_batch_matches_one_by_one(dt):
    """radhip.ops.wgrad_batch: the head's weight gradients of one pass collected and run as batched launches
    (rdx_wgrad_acc_many) equal the one-by-one launches to fp32 summation order (1e-5 of the max-norm), at the
    per-layer shapes of a B = 8 pass, with a strided view, a gradient without bias, a dw targeted twice (it must
    start a second launch: both adds land) and more than 32 problems (several launches); repeat runs bit-identical."""
    from radhip import ops
    g = torch.Generator(device="cpu").manual_seed(11)
    M = 1608
    shapes = [(576, 144), (41, 288), (288, 9), (144, 288), (576, 144), (144, 576)] * 6 + [(144, 1024), (2, 144)]
    big = torch.randn(M, 50, generator=g).to(DEV).to(dt)
    items, refs = [], []
    for i, (N, K) in enumerate(shapes):
        dy = big[:, 9:50] if (N, K) == (41, 288) else torch.randn(M, N, generator=g).to(DEV).to(dt)
        x = torch.randn(M, K, generator=g).to(DEV).to(dt)
        dw = torch.randn(N, K, generator=g).to(DEV)
        db = torch.randn(N, generator=g).to(DEV) if i % 3 else None
        items.append((dy, x, dw, db))
    items.append((items[0][0], items[0][1], items[0][2], items[0][3]))      # the same dw again
    outs = []
    for rep in range(2):
        got = [(dw.clone(), db.clone() if db is not None else None) for _, _, dw, db in items]
        seen = {}
        batch = []
        for (dy, x, dw, db), (gw, gb) in zip(items, got):
            key = dw.data_ptr()
            gw, gb = seen.get(key, (gw, gb))
            seen[key] = (gw, gb)
            batch.append((dy, x, gw, gb))
        with ops.wgrad_batch():
            for it in batch:
                ops.wgrad_acc(*it)
            assert ops._WGRAD_BATCH is not None and len(ops._WGRAD_BATCH[1]) == len(items)   # nothing launched yet
        outs.append([(b[2], b[3]) for b in batch])
    for (dy, x, dw, db), (gw, gb), (gw2, gb2) in zip(items, outs[0], outs[1]):
        assert torch.equal(gw, gw2) and (gb is None or torch.equal(gb, gb2))
    n0 = sum(1 for it in items if it[2].data_ptr() == items[0][2].data_ptr())
    for i, ((dy, x, dw, db), (gw, gb)) in enumerate(zip(items, outs[0])):
        reps = n0 if dw.data_ptr() == items[0][2].data_ptr() else 1
        prod = dy.double().t() @ x.double()
        ref = dw.double() + reps * prod
        assert float((gw.double() - ref).abs().max()) / float(prod.abs().max().clamp_min(1.0)) < 1e-5, i
        if db is not None:
            s = dy.double().sum(0)
            assert float((gb.double() - (db.double() + reps * s)).abs().max()) / float(s.abs().max().clamp_min(1.0)) < 1e-5
