"""Host logic of the batched head weight gradients (radhip.ops.wgrad_groups): launches of at most 32 problems of
one dtype, every dW / db targeted once per launch, item order kept (a repeated gradient starts the next launch, so
its adds land in stream order)."""
import torch

from radhip import ops


def _item(dt, dw, db=None):
    return (torch.zeros(4, 2, dtype=dt), torch.zeros(4, 3, dtype=dt), dw, db)


def test_groups_split_on_repeat_size_and_dtype():
    ws = [torch.zeros(2, 3) for _ in range(40)]
    bs = [torch.zeros(2) for _ in range(40)]
    items = [_item(torch.bfloat16, ws[i], bs[i] if i % 2 else None) for i in range(40)]
    g = ops.wgrad_groups(items)
    assert [len(x) for x in g] == [32, 8]
    assert [it for grp in g for it in grp] == items
    rep = items[:3] + [items[1]] + items[3:5]                  # the second item's dw / db again
    g = ops.wgrad_groups(rep)
    assert [len(x) for x in g] == [3, 3] and g[1][0] is items[1]
    shared_b = [_item(torch.float16, ws[0], bs[0]), _item(torch.float16, ws[1], bs[0])]   # same db, new dw
    assert [len(x) for x in ops.wgrad_groups(shared_b)] == [1, 1]
    mixed = [_item(torch.bfloat16, ws[0]), _item(torch.float16, ws[1]), _item(torch.float16, ws[2])]
    assert [len(x) for x in ops.wgrad_groups(mixed)] == [1, 2]
    assert ops.wgrad_groups([]) == []


def test_batch_block_is_a_no_op_without_gpu():
    with ops.wgrad_batch() as b:
        assert not b.on or torch.cuda.is_available()
    assert ops._WGRAD_BATCH is None
