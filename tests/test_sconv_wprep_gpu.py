"""rdx_sconv_wprep_many (csrc/sconv.hip) against the torch layouts it replaces (radhip/ops.py _sconv_w_prep): both
16-bit operand layouts of the SincNet stack's convolution weights, bit-exact (a cast and two permutations)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_wprep_many_matches_torch_layouts(dt):
    from radhip import ops
    g = torch.Generator(device="cpu").manual_seed(0)
    shapes = [(32, 32, 2, 3), (64, 32, 2, 3), (64, 64, 2, 3), (64, 32, 1, 3), (32, 64, 1, 3), (64, 64, 1, 3)]
    ws = [torch.nn.Parameter(torch.randn(*s, generator=g).cuda()) for s in shapes]
    saved = ops.SCONV_WCACHE
    try:
        ops.SCONV_WCACHE = {}
        ops.sconv_prep_many(ws, dt)
        torch.cuda.synchronize()
        for w in ws:
            wf0, wd0 = ops._sconv_w_prep(w, dt)
            hit = ops.SCONV_WCACHE[(id(w), dt)]
            assert hit[0] is w
            assert torch.equal(hit[1], wf0) and torch.equal(hit[2], wd0)
            assert ops._sconv_w(w, dt)[0] is hit[1]        # the convolutions' lookup finds them
    finally:
        ops.SCONV_WCACHE = saved
