"""Split-K graph workspace grown inside a capture (radhip/ops.py _grow_workspace / finalize_graph_workspace).

A split-K hgemm (csrc/hgemm.hip, last-arriver tickets) captured while the device's graph workspace is too small grows
it inside the capture; the new tickets' zero fill is then only a node of that graph. A second graph captured later
on the same workspace must still find zeroed tickets if it replays FIRST: finalize_graph_workspace zeroes them
eagerly after the capture. Checked by replaying the second graph before the first."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_split_k_graph_workspace_grown_in_capture_replays_in_any_order():
    from radhip import ops
    dev = torch.device("cuda", 0)
    key = (dev.index, "graph")
    saved = ops._WG_WS.get(key)
    g = torch.Generator(device="cpu").manual_seed(0)
    M, N, K = 1608, 1024, 4096
    a1 = torch.randn(M, K, generator=g).to(dev).to(torch.bfloat16)
    a2 = torch.randn(M, K, generator=g).to(dev).to(torch.bfloat16)
    b = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev).to(torch.bfloat16)
    ref1 = a1.float() @ b.float().t()
    ref2 = a2.float() @ b.float().t()
    try:
        # an undersized graph workspace: the first capture must grow it
        ops._WG_WS[key] = (torch.empty(16, dtype=torch.uint8, device=dev), torch.zeros(1, dtype=torch.int32, device=dev))
        torch.cuda.synchronize()
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            g1 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1, stream=side):
                out1 = ops.hgemm(a1, b, tile=4, splits=2, group_m=4)
            grown = ops._WG_WS[key]
            assert grown[1].numel() >= int(ops.lib().rdx_hgemm_counters(M, N, 4)), "capture did not grow the tickets"
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, stream=side):
                out2 = ops.hgemm(a2, b, tile=4, splits=2, group_m=4)
            assert ops._WG_WS[key] is grown
        torch.cuda.current_stream(dev).wait_stream(side)
        ops.finalize_graph_workspace(dev)
        assert int(grown[1].abs().sum()) == 0
        for order in ((g2, g1), (g1, g2), (g2, g2)):
            out1.zero_()
            out2.zero_()
            for gr in order:
                gr.replay()
            torch.cuda.synchronize()
            for gr, out, ref in ((g1, out1, ref1), (g2, out2, ref2)):
                if gr in order:
                    err = float((out.float() - ref).abs().max() / ref.abs().max())
                    assert err < 1e-2, (order, err)
            assert int(grown[1].abs().sum()) == 0, "a launch left a ticket non-zero"
    finally:
        if saved is not None:
            ops._WG_WS[key] = saved
        else:
            ops._WG_WS.pop(key, None)
