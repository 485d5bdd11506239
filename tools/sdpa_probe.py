"""Which SDPA backends accept the WavLM attention (bf16, [B,16,201,64], additive bias that requires
grad, dropout 0.1)? Forces each backend and prints the refusal reason or the kernels it ran."""
import warnings

import torch
import torch.nn.functional as F
from torch.nn.attention import SDPBackend, sdpa_kernel
from torch.profiler import ProfilerActivity, profile

dev = "cuda"
B, H, T, D = 8, 16, 201, 64


def run(backend, bias_grad, dropout):
    q = torch.randn(B, H, T, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn_like(q, requires_grad=True)
    v = torch.randn_like(q, requires_grad=True)
    bias = torch.randn(B, H, T, T, device=dev, dtype=torch.bfloat16, requires_grad=bias_grad)
    tag = f"{backend.name:22s} bias_grad={bias_grad} dropout={dropout}"
    try:
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            with sdpa_kernel([backend]):
                for _ in range(2):
                    o = F.scaled_dot_product_attention(q, k, v, attn_mask=bias, dropout_p=dropout)
                    o.float().sum().backward()
                torch.cuda.synchronize()
                with profile(activities=[ProfilerActivity.CUDA]) as prof:
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                    ev[0].record()
                    o = F.scaled_dot_product_attention(q, k, v, attn_mask=bias, dropout_p=dropout)
                    o.float().sum().backward()
                    ev[1].record()
                    torch.cuda.synchronize()
        ks = sorted({e.key[:60] for e in prof.key_averages() if "CUDA" in str(e.device_type)})
        print(f"OK   {tag}  {ev[0].elapsed_time(ev[1]):.3f} ms  grad_bias={'yes' if bias.grad is not None else 'no'}"
              f"  kernels={ks[:6]}", flush=True)
    except Exception as e:  # noqa: BLE001
        msg = str(e).replace("\n", " ")[:300]
        print(f"FAIL {tag}  {msg}  warn={[str(x.message)[:200] for x in w][:3]}", flush=True)


for be in (SDPBackend.EFFICIENT_ATTENTION, SDPBackend.FLASH_ATTENTION, SDPBackend.MATH):
    for bg in (True, False):
        run(be, bg, 0.1)
run(SDPBackend.EFFICIENT_ATTENTION, True, 0.0)
