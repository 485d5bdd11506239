"""The detector head's small-GEMM kernel (csrc/lgemm.hip) against torch fp32 references of the same unfused autocast
math (F.linear, nn.GELU, GELU's backward, the residual add of PN_BiMambas_Encoder, src/models/DualStreamSEMamba.py:
445-486), at every head linear's forward and input-gradient shape (M = 8 x 201 and 32 x 201 tokens, doubled for the
bidirectional x_proj / dt_proj) and ragged edges, bf16 and fp16, 16-bit and fp32 A, strided views.
Tolerance: 16-bit operands with fp32 accumulation vs an fp32 GEMM of the same operands, max-norm relative 1e-2 (bf16)
/ 2e-3 (fp16) before the final rounding; the GELU output is compared with gelu of the kernel's own rounded u."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = {torch.bfloat16: 1e-2, torch.float16: 2e-3}

# (M, N, K): the head's forward linears and their input gradients (N and K swapped)
SHAPES = [(1608, 144, 1024), (232, 144, 64), (1608, 144, 288), (8, 9, 144), (8, 144, 9), (1608, 576, 144),
          (3216, 41, 288), (3216, 288, 9), (1608, 144, 576), (1608, 1, 144), (8, 2, 144), (6432, 576, 144),
          (12864, 41, 288), (1608, 1024, 144), (1608, 288, 144), (3216, 288, 41), (3216, 9, 288), (1608, 144, 2),
          (1, 4, 8), (33, 65, 321), (100, 70, 700)]


def _rel(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-12))


def _mk(M, N, K, dt, seed=0, a_f32=False):
    g = torch.Generator(device="cpu").manual_seed(seed)
    a = torch.randn(M, K, generator=g).to(DEV)
    a = a if a_f32 else a.to(dt)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV).to(dt)
    b = (0.1 * torch.randn(N, generator=g)).to(DEV).to(dt)
    return a, w, b


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_lgemm_bias(M, N, K, dt):
    from radhip.ops import lgemm
    a, w, b = _mk(M, N, K, dt)
    ref = a.float() @ w.float().t() + b.float()
    got = lgemm(a, w, b)
    assert got.dtype == dt and got.shape == (M, N)
    assert _rel(got, ref) < TOL[dt]
    assert _rel(lgemm(a, w), a.float() @ w.float().t()) < TOL[dt]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(1608, 144, 288), (3216, 288, 9), (1608, 1024, 144), (33, 65, 321)])
def test_lgemm_fp32_in_out_and_residual(M, N, K, dt):
    """fp32 A rounded on load (autocast's input cast), fp32 output = the 16-bit result widened, plus a residual."""
    from radhip.ops import lgemm
    a, w, b = _mk(M, N, K, dt, seed=1, a_f32=True)
    ref16 = F.linear(a.to(dt), w, b)
    got = lgemm(a, w, b, out_dtype=torch.float32)
    assert got.dtype == torch.float32
    assert _rel(got, ref16) < TOL[dt]
    # the widened value is exactly representable in the 16-bit type
    assert torch.equal(got.to(dt).float(), got)
    r = torch.randn(M, N, device=DEV)
    got_r = lgemm(a, w, b, out_dtype=torch.float32, residual=r)
    assert float((got_r - (r + got)).abs().max()) == 0.0


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M", [1608, 6432, 77])
def test_lgemm_gelu_and_gelu_bwd(M, dt):
    """FFN1 + GELU forward (u, gelu(u)) and FFN2's input gradient times gelu'(u) (PN_BiMambas_Encoder's FFN)."""
    from radhip import _lib
    from radhip.ops import lgemm
    a, w1, b1 = _mk(M, 576, 144, dt, seed=2)
    u, h = lgemm(a, w1, b1, epilogue=_lib.EPI_BIAS_GELU)
    assert _rel(u, a.float() @ w1.float().t() + b1.float()) < TOL[dt]
    ref_h = F.gelu(u.float())
    assert _rel(h, ref_h) < TOL[dt]
    assert float((h.float() - ref_h.to(dt).float()).abs().max()) <= 2 * torch.finfo(dt).eps * float(ref_h.abs().max())
    g = torch.Generator(device="cpu").manual_seed(3)
    dy = (0.1 * torch.randn(M, 144, generator=g)).to(DEV).to(dt)
    w2t = (torch.randn(576, 144, generator=g) / 12).to(DEV).to(dt)   # FFN2 weight transposed: [576, 144]
    du = lgemm(dy, w2t, epilogue=_lib.EPI_GELU_BWD, aux=u)
    dh = (dy.float() @ w2t.float().t()).to(dt).float()
    ref = torch.ops.aten.gelu_backward(dh, u.float())
    assert _rel(du, ref) < TOL[dt]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_lgemm_strided_views(dt):
    """dt_proj's input: the first 9 columns of x_proj's [2, B, L, 41] output (row stride 41), and a weight view."""
    from radhip.ops import lgemm
    g = torch.Generator(device="cpu").manual_seed(4)
    x_dbl = torch.randn(3216, 41, generator=g).to(DEV).to(dt)
    dtv = x_dbl[:, :9]
    w = (torch.randn(288, 9, generator=g) / 3).to(DEV).to(dt)
    assert dtv.stride(0) == 41
    assert _rel(lgemm(dtv, w), dtv.float() @ w.float().t()) < TOL[dt]
    wide = torch.randn(300, 160, generator=g).to(DEV).to(dt)
    wv = wide[:288, 8:152]                    # [288, 144] at row stride 160, 16-byte aligned
    a = torch.randn(1608, 144, generator=g).to(DEV).to(dt)
    assert _rel(lgemm(a, wv), a.float() @ wv.float().t()) < TOL[dt]
    wu = wide[:64, 3:147]                     # unaligned rows: element loads
    assert _rel(lgemm(a, wu), a.float() @ wu.float().t()) < TOL[dt]
