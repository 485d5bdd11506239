"""The hand-written bf16 MFMA GEMM (csrc/gemm.hip) with its fused epilogues against torch fp32 references
of the same unfused math, at the WavLM layer's shapes (M = 8 x 201 and 32 x 201 tokens; the q|k|v +
LoRA, out_proj, FFN1 and FFN2 projections and their input gradients) and ragged edges.
Tolerances: bf16 operands with fp32 accumulation vs an fp32 GEMM of the same bf16 operands, 1e-2
relative (max-norm) before the final bf16 rounding; the dropout mask of the residual epilogue is the
element-wise hash (rdx_dropout_mask) and must match exactly."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-12))


def _ops(M, N, K, seed=0, lda=None):
    g = torch.Generator(device="cpu").manual_seed(seed)
    lda = lda or K
    a_full = torch.randn(M, lda, generator=g).to(DEV).to(torch.bfloat16)
    a = a_full[:, :K]
    b = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV).to(torch.bfloat16)
    bias = (0.1 * torch.randn(N, generator=g)).to(DEV).to(torch.bfloat16)
    return a, b, bias


@pytest.mark.parametrize("M,N,K", [(1608, 3072, 1040), (1608, 1024, 1024), (6432, 4096, 1024), (1608, 1024, 4096),
                                   (1608, 1040, 3072), (1, 4, 8), (130, 132, 72), (257, 260, 136)])
def test_gemm_bias_matches_fp32(M, N, K):
    from radhip.ops import gemm
    a, b, bias = _ops(M, N, K)
    got = gemm(a, b, bias)
    ref = a.float() @ b.float().t() + bias.float()
    assert got.dtype == torch.bfloat16 and got.shape == (M, N)
    assert _rel(got, ref) < 1e-2
    got0 = gemm(a, b)                                   # no bias
    assert _rel(got0, a.float() @ b.float().t()) < 1e-2


def test_gemm_strided_operand_view():
    """A as a column slice of a wider buffer (lda > K), as the LoRA-extended x1 is used."""
    from radhip.ops import gemm
    a, b, bias = _ops(333, 256, 1040, lda=1088)
    assert a.stride(0) == 1088
    assert _rel(gemm(a, b, bias), a.float() @ b.float().t() + bias.float()) < 1e-2


def test_gemm_bias_gelu_epilogue():
    from radhip import _lib
    from radhip.ops import gemm
    a, b, bias = _ops(1608, 4096, 1024, seed=1)
    u, v = gemm(a, b, bias, epilogue=_lib.EPI_BIAS_GELU)
    ref_u = (a.float() @ b.float().t() + bias.float())
    assert _rel(u, ref_u) < 1e-2
    # v is gelu of the stored (bf16) u, exactly as the unfused GELU kernel computes it
    ref_v = torch.nn.functional.gelu(u.float())
    assert _rel(v, ref_v) < 1e-2
    assert float((v.float() - ref_v.to(torch.bfloat16).float()).abs().max()) <= 2 ** -7 * float(ref_v.abs().max())


def test_gemm_gelu_backward_epilogue():
    from radhip import _lib
    from radhip.ops import gemm
    a, b, _ = _ops(1608, 4096, 1024, seed=2)
    u = torch.randn(1608, 4096, device=DEV).to(torch.bfloat16)
    du = gemm(a, b, epilogue=_lib.EPI_GELU_BWD, aux=u)
    dv = (a.float() @ b.float().t()).to(torch.bfloat16).float()
    x = u.float()
    grad = 0.5 * (1 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5
    assert _rel(du, dv * grad) < 2e-2


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_gemm_residual_dropout_epilogue(p):
    from radhip import _lib
    from radhip.ops import dropout_mask, gemm
    M, N, K = 1608, 1024, 4096
    a, b, bias = _ops(M, N, K, seed=3)
    h = torch.randn(M, N, device=DEV)
    seed = torch.tensor([4242], dtype=torch.int64, device=DEV)
    out = gemm(a, b, bias, epilogue=_lib.EPI_RESID_DROP, aux=h, seed=seed, salt=7, p_drop=p)
    assert out.dtype == torch.float32
    fo = (a.float() @ b.float().t() + bias.float()).to(torch.bfloat16).float()
    mk = dropout_mask(seed, 7, p, (M, N)).float() / (1 - p) if p > 0 else torch.ones_like(h)
    ref = h + fo * mk
    assert _rel(out - h, ref - h) < 2e-2
    if p > 0:   # the mask itself is exact: dropped elements carry h unchanged
        dropped = mk == 0
        assert torch.equal(out[dropped], h[dropped])


# ---- csrc/wgemm.hip: the LDS-DMA pipelined GEMM of the WavLM projections (every tile configuration) ----
WG_TILES = [0, 1, 5, 6, 11, 12, 13, 14, 15, 16, 17, 18]


@pytest.mark.parametrize("tile", WG_TILES)
@pytest.mark.parametrize("M,N,K", [(1608, 1024, 1024), (333, 3072, 1024), (1608, 4096, 128), (64, 260, 4096)])
def test_wgemm_bias_every_tile(tile, M, N, K):
    """Row tails (M % tile != 0: the buffer range returns zeros past the last row), column tails, deep K."""
    from radhip.ops import wgemm
    a, b, bias = _ops(M, N, K, seed=tile)
    got = wgemm(a, b, bias, tile=tile)
    assert got.dtype == torch.bfloat16 and got.shape == (M, N)
    assert _rel(got, a.float() @ b.float().t() + bias.float()) < 1e-2
    assert _rel(wgemm(a, b, tile=tile), a.float() @ b.float().t()) < 1e-2


@pytest.mark.parametrize("staged,unstaged", [(5, 45), (6, 46), (12, 52), (16, 56)])
def test_wgemm_staged_epilogue_bit_exact(staged, unstaged):
    """The LDS-staged row epilogue stores exactly what the per-lane fragment epilogue stored (same fp32
    accumulation, same roundings), for all three epilogues and a column tail (N = 4100)."""
    from radhip import _lib
    from radhip.ops import wgemm
    for N in (4096, 4100):
        a, b, bias = _ops(1608, N, 1024, seed=N + staged)
        assert torch.equal(wgemm(a, b, bias, tile=staged), wgemm(a, b, bias, tile=unstaged))
        u1, v1 = wgemm(a, b, bias, epilogue=_lib.EPI_BIAS_GELU, tile=staged)
        u2, v2 = wgemm(a, b, bias, epilogue=_lib.EPI_BIAS_GELU, tile=unstaged)
        assert torch.equal(u1, u2) and torch.equal(v1, v2)
        uu = torch.randn(1608, N, device=DEV).to(torch.bfloat16)
        assert torch.equal(wgemm(a, b, epilogue=_lib.EPI_GELU_BWD, aux=uu, tile=staged),
                           wgemm(a, b, epilogue=_lib.EPI_GELU_BWD, aux=uu, tile=unstaged))


@pytest.mark.parametrize("tile", [5, 6, 12])
def test_wgemm_gelu_epilogues(tile):
    from radhip import _lib
    from radhip.ops import wgemm
    a, b, bias = _ops(1608, 4096, 1024, seed=11)
    u, v = wgemm(a, b, bias, epilogue=_lib.EPI_BIAS_GELU, tile=tile)
    assert _rel(u, a.float() @ b.float().t() + bias.float()) < 1e-2
    ref_v = torch.nn.functional.gelu(u.float())
    assert float((v.float() - ref_v.to(torch.bfloat16).float()).abs().max()) <= 2 ** -7 * float(ref_v.abs().max())
    uu = torch.randn(1608, 4096, device=DEV).to(torch.bfloat16)
    du = wgemm(a, b, epilogue=_lib.EPI_GELU_BWD, aux=uu, tile=tile)
    dv = (a.float() @ b.float().t()).to(torch.bfloat16).float()
    x = uu.float()
    grad = 0.5 * (1 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5
    assert _rel(du, dv * grad) < 2e-2


def test_wgemm_policy_shapes_match_hipblaslt():
    """Every (GEMM, token count) the fused WavLM layer routes to wgemm (radhip.ops.wgemm_policy) agrees with
    hipBLASLt's bf16 result to bf16 rounding, with its epilogue."""
    from radhip import _lib
    from radhip.ops import layer_gemm, wgemm_policy
    shapes = {"qkv": (3072, 1024), "out": (1024, 1024), "ffn1": (4096, 1024), "ffn2": (1024, 4096),
              "d_ffn2": (4096, 1024), "d_ffn1": (1024, 4096), "d_out": (1024, 1024), "d_qkv": (1024, 3072)}
    n = 0
    for M in (1608, 6432):
        for name, (N, K) in shapes.items():
            pol = wgemm_policy(name, M, N, K)
            if pol is None:
                continue
            n += 1
            a, b, bias = _ops(M, N, K, seed=N + K)
            if name == "d_ffn2":
                uu = torch.randn(M, N, device=DEV).to(torch.bfloat16)
                got = layer_gemm(pol, a, b, epilogue=_lib.EPI_GELU_BWD, aux=uu)
                x = uu.float()
                grad = 0.5 * (1 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5
                ref = torch.mm(a, b.t()).float() * grad
                assert _rel(got, ref) < 2e-2, name
                continue
            epi = _lib.EPI_BIAS_GELU if name == "ffn1" else _lib.EPI_BIAS
            got = layer_gemm(pol, a, b, bias, epilogue=epi)
            got = got[0] if isinstance(got, tuple) else got
            ref = torch.nn.functional.linear(a, b, bias)
            assert _rel(got, ref) < 1e-2, name
    assert n > 0


@pytest.mark.parametrize("tile,splits", [(12, 4), (20, 2), (5, 3), (16, 7)])
@pytest.mark.parametrize("M,N,K", [(1608, 1024, 4096), (333, 260, 3072)])
def test_wgemm_split_k(tile, splits, M, N, K):
    """Split-K with the last-arriver reduction: equal to the unsplit launch up to fp32 summation order, bit-for-bit
    repeatable (fixed split order whoever arrives last; the tickets re-zero themselves between launches), every
    epilogue, row and column tails."""
    from radhip import _lib
    from radhip.ops import wgemm
    a, b, bias = _ops(M, N, K, seed=splits)
    ref = a.float() @ b.float().t() + bias.float()
    outs = [wgemm(a, b, bias, tile=tile, splits=splits) for _ in range(3)]
    assert _rel(outs[0], ref) < 1e-2
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    one = wgemm(a, b, bias, tile=tile)
    assert float((outs[0].float() - one.float()).abs().max()) <= 2 ** -7 * float(one.float().abs().max())
    u, v = wgemm(a, b, bias, epilogue=_lib.EPI_BIAS_GELU, tile=tile, splits=splits)
    assert torch.equal(u, outs[0])
    assert torch.equal(v, torch.nn.functional.gelu(u.float()).to(torch.bfloat16)) or \
        float((v.float() - torch.nn.functional.gelu(u.float())).abs().max()) <= 2 ** -7 * float(v.float().abs().max())
    uu = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    du = wgemm(a, b, epilogue=_lib.EPI_GELU_BWD, aux=uu, tile=tile, splits=splits)
    du1 = wgemm(a, b, epilogue=_lib.EPI_GELU_BWD, aux=uu, tile=tile)
    assert _rel(du, du1) < 1e-2


# ---- csrc/pgemm.hip: the deep-pipelined 8-wave GEMM (every tile code, both K-step forms, group orders) ----
PG_TILES = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 104]


@pytest.mark.parametrize("tile", PG_TILES)
@pytest.mark.parametrize("M,N,K,gm", [(1608, 1024, 1024, 4), (333, 3072, 1024, 0), (1608, 4096, 128, 2),
                                      (64, 768, 4096, 1), (6432, 1024, 192, 8)])
def test_pgemm_bias_every_tile(tile, M, N, K, gm):
    """Row tails (rows past M read as zeros through the buffer range), column tiles, K = 2 steps (shorter than the
    ring) up to deep K, every group order."""
    from radhip.ops import pgemm
    a, b, bias = _ops(M, N, K, seed=tile + gm)
    got = pgemm(a, b, bias, tile=tile, group_m=gm)
    assert got.dtype == torch.bfloat16 and got.shape == (M, N)
    assert _rel(got, a.float() @ b.float().t() + bias.float()) < 1e-2
    assert _rel(pgemm(a, b, tile=tile, group_m=gm), a.float() @ b.float().t()) < 1e-2


@pytest.mark.parametrize("tile", [0, 2, 4, 5, 7])
def test_pgemm_epilogues_match_wgemm(tile):
    """The bias / bias + GELU / GELU-backward epilogues round where csrc/wgemm.hip's do: same values up to the
    fp32 summation order of the accumulator (bf16 rounding of C), the aux output gelu(u) of the stored u."""
    from radhip import _lib
    from radhip.ops import pgemm, wgemm
    a, b, bias = _ops(1608, 3072, 1024, seed=5)
    u, v = pgemm(a, b, bias, epilogue=_lib.EPI_BIAS_GELU, tile=tile)
    u2, v2 = wgemm(a, b, bias, epilogue=_lib.EPI_BIAS_GELU, tile=5)
    assert float((u.float() - u2.float()).abs().max()) <= 2 ** -7 * float(u2.float().abs().max())
    ref_v = torch.nn.functional.gelu(u.float())
    assert float((v.float() - ref_v.to(torch.bfloat16).float()).abs().max()) <= 2 ** -7 * float(ref_v.abs().max())
    uu = torch.randn(1608, 3072, device=DEV).to(torch.bfloat16)
    du = pgemm(a, b, epilogue=_lib.EPI_GELU_BWD, aux=uu, tile=tile)
    x = uu.float()
    grad = 0.5 * (1 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5
    assert _rel(du, (a.float() @ b.float().t()).to(torch.bfloat16).float() * grad) < 2e-2
    # repeatable: the same launch twice gives the same bits (no split, fixed summation order)
    assert torch.equal(pgemm(a, b, bias, tile=tile), pgemm(a, b, bias, tile=tile))


def test_pgemm_probe_stamps():
    """The diagnostic form stores per-workgroup stamps in order (entry <= stage 0 landed <= loop done <= exit) and
    the same C as the product form."""
    import ctypes
    from radhip import _lib
    from radhip.ops import pgemm
    a, b, bias = _ops(1608, 3072, 1024, seed=9)
    c = torch.empty(1608, 3072, device=DEV, dtype=torch.bfloat16)
    grid = 13 * 16
    prof = torch.zeros(grid, 8, dtype=torch.int64, device=DEV)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = _lib.lib().rdx_pgemm_prof(P(a), 1024, P(b), 1024, P(c), 3072, 1608, 3072, 1024, P(bias), 4, 4, P(prof), st)
    assert rc == 0
    torch.cuda.synchronize()
    assert torch.equal(c, pgemm(a, b, bias, tile=4, group_m=4))
    d = prof.cpu()
    assert bool(((d[:, 0] <= d[:, 1]) & (d[:, 1] <= d[:, 2]) & (d[:, 2] <= d[:, 3])).all())
    assert bool((d[:, 5] >= d[:, 4]).all())


# ---- csrc/hgemm.hip: the 8-wave ping-pong GEMM with the slab ring (every tile, split-K, group orders) ----
HG_TILES = [0, 1, 2, 3, 4, 5, 6, 7, 100, 202, 206]


@pytest.mark.parametrize("tile", HG_TILES)
@pytest.mark.parametrize("M,N,K,splits,gm", [(1608, 1024, 1024, 1, 4), (333, 3072, 1024, 1, 0),
                                             (1608, 4096, 128, 1, 2), (64, 768, 4096, 1, 1),
                                             (6432, 1024, 192, 1, 8), (1608, 1024, 4096, 2, 0),
                                             (200, 1000, 1024, 3, 0), (130, 260, 128, 2, 1),
                                             (1608, 1024, 4096, 2, -2), (1608, 3072, 1024, 1, -4),
                                             (6432, 4096, 256, 1, -2), (333, 260, 256, 3, -8), (130, 1000, 128, 1, -1)])
def test_hgemm_bias_every_tile(tile, M, N, K, splits, gm):
    """Row tails (rows past M read as zeros through the buffer range), ragged column tiles (N % 8 == 4 takes the
    8-byte row phase), K of 2-3 steps (shorter than the ring: the refills past the last step take the zero-record
    descriptor) up to deep K, split-K with the last-arriver sum, every group order (gm < 0: the R x 8/R XCD grid,
    with empty and uneven blocks)."""
    from radhip.ops import hgemm
    a, b, bias = _ops(M, N, K, seed=tile + gm + splits)
    got = hgemm(a, b, bias, tile=tile, splits=splits, group_m=gm)
    assert got.dtype == torch.bfloat16 and got.shape == (M, N)
    assert _rel(got, a.float() @ b.float().t() + bias.float()) < 1e-2
    assert _rel(hgemm(a, b, tile=tile, splits=splits, group_m=gm), a.float() @ b.float().t()) < 1e-2


@pytest.mark.parametrize("tile,splits", [(0, 1), (2, 1), (3, 1), (4, 2), (1, 1), (6, 1), (7, 2)])
def test_hgemm_epilogues_match_wgemm(tile, splits):
    """The bias / bias + GELU / GELU-backward epilogues round where csrc/wgemm.hip's do (bf16 rounding of C, the
    aux output gelu(u) of the stored u); split-K sums in split order, so two launches give the same bits."""
    from radhip import _lib
    from radhip.ops import hgemm, wgemm
    a, b, bias = _ops(1608, 3072, 1024, seed=5)
    u, v = hgemm(a, b, bias, epilogue=_lib.EPI_BIAS_GELU, tile=tile, splits=splits)
    u2, v2 = wgemm(a, b, bias, epilogue=_lib.EPI_BIAS_GELU, tile=5)
    assert float((u.float() - u2.float()).abs().max()) <= 2 ** -7 * float(u2.float().abs().max())
    ref_v = torch.nn.functional.gelu(u.float())
    assert float((v.float() - ref_v.to(torch.bfloat16).float()).abs().max()) <= 2 ** -7 * float(ref_v.abs().max())
    uu = torch.randn(1608, 3072, device=DEV).to(torch.bfloat16)
    du = hgemm(a, b, epilogue=_lib.EPI_GELU_BWD, aux=uu, tile=tile, splits=splits)
    x = uu.float()
    grad = 0.5 * (1 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5
    assert _rel(du, (a.float() @ b.float().t()).to(torch.bfloat16).float() * grad) < 2e-2
    assert torch.equal(hgemm(a, b, bias, tile=tile, splits=splits), hgemm(a, b, bias, tile=tile, splits=splits))


def test_hgemm_strided_views():
    """A as a column slice of a wider buffer and C written into a column slice (the fused layer's q/k/v views)."""
    from radhip.ops import hgemm
    a, b, bias = _ops(401, 512, 1024, lda=1088)
    out = torch.zeros(401, 1536, device=DEV, dtype=torch.bfloat16)
    hgemm(a, b, bias, out=out[:, 512:1024], tile=2)
    assert _rel(out[:, 512:1024], a.float() @ b.float().t() + bias.float()) < 1e-2
    assert float(out[:, :512].abs().max()) == 0.0 and float(out[:, 1024:].abs().max()) == 0.0


@pytest.mark.parametrize("tile", [2, 3, 4])
@pytest.mark.parametrize("M,N,K", [(1608, 1024, 4096), (1608, 1024, 1024), (6432, 1024, 3072), (200, 1000, 256),
                                   (64, 128, 64), (1608, 3072, 1024)])
def test_hgemm_stream_k(tile, M, N, K):
    """Stream-K (splits 0): runs of (tile, K step) units cut tiles anywhere (a tile may be shared by up to
    `maxc` runs, or held whole); fewer units than CUs (64 x 128 x 64); ragged M / N. The shared tiles' partials are
    summed in K order by their last arriver: two launches give the same bits."""
    from radhip import _lib
    from radhip.ops import hgemm
    a, b, bias = _ops(M, N, K, seed=tile + K)
    got = hgemm(a, b, bias, tile=tile, splits=0)
    assert _rel(got, a.float() @ b.float().t() + bias.float()) < 1e-2
    assert torch.equal(got, hgemm(a, b, bias, tile=tile, splits=0))
    uu = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    du = hgemm(a, b, epilogue=_lib.EPI_GELU_BWD, aux=uu, tile=tile, splits=0)
    x = uu.float()
    grad = 0.5 * (1 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5
    assert _rel(du, (a.float() @ b.float().t()).to(torch.bfloat16).float() * grad) < 2e-2
