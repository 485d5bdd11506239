// bf16 MFMA GEMM with fused epilogues for the WavLM encoder layer (the q/k/v + LoRA columns, out_proj and
// FFN projections of HF WavLMEncoderLayerStableLayerNorm, as run by WavLMFrontend,
// src/models/DualStreamSEMamba.py:292-439), forward and input-gradient.
//
//   C[M, N] = A[M, K] . B[N, K]^T   (both operands K-contiguous rows: x @ W^T of F.linear; the input
//                                     gradients use the transposed frozen weight cached as [K_out][N_in])
// epilogues (fp32 accumulator -> output):
//   RDX_EPI_BIAS       C = bf16(acc + bias)                             (bias optional)
//   RDX_EPI_BIAS_GELU  C = u = bf16(acc + bias), aux_out = bf16(gelu(u))    (FFN1 + GELU)
//   RDX_EPI_GELU_BWD   C = bf16(bf16(acc) * gelu'(aux))                 (FFN2 input grad + GELU backward)
//   RDX_EPI_RESID_DROP C(fp32) = aux(fp32) + bf16(acc + bias) * dropout   (FFN2 + dropout + residual)
// Each output rounds exactly where the unfused layer (hipBLASLt bf16 GEMM + the elementwise kernels of
// csrc/wavlm_layer.hip) rounds, so the fusion changes no value.
//
// Tiling: 128 x 128 output tile per 256-thread workgroup (4 waves of 64 x 64, 2 x 2 mfma_f32_32x32x16_bf16
// tiles each), K in steps of 64 through two LDS buffers (register-staged: the next step's global loads are
// in flight while the current step's MFMAs run), one barrier per K step. The MFMA computes C^T (the B
// tile is the A operand), so each lane owns one output row and 4-column groups: 8-byte bf16 / 16-byte fp32
// stores and fp32 residual loads. LDS rows are 128 B with the 16-byte chunk XOR-swizzled by
// (row >> 1) & 7, conflict-free for the ds_read_b128 fragment reads of both operands. Tiles are dealt to
// XCDs by column panel (a panel of B stays in one XCD's L2) when the column-tile count is a multiple of 8.
#include "common.h"

namespace rdx {

typedef __attribute__((ext_vector_type(16))) float gf32x16;

constexpr int GM = 128, GN = 128, GK = 64;
constexpr int G_THREADS = 256;
constexpr int G_TILE = GM * GK * 2;  // one operand tile: 16 KB

__device__ __forceinline__ int g_slot(int row, int ch) { return row * 128 + 16 * (ch ^ ((row >> 1) & 7)); }

__device__ __forceinline__ gf32x16 g_mfma(hx8 a, hx8 b, gf32x16 c) {
  return mfma32x32x16(a, b, c);
}

__device__ __forceinline__ float g_gelu(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float g_gelu_grad(float x) {
  return 0.5f * (1.0f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}
__device__ __forceinline__ uint32_t g_pack2(float a, float b) {
  hst x = f2h(a), y = f2h(b);
  return (uint32_t)(*reinterpret_cast<uint16_t*>(&x)) | ((uint32_t)(*reinterpret_cast<uint16_t*>(&y)) << 16);
}

struct GemmArgs {
  const hst* A;
  int64_t lda;
  const hst* B;
  int64_t ldb;
  void* C;
  int64_t ldc;
  int M, N, K;
  const hst* bias;  // [N] or null
  const void* aux;             // GELU_BWD: u bf16 [M, ldaux]; RESID_DROP: h fp32 [M, ldaux]
  int64_t ldaux;
  hst* aux_out;     // BIAS_GELU: gelu(u) bf16 [M, ldao]
  int64_t ldao;
  const int64_t* seed_dev;     // RESID_DROP dropout (element index m * N + n, csrc/wavlm_layer.hip hash)
  int salt;
  uint32_t thr;
  float inv_keep;
  int tiles_n;
  int xcd_panels;              // 1: deal column panels to XCDs
  int64_t sA;                  // batched (grid.y = batch index z): A advances z * sA elements and the
  int64_t crow;                //   output (and aux) row index by z * crow rows
};

template <int EPI>
__global__ __launch_bounds__(G_THREADS, 2) void gemm_nt_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) char g_lds[];
  const int tn = g.tiles_n;
  int mt, ntile;
  {
    const int bid = blockIdx.x;
    if (g.xcd_panels) {  // blocks b and b + 8 share an XCD: give each XCD whole column panels
      const int xcd = bid & 7, loc = bid >> 3, per = tn >> 3;
      ntile = xcd * per + loc % per;
      mt = loc / per;
    } else {
      mt = bid / tn;
      ntile = bid % tn;
    }
  }
  const int m0 = mt * GM, n0 = ntile * GN;
  const hst* __restrict__ Ab = g.A + (int64_t)blockIdx.y * g.sA;
  const int64_t mrow0 = (int64_t)blockIdx.y * g.crow;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wm = w >> 1, wn = w & 1;
  const int M = g.M, N = g.N, K = g.K;
  const int nk = (K + GK - 1) / GK;

  hx8 ra[4], rb[4];
  auto gload = [&](int kt) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int id = tid + G_THREADS * j, row = id >> 3, ch = id & 7;
      const int k = kt * GK + 8 * ch;
      const int am = m0 + row, bn = n0 + row;
      hx8 z;
#pragma unroll
      for (int e = 0; e < 8; ++e) z[e] = (hel)0.f;
      ra[j] = (am < M && k < K) ? *reinterpret_cast<const hx8*>(Ab + (int64_t)am * g.lda + k) : z;
      rb[j] = (bn < N && k < K) ? *reinterpret_cast<const hx8*>(g.B + (int64_t)bn * g.ldb + k) : z;
    }
  };
  auto swrite = [&](int buf) {
    char* base = g_lds + buf * 2 * G_TILE;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int id = tid + G_THREADS * j, row = id >> 3, ch = id & 7;
      *reinterpret_cast<hx8*>(base + g_slot(row, ch)) = ra[j];
      *reinterpret_cast<hx8*>(base + G_TILE + g_slot(row, ch)) = rb[j];
    }
  };

  gf32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  gload(0);
  swrite(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) gload(kt + 1);
    const char* As = g_lds + (kt & 1) * 2 * G_TILE;
    const char* Bs = As + G_TILE;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      hx8 af[2], bfr[2];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) af[mi] = *reinterpret_cast<const hx8*>(As + g_slot(wm * 64 + mi * 32 + r, 2 * s + h));
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
        bfr[ni] = *reinterpret_cast<const hx8*>(Bs + g_slot(wn * 64 + ni * 32 + r, 2 * s + h));
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = g_mfma(bfr[ni], af[mi], acc[mi][ni]);  // C^T tile
    }
    if (kt + 1 < nk) swrite((kt + 1) & 1);
    __syncthreads();
  }

  // ---- epilogue: lane owns output row m, columns n .. n + 3 of each 4-group (rows crow(4c + e, h) of C^T)
  const uint64_t seed = (EPI == RDX_EPI_RESID_DROP && g.thr) ? attn_seed(g.seed_dev, g.salt) : 0;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const int m = m0 + wm * 64 + mi * 32 + r;
    if (m >= M) continue;
    const int64_t mg = mrow0 + m;
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int n = n0 + wn * 64 + ni * 32 + 8 * c + 4 * h;
        if (n >= N) continue;  // N % 4 == 0: a group is all in or all out
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[mi][ni][4 * c + e];
        if (EPI != RDX_EPI_GELU_BWD && g.bias) {
          const uint2 bb = *reinterpret_cast<const uint2*>(g.bias + n);
          v[0] += hlo(bb.x);
          v[1] += hhi(bb.x);
          v[2] += hlo(bb.y);
          v[3] += hhi(bb.y);
        }
        if (EPI == RDX_EPI_BIAS) {
          *reinterpret_cast<uint2*>(reinterpret_cast<hst*>(g.C) + mg * g.ldc + n) =
              make_uint2(g_pack2(v[0], v[1]), g_pack2(v[2], v[3]));
        } else if (EPI == RDX_EPI_BIAS_GELU) {
          float u[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) u[e] = hround(v[e]);
          *reinterpret_cast<uint2*>(reinterpret_cast<hst*>(g.C) + mg * g.ldc + n) =
              make_uint2(g_pack2(u[0], u[1]), g_pack2(u[2], u[3]));
          *reinterpret_cast<uint2*>(g.aux_out + mg * g.ldao + n) =
              make_uint2(g_pack2(g_gelu(u[0]), g_gelu(u[1])), g_pack2(g_gelu(u[2]), g_gelu(u[3])));
        } else if (EPI == RDX_EPI_GELU_BWD) {
          const uint2 uu = *reinterpret_cast<const uint2*>(reinterpret_cast<const hst*>(g.aux) +
                                                           mg * g.ldaux + n);
          const float u[4] = {hlo(uu.x), hhi(uu.x),
                              hlo(uu.y), hhi(uu.y)};
          float d[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) d[e] = hround(v[e]) * g_gelu_grad(u[e]);
          *reinterpret_cast<uint2*>(reinterpret_cast<hst*>(g.C) + mg * g.ldc + n) =
              make_uint2(g_pack2(d[0], d[1]), g_pack2(d[2], d[3]));
        } else {  // RDX_EPI_RESID_DROP
          const float4 hv = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(g.aux) +
                                                             mg * g.ldaux + n);
          const float hx[4] = {hv.x, hv.y, hv.z, hv.w};
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float fo = hround(v[e]);
            const float ms = g.thr ? (drop_keep(seed, (uint64_t)m * N + n + e, g.thr) ? g.inv_keep : 0.f) : 1.f;
            o[e] = hx[e] + fo * ms;
          }
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(g.C) + mg * g.ldc + n) =
              make_float4(o[0], o[1], o[2], o[3]);
        }
      }
    }
  }
}

template <int EPI>
static int gemm_launch(const GemmArgs& g, hipStream_t st, int batch = 1) {
  const int tm = (g.M + GM - 1) / GM;
  hipLaunchKernelGGL((gemm_nt_kernel<EPI>), dim3((unsigned)(tm * g.tiles_n), (unsigned)batch), dim3(G_THREADS),
                     4 * G_TILE, st, g);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

}  // namespace rdx

using namespace rdx;

extern "C" int rdx_gemm_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N,
                             int K, const void* bias, int epilogue, const void* aux, int64_t ldaux, void* aux_out,
                             int64_t ldao, const int64_t* seed_dev, int salt, float p_drop, void* stream) {
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  RDX_REQUIRE(A && B && C && M > 0 && N > 0 && K > 0 && al(A) && al(B) && al(C));
  RDX_REQUIRE(lda % 8 == 0 && ldb % 8 == 0 && K % 8 == 0 && N % 4 == 0 && lda >= K && ldb >= K && ldc >= N);
  RDX_REQUIRE(!bias || ((uintptr_t)bias & 7) == 0);
  RDX_REQUIRE(epilogue >= RDX_EPI_BIAS && epilogue <= RDX_EPI_RESID_DROP);
  RDX_REQUIRE(epilogue == RDX_EPI_BIAS || ldc % 4 == 0);
  if (epilogue == RDX_EPI_BIAS_GELU) RDX_REQUIRE(aux_out && ldao >= N && ldao % 4 == 0 && ((uintptr_t)aux_out & 7) == 0);
  if (epilogue == RDX_EPI_GELU_BWD) RDX_REQUIRE(aux && ldaux >= N && ldaux % 4 == 0 && ((uintptr_t)aux & 7) == 0);
  if (epilogue == RDX_EPI_RESID_DROP) {
    RDX_REQUIRE(aux && al(aux) && al(C) && ldaux >= N && ldaux % 4 == 0 && ldc % 4 == 0);
    RDX_REQUIRE(p_drop >= 0.f && p_drop < 1.f && (p_drop == 0.f || seed_dev));
  }
  RDX_REQUIRE(ldc % 4 == 0 || epilogue == RDX_EPI_BIAS);
  GemmArgs g;
  g.A = (const hst*)A;
  g.lda = lda;
  g.B = (const hst*)B;
  g.ldb = ldb;
  g.C = C;
  g.ldc = ldc;
  g.M = M;
  g.N = N;
  g.K = K;
  g.bias = (const hst*)bias;
  g.aux = aux;
  g.ldaux = ldaux;
  g.aux_out = (hst*)aux_out;
  g.ldao = ldao;
  g.seed_dev = seed_dev;
  g.salt = salt;
  g.thr = (epilogue == RDX_EPI_RESID_DROP && p_drop > 0.f) ? (uint32_t)fminf(4294967295.0f, p_drop * 4294967296.0f) : 0u;
  g.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  g.tiles_n = (N + GN - 1) / GN;
  g.xcd_panels = (g.tiles_n % 8 == 0) ? 1 : 0;
  g.sA = 0;
  g.crow = 0;
  const int64_t tiles = (int64_t)((M + GM - 1) / GM) * g.tiles_n;
  RDX_REQUIRE(tiles <= 0x7fffffff);
  hipStream_t st = as_stream(stream);
  switch (epilogue) {
    case RDX_EPI_BIAS: return gemm_launch<RDX_EPI_BIAS>(g, st);
    case RDX_EPI_BIAS_GELU: return gemm_launch<RDX_EPI_BIAS_GELU>(g, st);
    case RDX_EPI_GELU_BWD: return gemm_launch<RDX_EPI_GELU_BWD>(g, st);
    default: return gemm_launch<RDX_EPI_RESID_DROP>(g, st);
  }
}

// Batched / implicit-GEMM form, bias epilogue only: for z < batch, C[z*crow + m, :] = bf16(A_z[m, :] . B^T + bias)
// with A_z = A + z*sA, row m at A_z + m*lda. lda may be SMALLER than K: rows then overlap, which is how a
// strided convolution over token-major activations reads its im2col matrix in place (featconv.hip).
extern "C" int rdx_gemm_bf16_strided(const void* A, int64_t lda, int64_t sA, const void* B, int64_t ldb, void* C,
                                     int64_t ldc, int64_t crow, int batch, int M, int N, int K, const void* bias,
                                     void* stream) {
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  RDX_REQUIRE(A && B && C && M > 0 && N > 0 && K > 0 && batch > 0 && batch <= 65535 && al(A) && al(B) && al(C));
  RDX_REQUIRE(lda > 0 && lda % 8 == 0 && sA >= 0 && sA % 8 == 0 && ldb % 8 == 0 && ldb >= K && K % 8 == 0);
  RDX_REQUIRE(N % 4 == 0 && ldc >= N && ldc % 4 == 0 && crow >= 0 && (batch == 1 || crow >= M));
  RDX_REQUIRE(!bias || ((uintptr_t)bias & 7) == 0);
  GemmArgs g;
  g.A = (const hst*)A;
  g.lda = lda;
  g.B = (const hst*)B;
  g.ldb = ldb;
  g.C = C;
  g.ldc = ldc;
  g.M = M;
  g.N = N;
  g.K = K;
  g.bias = (const hst*)bias;
  g.aux = nullptr;
  g.ldaux = 0;
  g.aux_out = nullptr;
  g.ldao = 0;
  g.seed_dev = nullptr;
  g.salt = 0;
  g.thr = 0;
  g.inv_keep = 1.f;
  g.tiles_n = (N + GN - 1) / GN;
  g.xcd_panels = (g.tiles_n % 8 == 0) ? 1 : 0;
  g.sA = sA;
  g.crow = crow;
  const int64_t tiles = (int64_t)((M + GM - 1) / GM) * g.tiles_n;
  RDX_REQUIRE(tiles <= 0x7fffffff);
  return gemm_launch<RDX_EPI_BIAS>(g, as_stream(stream), batch);
}
