// Small-GEMM kernel of the detector head (the fusion, PN-BiMamba, pooling and classifier linears,
// src/models/DualStreamSEMamba.py:445-531,537-637,700-770): C[M, N] = A[M, K] W[N, K]^T with the linear's bias and the
// operations autocast puts around it fused into one launch.
//
// The head's shapes are narrow (N, K in {1, 2, 9, 41, 64, 144, 288, 576, 1024}) over 1 608 - 12 864 token rows: each
// GEMM is a few hundred MFLOP and its time is launch and load latency, not arithmetic (hipBLASLt took 7-9 us per
// call on them, and the casts, GELU, residual add and bias reduction around them were launches of their own). Here a
// 256-thread workgroup owns 32 token rows x 64 output features; it loads whole K chunks of 320 (every head K but
// 576 and 1024 in one chunk) with all of its loads in flight at once, prefetching the next chunk into registers
// while the MFMAs (v_mfma_f32_16x16x32, wave w: features 16 w .. 16 w + 15 of the tile, both 16-row token tiles)
// run on the current one from LDS. Operands may be strided views with any K (the x_proj output's dt columns):
// 16-byte loads where rows are 16-byte aligned, element loads with zero fill elsewhere. A may be fp32 (converted to
// the 16-bit type on load, the cast F.linear's autocast does first).
//
// Epilogues, each the rounding sequence of the unfused autocast ops:
//   RDX_EPI_BIAS      C = half(acc + bias)                         (F.linear; bias optional)
//   RDX_EPI_BIAS_GELU C = u = half(acc + bias), aux_out = half(gelu(u))      (F.linear then nn.GELU)
//   RDX_EPI_GELU_BWD  C = half(half(acc) * gelu'(aux))            (the input-gradient matmul, then GELU's backward)
// then C = R + C in C's type when a residual R (of C's type) is given: fp32 (x + ffn(...).to(x.dtype)) or 16-bit
// (round(R + C): autograd's sum of two 16-bit gradients). C may alias R (each element is read, then written, by one
// thread).
#include "common.h"

namespace rdx {
namespace lg {

constexpr int BM = 32;          // token rows per workgroup
constexpr int BN = 64;          // output features per workgroup (16 per wave)
constexpr int KC = 320;         // K chunk staged in LDS
constexpr int KP = KC + 8;      // LDS row pitch (16-bit elements): 656 B, rows 36 banks apart (conflict-free b128)
constexpr int T = 256;
constexpr int CH = KC / 8;      // 16-byte items per row chunk
constexpr int A_IT = BM * CH / T;   // 5
constexpr int B_IT = BN * CH / T;   // 10
constexpr int LDS = (BM + BN) * KP * 2;

struct Args {
  const void* A;     // [M, K] rows at lda (16-bit storage type, or fp32 when A_F32)
  int64_t lda;
  const hst* W;      // [N, K] rows at ldw
  int64_t ldw;
  void* C;           // [M, N] rows at ldc (16-bit, or fp32 when C_F32)
  int64_t ldc;
  const hst* bias;   // [N] or null
  const hst* aux;    // GELU_BWD: u [M, N] rows at ldaux
  int64_t ldaux;
  hst* aux_out;      // GELU: gelu(u) [M, N] rows at ldao
  int64_t ldao;
  const void* R;     // residual [M, N] of C's type, rows at ldr, or null
  int64_t ldr;
  int M, N, K;
  int vec_a, vec_w;  // rows 16-byte aligned (16-byte loads where 8 elements fit)
  int vec_c;         // C rows 8-byte (16-bit) / 16-byte (fp32) aligned
};

// 8 consecutive elements of row `row` from column k as packed 16-bit values, zero past nrows / K
template <bool F32>
__device__ __forceinline__ uint4 load8(const void* base, int64_t ld, int row, int nrows, int k, int K, bool vec) {
  uint4 z = make_uint4(0u, 0u, 0u, 0u);
  if (row >= nrows || k >= K) return z;
  if constexpr (F32) {
    const float* p = reinterpret_cast<const float*>(base) + (int64_t)row * ld + k;
    float v[8];
    if (vec && k + 8 <= K) {
      const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = k + j < K ? p[j] : 0.f;
    }
    return make_uint4(hpack2(v[0], v[1]), hpack2(v[2], v[3]), hpack2(v[4], v[5]), hpack2(v[6], v[7]));
  } else {
    const uint16_t* p = reinterpret_cast<const uint16_t*>(base) + (int64_t)row * ld + k;
    if (vec && k + 8 <= K) return *reinterpret_cast<const uint4*>(p);
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t lo = k + 2 * j < K ? p[2 * j] : 0u, hi = k + 2 * j + 1 < K ? p[2 * j + 1] : 0u;
      w[j] = lo | (hi << 16);
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
}

template <bool A_F32, bool C_F32, int EPI>
__global__ __launch_bounds__(T, 2) void lgemm_kernel(Args g) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  uint16_t* As = reinterpret_cast<uint16_t*>(lds);   // [BM][KP]
  uint16_t* Ws = As + BM * KP;                         // [BN][KP]
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, l16 = lane & 15, lg = lane >> 4;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int nch = (g.K + KC - 1) / KC;
  uint4 ra[A_IT], rw[B_IT];
  auto fetch = [&](int c) {
    const int k0 = c * KC, kcp = min(KC, ((g.K - k0 + 31) / 32) * 32);
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int it = tid + T * i, row = it / CH, kk = (it % CH) * 8;
      ra[i] = kk < kcp ? load8<A_F32>(g.A, g.lda, m0 + row, g.M, k0 + kk, g.K, g.vec_a) : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
      const int it = tid + T * i, row = it / CH, kk = (it % CH) * 8;
      rw[i] = kk < kcp ? load8<false>(g.W, g.ldw, n0 + row, g.N, k0 + kk, g.K, g.vec_w) : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  rdx_f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  fetch(0);
  for (int c = 0; c < nch; ++c) {
    const int k0 = c * KC, kcp = min(KC, ((g.K - k0 + 31) / 32) * 32);
    if (c > 0) __syncthreads();   // the previous chunk's MFMA reads are done
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int it = tid + T * i, row = it / CH, kk = (it % CH) * 8;
      if (kk < kcp) *reinterpret_cast<uint4*>(As + row * KP + kk) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
      const int it = tid + T * i, row = it / CH, kk = (it % CH) * 8;
      if (kk < kcp) *reinterpret_cast<uint4*>(Ws + row * KP + kk) = rw[i];
    }
    __syncthreads();
    if (c + 1 < nch) fetch(c + 1);
    // D^T tiles: A operand = the weights (rows = features 16 wv + l16), B operand = tokens l16 / 16 + l16
    const uint16_t* wp = Ws + (16 * wv + l16) * KP + 8 * lg;
    const uint16_t* ap0 = As + l16 * KP + 8 * lg;
    const uint16_t* ap1 = ap0 + 16 * KP;
    for (int ks = 0; ks < kcp; ks += 32) {
      const hx8 w = *reinterpret_cast<const hx8*>(wp + ks);
      acc0 = mfma16x16x32(w, *reinterpret_cast<const hx8*>(ap0 + ks), acc0);
      acc1 = mfma16x16x32(w, *reinterpret_cast<const hx8*>(ap1 + ks), acc1);
    }
  }
  // lane holds features n = n0 + 16 wv + 4 lg + i (i < 4) of token m0 + l16 (acc0) and m0 + 16 + l16 (acc1)
  const int n = n0 + 16 * wv + 4 * lg;
  if (n >= g.N) return;
  const int nv = min(4, g.N - n);
  float bv[4] = {0.f, 0.f, 0.f, 0.f};
  if (EPI != RDX_EPI_GELU_BWD && g.bias) {
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[i] = i < nv ? h2f(g.bias[n + i]) : 0.f;
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int m = m0 + 16 * t + l16;
    if (m >= g.M) continue;
    const rdx_f32x4 a = t ? acc1 : acc0;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = hround(a[i] + bv[i]);
    if constexpr (EPI == RDX_EPI_GELU_BWD) {
      const hst* up = g.aux + (int64_t)m * g.ldaux + n;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = i < nv ? hround(v[i] * gelu_grad(h2f(up[i]))) : 0.f;
    }
    if constexpr (EPI == RDX_EPI_BIAS_GELU) {
      hst* gp = g.aux_out + (int64_t)m * g.ldao + n;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < nv) gp[i] = f2h(gelu(v[i]));
    }
    if constexpr (C_F32) {
      float* cp = reinterpret_cast<float*>(g.C) + (int64_t)m * g.ldc + n;
      if (g.R) {
        const float* rp = reinterpret_cast<const float*>(g.R) + (int64_t)m * g.ldr + n;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = i < nv ? rp[i] + v[i] : 0.f;
      }
      if (nv == 4 && g.vec_c) {
        *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (i < nv) cp[i] = v[i];
      }
    } else {
      hst* cp = reinterpret_cast<hst*>(g.C) + (int64_t)m * g.ldc + n;
      if (g.R) {
        const hst* rp = reinterpret_cast<const hst*>(g.R) + (int64_t)m * g.ldr + n;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = i < nv ? hround(h2f(rp[i]) + v[i]) : 0.f;
      }
      if (nv == 4 && g.vec_c) {
        *reinterpret_cast<uint2*>(cp) = make_uint2(hpack2(v[0], v[1]), hpack2(v[2], v[3]));
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (i < nv) cp[i] = f2h(v[i]);
      }
    }
  }
}

template <bool A_F32, bool C_F32, int EPI>
int launch(const Args& g, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&lgemm_kernel<A_F32, C_F32, EPI>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  hipLaunchKernelGGL((lgemm_kernel<A_F32, C_F32, EPI>), dim3((unsigned)((g.N + BN - 1) / BN), (unsigned)((g.M + BM - 1) / BM)),
                     dim3(T), LDS, st, g);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

}  // namespace lg
}  // namespace rdx

using namespace rdx;

extern "C" int rdx_lgemm(const void* A, int64_t lda, int a_f32, const void* W, int64_t ldw, void* C, int64_t ldc,
                         int c_f32, int M, int N, int K, const void* bias, int epilogue, const void* aux, int64_t ldaux,
                         void* aux_out, int64_t ldao, const void* R, int64_t ldr, void* stream) {
  RDX_REQUIRE(A && W && C && M > 0 && N > 0 && K > 0 && M < (1 << 24) && N < (1 << 20));
  RDX_REQUIRE(lda >= K && ldw >= K && ldc >= N);
  RDX_REQUIRE(epilogue == RDX_EPI_BIAS || epilogue == RDX_EPI_BIAS_GELU || epilogue == RDX_EPI_GELU_BWD);
  RDX_REQUIRE(epilogue != RDX_EPI_BIAS_GELU || (aux_out && ldao >= N && !c_f32));
  RDX_REQUIRE(epilogue != RDX_EPI_GELU_BWD || (aux && ldaux >= N && !bias));
  RDX_REQUIRE(!R || ldr >= N);
  lg::Args g{A, lda, (const hst*)W, ldw, C, ldc, (const hst*)bias, (const hst*)aux, ldaux, (hst*)aux_out, ldao,
             R, ldr, M, N, K, 0, 0, 0};
  g.vec_a = (((uintptr_t)A & 15) == 0 && (lda % (a_f32 ? 4 : 8)) == 0) ? 1 : 0;
  g.vec_w = (((uintptr_t)W & 15) == 0 && (ldw % 8) == 0) ? 1 : 0;
  g.vec_c = c_f32 ? ((((uintptr_t)C & 15) == 0 && (ldc % 4) == 0) ? 1 : 0)
                  : ((((uintptr_t)C & 7) == 0 && (ldc % 4) == 0) ? 1 : 0);
  const hipStream_t st = as_stream(stream);
  if (epilogue == RDX_EPI_BIAS_GELU) return a_f32 ? lg::launch<true, false, RDX_EPI_BIAS_GELU>(g, st)
                                                  : lg::launch<false, false, RDX_EPI_BIAS_GELU>(g, st);
  if (epilogue == RDX_EPI_GELU_BWD) {
    if (a_f32) return c_f32 ? lg::launch<true, true, RDX_EPI_GELU_BWD>(g, st) : lg::launch<true, false, RDX_EPI_GELU_BWD>(g, st);
    return c_f32 ? lg::launch<false, true, RDX_EPI_GELU_BWD>(g, st) : lg::launch<false, false, RDX_EPI_GELU_BWD>(g, st);
  }
  if (a_f32) return c_f32 ? lg::launch<true, true, RDX_EPI_BIAS>(g, st) : lg::launch<true, false, RDX_EPI_BIAS>(g, st);
  return c_f32 ? lg::launch<false, true, RDX_EPI_BIAS>(g, st) : lg::launch<false, false, RDX_EPI_BIAS>(g, st);
}
