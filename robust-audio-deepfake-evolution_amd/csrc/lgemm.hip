// Small-GEMM kernel of the detector head (the fusion, PN-BiMamba, pooling and classifier linears,
// src/models/DualStreamSEMamba.py:445-531,537-637,700-770): C[M, N] = A[M, K] W[N, K]^T with the linear's bias and the
// operations autocast puts around it fused into one launch.
//
// The head's shapes are narrow (N, K in {1, 2, 9, 41, 64, 144, 288, 576, 1024}) over 1 608 - 12 864 token rows: each
// GEMM is a few hundred MFLOP and its time is launch and load latency, not arithmetic (hipBLASLt took 7-9 us per
// call on them, and the casts, GELU, residual add and bias reduction around them were launches of their own). Here a
// 256-thread workgroup owns 32 token rows x 64 output features and stages K in LDS with every load of a chunk in
// flight at once: 16-bit operands with aligned rows by LDS-DMA (buffer_load ... lds, 36 VGPRs; chunks of up to 640,
// every head K but 1024 in one), others (fp32 A converted on load, strided views with any K such as the x_proj
// output's dt columns) through registers with zero-filled element loads (chunks of up to 320).
// The MFMAs are v_mfma_f32_16x16x32, wave w: features 16 w .. 16 w + 15 of the tile against both 16-row token tiles.
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
constexpr int T = 256;
// K is staged in LDS in chunks, kce = the chunk rounded up to 32 elements; LDS is sized by the launch. Register-path rows are kce + 8 elements: a pitch of an odd number of
// 16-byte bank groups, so the 16 rows one ds_read_b128 covers fall on distinct groups.
__host__ __device__ constexpr int kce_of(int KC, int K) { return K < KC ? ((K + 31) / 32) * 32 : KC; }

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
  int vec_a, vec_w;  // rows 16-byte aligned and K % 8 == 0 (16-byte loads)
  int vec_c;         // C rows 8-byte (16-bit) / 16-byte (fp32) aligned
};

// 8 consecutive elements of row `row` from column k as packed 16-bit values, zero past nrows / K. Buffer loads:
// an invalid element gets an offset past the buffer's range and reads as 0, so no load sits in a branch and every
// load of a chunk is in flight before the first wait.
constexpr uint32_t OOB = 0x80000000u;
template <bool F32>
__device__ __forceinline__ uint4 load8(__amdgpu_buffer_rsrc_t rs, int64_t ld, int row, int nrows, int k, int K,
                                       bool vec) {
  constexpr int ES = F32 ? 4 : 2;
  const bool rv = row < nrows;
  const uint32_t base = (uint32_t)(((int64_t)row * ld + k) * ES);
  if (vec) {   // rows 16-byte aligned and K % 8 == 0: whole 16-byte items
    const uint32_t off = (rv && k + 8 <= K) ? base : OOB;
    if constexpr (F32) {
      const uint4 a = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      const uint4 b = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0));
      const float v[8] = {__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z), __uint_as_float(a.w),
                          __uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z), __uint_as_float(b.w)};
      return make_uint4(hpack2(v[0], v[1]), hpack2(v[2], v[3]), hpack2(v[4], v[5]), hpack2(v[6], v[7]));
    } else {
      return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
  } else {     // element loads (unaligned rows: the x_proj output's dt columns, odd widths)
    if constexpr (F32) {
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        t[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (rv && k + j < K) ? base + 4 * j : OOB, 0, 0));
      return make_uint4(hpack2(t[0], t[1]), hpack2(t[2], t[3]), hpack2(t[4], t[5]), hpack2(t[6], t[7]));
    } else {
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b16(rs, (rv && k + 2 * j < K) ? base + 4 * j : OOB, 0, 0);
        const uint32_t hi =
            __builtin_amdgcn_raw_buffer_load_b16(rs, (rv && k + 2 * j + 1 < K) ? base + 4 * j + 2 : OOB, 0, 0);
        w[j] = lo | (hi << 16);
      }
      return make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

typedef __attribute__((ext_vector_type(4))) int lg_i32x4;
__device__ void lg_load_lds(lg_i32x4 rsrc, __attribute__((address_space(3))) uint32_t* lds, int size, int voffset,
                            int soffset, int offset, int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");
__device__ __forceinline__ lg_i32x4 lg_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  lg_i32x4 r;
  r.x = (int)(uint32_t)a;
  r.y = (int)(uint32_t)(a >> 32);
  r.z = (int)bytes;
  r.w = 0x00020000;  // raw buffer, range-checked
  return r;
}

// DMA: 16-bit operands with 16-byte aligned rows and K % 8 == 0 go global -> LDS by buffer_load ... lds (no
// registers, every load of a chunk in flight at once) into chunk-major images: the 16-byte item (k chunk j, row r)
// at 16 (j ROWS + r), so a wave instruction fills 64 consecutive items and the 16 rows one MFMA operand read covers
// are 256 contiguous bytes (conflict-free). Otherwise (fp32 A, unaligned rows, K % 8 != 0) through registers into
// row-major images of pitch kce + 8.
template <bool A_F32, bool C_F32, int EPI, bool DMA>
__global__ __launch_bounds__(T, 2) void lgemm_kernel(Args g) {
  constexpr int KC = DMA ? 640 : 320;
  constexpr int A_IT = DMA ? 1 : BM * (KC / 8) / T;   // 5
  constexpr int B_IT = DMA ? 1 : BN * (KC / 8) / T;   // 10
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int kce = kce_of(KC, g.K);
  const int KP = kce + 8;
  uint16_t* As = reinterpret_cast<uint16_t*>(lds);                      // register path: [BM][KP]
  uint16_t* Ws = As + BM * KP;                                          //                [BN][KP]
  char* Ab = lds;                                                       // DMA path: [kce / 8][BM] items
  char* Wb = lds + (kce / 8) * BM * 16;                                 //           [kce / 8][BN] items
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, l16 = lane & 15, lg = lane >> 4;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int nch = (g.K + KC - 1) / KC;
  const uint32_t abytes = (uint32_t)(((int64_t)(g.M - 1) * g.lda + g.K) * (A_F32 ? 4 : 2));
  const uint32_t wbytes = (uint32_t)(((int64_t)(g.N - 1) * g.ldw + g.K) * 2);
  rdx_f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if constexpr (DMA) {
    const lg_i32x4 ra = lg_rsrc(g.A, abytes), rw = lg_rsrc(g.W, wbytes);
    for (int c = 0; c < nch; ++c) {
      const int k0 = c * KC, kcp = min(KC, ((g.K - k0 + 31) / 32) * 32), nj = kcp / 8;
      if (c > 0) __syncthreads();   // the previous chunk's MFMA reads are done
      for (int q = wv; q < nj / 2; q += 4) {      // A: two k chunks of 32 rows per instruction
        const int i = 64 * q + lane, j = i / BM, r = i % BM;
        const bool ok = m0 + r < g.M && k0 + 8 * j < g.K;
        const int off = ok ? (int)((((int64_t)(m0 + r)) * g.lda + k0 + 8 * j) * 2) : (int)OOB;
        lg_load_lds(ra, (__attribute__((address_space(3))) uint32_t*)(Ab + 1024 * q), 16, off, 0, 0, 0);
      }
      for (int q = wv; q < nj; q += 4) {          // W: one k chunk of 64 rows per instruction
        const bool ok = n0 + lane < g.N && k0 + 8 * q < g.K;
        const int off = ok ? (int)((((int64_t)(n0 + lane)) * g.ldw + k0 + 8 * q) * 2) : (int)OOB;
        lg_load_lds(rw, (__attribute__((address_space(3))) uint32_t*)(Wb + 1024 * q), 16, off, 0, 0, 0);
      }
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      const char* wp = Wb + (16 * wv + l16) * 16 + lg * BN * 16;
      const char* ap0 = Ab + l16 * 16 + lg * BM * 16;
      const char* ap1 = ap0 + 16 * 16;
      for (int ks = 0; ks < kcp; ks += 32) {     // K step = 4 chunks
        const int j4 = ks / 8;
        const hx8 w = *reinterpret_cast<const hx8*>(wp + j4 * BN * 16);
        const hx8 a0 = *reinterpret_cast<const hx8*>(ap0 + j4 * BM * 16);
        const hx8 a1 = *reinterpret_cast<const hx8*>(ap1 + j4 * BM * 16);
        acc0 = mfma16x16x32(w, a0, acc0);
        acc1 = mfma16x16x32(w, a1, acc1);
      }
    }
  } else {
    uint4 ra[A_IT], rw[B_IT];
    // byte ranges of the operands (the last row ends at K): offsets past them read 0
    const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(g.A), 0, (int)abytes,
                                                                          0x00020000);
    const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(const_cast<hst*>(g.W), 0, (int)wbytes,
                                                                          0x00020000);
    // items enumerated chunk-major (item it: k chunk it / ROWS, row it % ROWS), so whether a wave's items lie inside
    // the chunk's kcp is the same for all its lanes: items past it issue no loads at all
    auto fetch = [&](int c) {
      const int k0 = c * KC, nj = min(KC, ((g.K - k0 + 31) / 32) * 32) / 8;
#pragma unroll
      for (int i = 0; i < A_IT; ++i) {
        const int it = tid + T * i, j = it / BM, row = it % BM;
        ra[i] = make_uint4(0u, 0u, 0u, 0u);
        if (j < nj) ra[i] = load8<A_F32>(rsa, g.lda, m0 + row, g.M, k0 + 8 * j, g.K, g.vec_a);
      }
#pragma unroll
      for (int i = 0; i < B_IT; ++i) {
        const int it = tid + T * i, j = it / BN, row = it % BN;
        rw[i] = make_uint4(0u, 0u, 0u, 0u);
        if (j < nj) rw[i] = load8<false>(rsw, g.ldw, n0 + row, g.N, k0 + 8 * j, g.K, g.vec_w);
      }
    };
    fetch(0);
    for (int c = 0; c < nch; ++c) {
      const int kcp = min(KC, ((g.K - c * KC + 31) / 32) * 32);
      if (c > 0) __syncthreads();   // the previous chunk's MFMA reads are done
#pragma unroll
      for (int i = 0; i < A_IT; ++i) {
        const int it = tid + T * i, j = it / BM, row = it % BM;
        if (8 * j < kcp) *reinterpret_cast<uint4*>(As + row * KP + 8 * j) = ra[i];
      }
#pragma unroll
      for (int i = 0; i < B_IT; ++i) {
        const int it = tid + T * i, j = it / BN, row = it % BN;
        if (8 * j < kcp) *reinterpret_cast<uint4*>(Ws + row * KP + 8 * j) = rw[i];
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

template <bool A_F32, bool C_F32, int EPI, bool DMA>
int launch_dma(const Args& g, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&lgemm_kernel<A_F32, C_F32, EPI, DMA>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             DMA ? (BM + BN) * 640 * 2 : (BM + BN) * (320 + 8) * 2);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  const int lds = DMA ? (BM + BN) * kce_of(640, g.K) * 2 : (BM + BN) * (kce_of(320, g.K) + 8) * 2;
  hipLaunchKernelGGL((lgemm_kernel<A_F32, C_F32, EPI, DMA>),
                     dim3((unsigned)((g.N + BN - 1) / BN), (unsigned)((g.M + BM - 1) / BM)), dim3(T), lds, st, g);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
template <bool A_F32, bool C_F32, int EPI>
int launch(const Args& g, hipStream_t st) {
  if constexpr (!A_F32)
    if (g.vec_a && g.vec_w) return launch_dma<false, C_F32, EPI, true>(g, st);
  return launch_dma<A_F32, C_F32, EPI, false>(g, st);
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
  // 32-bit buffer ranges and element offsets (the OOB sentinel 0x80000000 must lie outside every operand's range)
  RDX_REQUIRE(((int64_t)(M - 1) * lda + K) * (a_f32 ? 4 : 2) < 0x7fffffffLL &&
              ((int64_t)(N - 1) * ldw + K) * 2 < 0x7fffffffLL);
  lg::Args g{A, lda, (const hst*)W, ldw, C, ldc, (const hst*)bias, (const hst*)aux, ldaux, (hst*)aux_out, ldao,
             R, ldr, M, N, K, 0, 0, 0};
  g.vec_a = (((uintptr_t)A & 15) == 0 && (lda % (a_f32 ? 4 : 8)) == 0 && K % 8 == 0) ? 1 : 0;
  g.vec_w = (((uintptr_t)W & 15) == 0 && (ldw % 8) == 0 && K % 8 == 0) ? 1 : 0;
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
