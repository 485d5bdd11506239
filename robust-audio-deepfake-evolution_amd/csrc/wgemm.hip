// bf16 MFMA GEMM for the WavLM encoder's dense projections on gfx950: the q/k/v, out_proj, FFN1 and FFN2
// GEMMs of HF WavLMEncoderLayerStableLayerNorm (as run by WavLMFrontend, src/models/DualStreamSEMamba.py:
// 292-439) and their input-gradient GEMMs, at M = B x 201 token rows (B = 8: M = 1608; B = 32: M = 6432).
//
//   C[M, N] = A[M, K] . B[N, K]^T     (both operands K-contiguous: x @ W^T; the input gradients use the frozen
//                                      weight's transposed copy, cached as [K_out][N_in])
// epilogues (the fp32 accumulator rounds where the unfused layer rounds, so the fusion changes no value):
//   RDX_EPI_BIAS       C = bf16(acc + bias)                          (bias optional)
//   RDX_EPI_BIAS_GELU  C = u = bf16(acc + bias), aux_out = bf16(gelu(u))   (FFN1 + GELU)
//   RDX_EPI_GELU_BWD   C = bf16(bf16(acc) * gelu'(aux))               (FFN2 input grad + GELU backward)
//
// Structure (MI355X_MICROARCH.md / cdna_hip_programming.md §5):
//   * workgroup = 4 waves (2 x 2) over a BM x BN output tile, K in steps of 64 through an NST-deep LDS ring;
//   * operands go HBM/L2 -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds, 1 KB = 8 rows x 128 B per wave
//     instruction), so no VGPR staging and no ds_write; the buffer's range clamps the row tail (rows >= M read
//     as zeros);
//   * one raw s_barrier per K step, preceded by a counted `s_waitcnt vmcnt` that retires only the stage about to
//     be read (the next NST - 2 stages stay in flight across the barrier; __syncthreads would drain them);
//   * LDS images are 128-B rows with the 16-byte chunk XOR-swizzled by (row >> 1) & 7 (conflict-free
//     ds_read_b128 for the 16x16x32 fragments); the DMA writes lane-linear, so the swizzle is applied to the
//     SOURCE address (the same involution on both sides);
//   * v_mfma_f32_16x16x32_bf16 computing C^T (the B tile is the MFMA's A operand): a lane ends with 4
//     consecutive output columns of one row (8-byte bf16 stores);
//   * tiles are numbered column-panel-major and dealt to XCDs in contiguous runs (blocks b and b + 8 share an
//     XCD; bijective remap), so one XCD's L2 holds its weight panels plus the shared activation rows.
#include "common.h"

namespace rdx {

typedef __attribute__((ext_vector_type(8))) __bf16 wbf16x8;
typedef __attribute__((ext_vector_type(4))) float wf32x4;
typedef __attribute__((ext_vector_type(4))) int wi32x4;

__device__ void wg_buffer_load_lds(wi32x4 rsrc, __attribute__((address_space(3))) uint32_t* lds, int size, int voffset,
                                   int soffset, int offset, int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");

__device__ __forceinline__ wi32x4 wg_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  wi32x4 r;
  r.x = (int)(uint32_t)a;
  r.y = (int)(uint32_t)(a >> 32);
  r.z = (int)bytes;
  r.w = 0x00020000;  // gfx9 raw buffer: dword-aligned, no swizzle, range-checked
  return r;
}

constexpr int WG_BK = 64;

__device__ __forceinline__ int wg_swz(int row, int ch) { return ch ^ ((row >> 1) & 7); }

__device__ __forceinline__ float wg_gelu(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float wg_gelu_grad(float x) {
  return 0.5f * (1.0f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}
__device__ __forceinline__ float wg_bf16(float x) { return __bfloat162float(__float2bfloat16(x)); }
__device__ __forceinline__ uint32_t wg_pack2(float a, float b) {
  __hip_bfloat16 x = __float2bfloat16(a), y = __float2bfloat16(b);
  return (uint32_t)(*reinterpret_cast<uint16_t*>(&x)) | ((uint32_t)(*reinterpret_cast<uint16_t*>(&y)) << 16);
}

struct WgArgs {
  const __hip_bfloat16* A;
  int64_t lda;
  const __hip_bfloat16* B;
  int64_t ldb;
  __hip_bfloat16* C;
  int64_t ldc;
  int M, N, K;
  const __hip_bfloat16* bias;  // [N] or null
  const __hip_bfloat16* aux;   // GELU_BWD: u [M, ldaux]
  int64_t ldaux;
  __hip_bfloat16* aux_out;     // BIAS_GELU: gelu(u) [M, ldao]
  int64_t ldao;
  int tiles_m, tiles_n;
};

// LDS-DMA of rows [r0, r0 + ROWS) x 64 k of a K-contiguous operand into a ROWS x 128-B swizzled image.
// `rs` covers the operand from row r0 on (its range ends at the last valid row). Each wave instruction moves
// 8 rows; the ROWS / 8 instructions are dealt round-robin to the NW waves.
template <int ROWS, int NW>
__device__ __forceinline__ void wg_stage(wi32x4 rs, int64_t ld_bytes, int k0_bytes, char* img, int wave, int lane) {
  constexpr int PER_WAVE = ROWS / 8 / NW;
  static_assert(ROWS % (8 * NW) == 0, "tile rows must be a multiple of 8 x waves");
  const int rr = lane >> 3, slot = lane & 7;
#pragma unroll
  for (int j = 0; j < PER_WAVE; ++j) {
    const int row = (j * NW + wave) * 8 + rr;
    const int ch = wg_swz(row, slot);
    const int voff = (int)(row * ld_bytes) + k0_bytes + ch * 16;
    wg_buffer_load_lds(rs, (__attribute__((address_space(3))) uint32_t*)(img + (j * NW + wave) * 1024), 16, voff, 0,
                       0, 0);
  }
}

// Retire all but this wave's N youngest LDS-DMA loads, then the workgroup barrier, in ONE asm statement with a
// memory clobber: no LDS access can be scheduled across it (the s_barrier builtin alone orders no memory).
template <int N>
__device__ __forceinline__ void wg_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

template <int BM, int BN, int WM, int WN, int NST, int OCC, int EPI, int ABL = 0>
__global__ __launch_bounds__(64 * WM * WN, OCC) void wgemm_kernel(WgArgs g) {
  constexpr int BK = WG_BK;
  constexpr int NW = WM * WN;
  constexpr int IMG_A = BM * 128, IMG_B = BN * 128, STAGE = IMG_A + IMG_B;
  constexpr int WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  constexpr int LPS = (BM + BN) / 8 / NW;  // LDS-DMA instructions per wave per stage
  static_assert(NST >= 2 && NST <= 4, "ring depth");
  extern __shared__ __attribute__((aligned(1024))) char lds[];

  // tile id: XCD-contiguous runs of the column-panel-major tile order
  const int nwg = g.tiles_m * g.tiles_n;
  int t;
  {
    const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int nt = t / g.tiles_m, mt = t - nt * g.tiles_m;
  const int m0 = mt * BM, n0 = nt * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int M = g.M, N = g.N, K = g.K;
  const int nk = K / BK;

  const int64_t lda_b = g.lda * 2, ldb_b = g.ldb * 2;
  const int rows_a = min(BM, M - m0), rows_b = min(BN, N - n0);
  const wi32x4 ra = wg_rsrc(g.A + (int64_t)m0 * g.lda, (uint32_t)((int64_t)(rows_a - 1) * lda_b + (int64_t)K * 2));
  const wi32x4 rb = wg_rsrc(g.B + (int64_t)n0 * g.ldb, (uint32_t)((int64_t)(rows_b - 1) * ldb_b + (int64_t)K * 2));

  auto issue = [&](int kt) {
    char* st = lds + (kt % NST) * STAGE;
    wg_stage<BM, NW>(ra, lda_b, kt * BK * 2, st, wave, lane);
    wg_stage<BN, NW>(rb, ldb_b, kt * BK * 2, st + IMG_A, wave, lane);
  };

  wf32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = wf32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: NST - 1 stages in flight
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) issue(s);

  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    // retire stage kt (this wave's share), keep the younger stages in flight, then make every wave's share
    // visible; the barrier also orders the previous step's fragment reads before the refill below
    const int younger = min(NST - 2, nk - 1 - kt);
    if (NST >= 4 && younger >= 2) wg_wait_barrier<2 * LPS>();
    else if (NST >= 3 && younger >= 1) wg_wait_barrier<LPS>();
    else wg_wait_barrier<0>();
    __builtin_amdgcn_sched_barrier(0);
    if (ABL != 1 && kt + NST - 1 < nk) issue(kt + NST - 1);   // ABL 1: timing probe, no refills
    const char* As = lds + (kt % NST) * STAGE;
    const char* Bs = As + IMG_A;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + fq;
      wbf16x8 af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * WTM + i * 16 + fr;
        af[i] = *reinterpret_cast<const wbf16x8*>(As + row * 128 + 16 * wg_swz(row, ch));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * WTN + j * 16 + fr;
        bf[j] = *reinterpret_cast<const wbf16x8*>(Bs + row * 128 + 16 * wg_swz(row, ch));
      }
      if (ABL == 2) {                // timing probe: fragments read, no MFMA
#pragma unroll
        for (int i = 0; i < FM; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
        for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(bf[j]));
      } else {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
      }
    }
  }

  // epilogue: acc[i][j][e] = C[m0 + wm*WTM + i*16 + fr][n0 + wn*WTN + j*16 + 4*fq + e]
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wm * WTM + i * 16 + fr;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * WTN + j * 16 + 4 * fq;
      if (n >= N) continue;  // N % 4 == 0
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (EPI != RDX_EPI_GELU_BWD && g.bias) {
        const uint2 bb = *reinterpret_cast<const uint2*>(g.bias + n);
        v[0] += __uint_as_float(bb.x << 16);
        v[1] += __uint_as_float(bb.x & 0xffff0000u);
        v[2] += __uint_as_float(bb.y << 16);
        v[3] += __uint_as_float(bb.y & 0xffff0000u);
      }
      __hip_bfloat16* cp = g.C + (int64_t)m * g.ldc + n;
      if (EPI == RDX_EPI_BIAS) {
        *reinterpret_cast<uint2*>(cp) = make_uint2(wg_pack2(v[0], v[1]), wg_pack2(v[2], v[3]));
      } else if (EPI == RDX_EPI_BIAS_GELU) {
        float u[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) u[e] = wg_bf16(v[e]);
        *reinterpret_cast<uint2*>(cp) = make_uint2(wg_pack2(u[0], u[1]), wg_pack2(u[2], u[3]));
        *reinterpret_cast<uint2*>(g.aux_out + (int64_t)m * g.ldao + n) =
            make_uint2(wg_pack2(wg_gelu(u[0]), wg_gelu(u[1])), wg_pack2(wg_gelu(u[2]), wg_gelu(u[3])));
      } else {  // RDX_EPI_GELU_BWD
        const uint2 uu = *reinterpret_cast<const uint2*>(g.aux + (int64_t)m * g.ldaux + n);
        const float u[4] = {__uint_as_float(uu.x << 16), __uint_as_float(uu.x & 0xffff0000u),
                            __uint_as_float(uu.y << 16), __uint_as_float(uu.y & 0xffff0000u)};
        float d[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) d[e] = wg_bf16(v[e]) * wg_gelu_grad(u[e]);
        *reinterpret_cast<uint2*>(cp) = make_uint2(wg_pack2(d[0], d[1]), wg_pack2(d[2], d[3]));
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, int NST, int OCC, int EPI, int ABL = 0>
static int wg_launch(WgArgs g, hipStream_t st) {
  g.tiles_m = (g.M + BM - 1) / BM;
  g.tiles_n = (g.N + BN - 1) / BN;
  constexpr int lds = NST * (BM + BN) * 128;
  static bool lds_ok = false;       // rings above the default 64 KB dynamic-LDS cap (160 KB per CU on gfx950)
  if (!lds_ok) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgemm_kernel<BM, BN, WM, WN, NST, OCC, EPI, ABL>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int)e;
    lds_ok = true;
  }
  hipLaunchKernelGGL((wgemm_kernel<BM, BN, WM, WN, NST, OCC, EPI, ABL>), dim3((unsigned)(g.tiles_m * g.tiles_n)),
                     dim3(64 * WM * WN), lds,
                     st, g);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

template <int EPI>
static int wg_dispatch(const WgArgs& g, int tile, hipStream_t st) {
  switch (tile) {
    case 0: return wg_launch<128, 128, 2, 2, 3, 1, EPI>(g, st);
    case 1: return wg_launch<64, 128, 2, 2, 3, 1, EPI>(g, st);
    case 5: return wg_launch<64, 64, 2, 2, 4, 1, EPI>(g, st);
    case 6: return wg_launch<128, 128, 2, 2, 2, 2, EPI>(g, st);
    case 11: return wg_launch<64, 128, 2, 2, 4, 1, EPI>(g, st);
    // 8 waves (two per SIMD)
    case 12: return wg_launch<128, 256, 2, 4, 3, 1, EPI>(g, st);
    case 13: return wg_launch<256, 128, 4, 2, 3, 1, EPI>(g, st);
    case 14: return wg_launch<128, 128, 2, 4, 4, 1, EPI>(g, st);
    case 15: return wg_launch<64, 256, 2, 4, 4, 1, EPI>(g, st);
    case 16: return wg_launch<128, 256, 2, 4, 2, 1, EPI>(g, st);
    case 17: return wg_launch<64, 128, 2, 4, 4, 1, EPI>(g, st);
    case 18: return wg_launch<256, 256, 2, 4, 2, 1, EPI>(g, st);
    // timing probes (ABL 1: no refills in the loop, ABL 2: no MFMA) of tiles 12 and 5: wrong results by design
    case 90: return wg_launch<128, 256, 2, 4, 3, 1, EPI, 1>(g, st);
    case 91: return wg_launch<128, 256, 2, 4, 3, 1, EPI, 2>(g, st);
    case 92: return wg_launch<64, 64, 2, 2, 4, 1, EPI, 1>(g, st);
    case 93: return wg_launch<64, 64, 2, 2, 4, 1, EPI, 2>(g, st);
    default: return RDX_EINVAL;
  }
}

}  // namespace rdx

using namespace rdx;

// tile: 0 = 128x128 (3-deep ring), 1 = 64x128, 2 = 128x256 (2-deep), 3 = 64x256, 4 = 128x64, 5 = 64x64;
// -1 = the built-in choice for the shape (rdx_wgemm_pick).
extern "C" int rdx_wgemm_pick(int M, int N, int K) {
  (void)K;
  const int64_t t128 = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  if (t128 >= 256) return 0;
  const int64_t t64 = (int64_t)((M + 63) / 64) * ((N + 127) / 128);
  if (t64 >= 160) return 1;
  return 5;
}

extern "C" int rdx_wgemm_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M,
                              int N, int K, const void* bias, int epilogue, const void* aux, int64_t ldaux,
                              void* aux_out, int64_t ldao, int tile, void* stream) {
  auto al = [](const void* p, int a) { return ((uintptr_t)p & (a - 1)) == 0; };
  RDX_REQUIRE(A && B && C && M > 0 && N > 0 && K > 0 && al(A, 16) && al(B, 16) && al(C, 8));
  RDX_REQUIRE(K % WG_BK == 0 && lda % 8 == 0 && ldb % 8 == 0 && lda >= K && ldb >= K && N % 4 == 0 && ldc >= N &&
              ldc % 4 == 0);
  // the per-tile buffer range is 32-bit
  RDX_REQUIRE((int64_t)256 * lda * 2 + (int64_t)K * 2 < 0x7fffffffLL && (int64_t)256 * ldb * 2 < 0x7fffffffLL);
  RDX_REQUIRE((int64_t)M * lda * 2 < 0x7fffffffLL && (int64_t)N * ldb * 2 < 0x7fffffffLL);
  RDX_REQUIRE(!bias || al(bias, 8));
  RDX_REQUIRE(epilogue == RDX_EPI_BIAS || epilogue == RDX_EPI_BIAS_GELU || epilogue == RDX_EPI_GELU_BWD);
  if (epilogue == RDX_EPI_BIAS_GELU) RDX_REQUIRE(aux_out && ldao >= N && ldao % 4 == 0 && al(aux_out, 8));
  if (epilogue == RDX_EPI_GELU_BWD) RDX_REQUIRE(aux && ldaux >= N && ldaux % 4 == 0 && al(aux, 8));
  if (tile < 0) tile = rdx_wgemm_pick(M, N, K);
  WgArgs g;
  g.A = (const __hip_bfloat16*)A;
  g.lda = lda;
  g.B = (const __hip_bfloat16*)B;
  g.ldb = ldb;
  g.C = (__hip_bfloat16*)C;
  g.ldc = ldc;
  g.M = M;
  g.N = N;
  g.K = K;
  g.bias = (const __hip_bfloat16*)bias;
  g.aux = (const __hip_bfloat16*)aux;
  g.ldaux = ldaux;
  g.aux_out = (__hip_bfloat16*)aux_out;
  g.ldao = ldao;
  g.tiles_m = g.tiles_n = 0;
  hipStream_t st = as_stream(stream);
  switch (epilogue) {
    case RDX_EPI_BIAS: return wg_dispatch<RDX_EPI_BIAS>(g, tile, st);
    case RDX_EPI_BIAS_GELU: return wg_dispatch<RDX_EPI_BIAS_GELU>(g, tile, st);
    default: return wg_dispatch<RDX_EPI_GELU_BWD>(g, tile, st);
  }
}
