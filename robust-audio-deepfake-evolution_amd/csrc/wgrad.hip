// Weight / bias gradients of the detector head's linears (SideLinear: the fusion projections, PN-BiMamba's
// in_proj / x_proj / dt_proj / out_proj and feed-forward, pooling and classifier of src/models/DualStreamSEMamba.py:
// 445-531, 537-637, 700-770), accumulated in fp32 into the flat gradient buffer:
//     dW[n][k] += sum_m dY[m][n] X[m][k]        db[n] += sum_m dY[m][n]          (bf16 dY, X; fp32 sums)
// These are long-K GEMMs with a tiny output ([576 x 144] over 1608 .. 12864 token rows): hipBLASLt runs them on
// 5-27 workgroups (the output tiles) for 18-80 us each. Here the token rows are split over the chip: a workgroup
// owns (64 x 64 output block, chunk of token rows), stages the chunk's dY and X column panels row-major in LDS
// and reduces over the rows with mfma_f32_32x32x16_bf16, both operands read down their columns by
// ds_read_b64_tr_b16 (csrc/sconv.hip's weight-gradient scheme); one fp32 partial per (chunk, block), then a second
// kernel adds the chunks in a fixed order into dW / db (deterministic, no atomics).
#include "common.h"

namespace rdx {

typedef __attribute__((ext_vector_type(16))) float wrf32x16;

constexpr int WR_T = 256;
constexpr int WR_MAXMC = 256;   // token rows per chunk (multiple of 16)

// [row][64] bf16 image: 8-row x 32-column subtiles of 512 B, 16-byte chunks XOR-swizzled by (row >> 2) & 3
__device__ __forceinline__ int wr_img(int row, int ch) {
  return 1024 * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}
// element j = IMG[16 s + 8 (j >> 2) + 4 h + (j & 3)][c0 + (lane & 31)]
__device__ __forceinline__ hx8 wr_read_tr(const char* img, int c0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int row = 16 * s + 4 * (g >> 1) + (i >> 2);
  const int col = c0 + 16 * (g & 1) + 4 * (i & 3);
  const int sub = 2 * (col & 7);
  const hx4v lo = ds_tr4((img + wr_img(row, col >> 3) + sub));
  const hx4v hi = ds_tr4((img + wr_img(row + 8, col >> 3) + sub));
  hx8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = lo[j];
    r[4 + j] = hi[j];
  }
  return r;
}

// rows [m0, m0 + mc) x columns [c0, c0 + 64) of a [M][ld] bf16 matrix into an image (zeros outside): every
// load of the thread is issued before the first LDS store, so their latencies overlap
constexpr int WR_ITEMS = WR_MAXMC * 8 / WR_T;   // 16-byte items per thread, at most
__device__ __forceinline__ void wr_gather(uint4 (&v)[WR_ITEMS], const hst* __restrict__ src, int64_t ld,
                                          int M, int C, int m0, int c0, int mc, bool vec) {
#pragma unroll
  for (int j = 0; j < WR_ITEMS; ++j) {
    const int i = threadIdx.x + WR_T * j;
    const int row = i >> 3, ch = i & 7;
    const int m = m0 + row, c = c0 + 8 * ch;
    v[j] = make_uint4(0u, 0u, 0u, 0u);
    if (i < mc * 8 && m < M) {
      const hst* p = src + (int64_t)m * ld + c;
      if (vec && c + 8 <= C) {
        v[j] = *reinterpret_cast<const uint4*>(p);
      } else {
        uint16_t e[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) e[t] = (c + t < C) ? hbits_of(p[t]) : (uint16_t)0;
        v[j] = make_uint4(e[0] | ((uint32_t)e[1] << 16), e[2] | ((uint32_t)e[3] << 16), e[4] | ((uint32_t)e[5] << 16),
                          e[6] | ((uint32_t)e[7] << 16));
      }
    }
  }
}
__device__ __forceinline__ void wr_put(char* img, const uint4 (&v)[WR_ITEMS], int mc) {
#pragma unroll
  for (int j = 0; j < WR_ITEMS; ++j) {
    const int i = threadIdx.x + WR_T * j;
    if (i < mc * 8) *reinterpret_cast<uint4*>(img + wr_img(i >> 3, i & 7)) = v[j];
  }
}

struct WgradArgs {
  const hst* dy;   // [M][ldy], columns 0..N-1
  const hst* x;    // [M][ldx], columns 0..K-1
  int64_t ldy, ldx;
  float* part;                // [S][N][K] partial dW per chunk
  float* partb;               // [S][N] partial db (or null)
  int M, N, K, mc, nbn, nbk;
  int vy, vx;                 // 16-byte aligned rows (ld % 8 == 0, 16-byte aligned base)
};

__global__ __launch_bounds__(WR_T) void wgrad_part_kernel(WgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* iy = lds;                        // dY chunk [mc][64]
  char* ix = lds + WR_MAXMC * 128;       // X chunk [mc][64]
  const int blk = blockIdx.x, s = blockIdx.y;
  const int bn = blk / a.nbk, bk = blk - bn * a.nbk;
  const int n0 = bn * 64, k0 = bk * 64, m0 = s * a.mc;
  const int mc = a.mc;
  {
    uint4 vy[WR_ITEMS], vx[WR_ITEMS];
    wr_gather(vy, a.dy, a.ldy, a.M, a.N, m0, n0, mc, a.vy);
    wr_gather(vx, a.x, a.ldx, a.M, a.K, m0, k0, mc, a.vx);
    wr_put(iy, vy, mc);
    wr_put(ix, vx, mc);
  }
  __syncthreads();
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int tn = wv >> 1, tk = wv & 1;
  wrf32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  for (int st = 0; st < mc / 16; ++st)
    acc = mfma32x32x16(wr_read_tr(iy, tn * 32, st, lane), wr_read_tr(ix, tk * 32, st, lane),
                                                  acc);
  // D[n][k]: k = tk * 32 + (lane & 31), n = tn * 32 + (i & 3) + 8 (i >> 2) + 4 hh
  const int r = lane & 31, hh = lane >> 5;
  const int k = k0 + tk * 32 + r;
  float* out = a.part + (int64_t)s * a.N * a.K;
  if (k < a.K) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int n = n0 + tn * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
      if (n < a.N) out[(int64_t)n * a.K + k] = acc[i];
    }
  }
  if (a.partb && bk == 0 && tid < 64 && n0 + tid < a.N) {   // db: column sums of the dY chunk, in row order
    const int ch = tid >> 3, sub = 2 * (tid & 7);
    float v = 0.f;
    for (int row = 0; row < mc; ++row)
      v += hlo((uint32_t)(*reinterpret_cast<const uint16_t*>(iy + wr_img(row, ch) + sub)));
    a.partb[(int64_t)s * a.N + n0 + tid] = v;
  }
}

// dW[n][k] += sum_s part[s][n][k], db[n] += sum_s partb[s][n]. A 256-thread block owns 64 consecutive outputs;
// wave w sums the chunks s = w, w + 4, ... in four independent chains (the loads of a thread overlap instead of
// running S dependent steps), and the four waves' sums are added in a fixed order: deterministic.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part,
                                                           const float* __restrict__ partb, int S, int N, int K,
                                                           float* __restrict__ dw, int64_t ldw,
                                                           float* __restrict__ db) {
  __shared__ float red[4][64];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t nk = (int64_t)N * K;
  const int64_t tot = nk + (db ? N : 0);
  const int64_t i = (int64_t)blockIdx.x * 64 + l;
  float v = 0.f;
  if (i < tot) {
    const float* src = i < nk ? part + i : partb + (i - nk);
    const int64_t st = i < nk ? nk : (int64_t)N;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int s = w;
    for (; s + 12 < S; s += 16) {
      a0 += src[(int64_t)s * st];
      a1 += src[(int64_t)(s + 4) * st];
      a2 += src[(int64_t)(s + 8) * st];
      a3 += src[(int64_t)(s + 12) * st];
    }
    for (; s < S; s += 4) a0 += src[(int64_t)s * st];
    v = (a0 + a1) + (a2 + a3);
  }
  red[w][l] = v;
  __syncthreads();
  if (w == 0 && i < tot) {
    const float t = ((red[0][l] + red[1][l]) + red[2][l]) + red[3][l];
    if (i < nk) {
      const int n = (int)(i / K), k = (int)(i - (int64_t)n * K);
      dw[(int64_t)n * ldw + k] += t;
    } else {
      db[i - nk] += t;
    }
  }
}

}  // namespace rdx

using namespace rdx;

// chunking for (M, N, K): about 2 workgroups per CU over the output blocks x chunks
extern "C" int rdx_wgrad_chunk(int M, int N, int K) {
  const int64_t blocks = (int64_t)((N + 63) / 64) * ((K + 63) / 64);
  int64_t S = (512 + blocks - 1) / blocks;
  const int64_t smax = (M + 15) / 16;
  if (S > smax) S = smax;
  if (S < 1) S = 1;
  int64_t mc = (M + S - 1) / S;
  mc = (mc + 15) / 16 * 16;
  if (mc > WR_MAXMC) mc = WR_MAXMC;
  return (int)mc;
}

extern "C" int64_t rdx_wgrad_ws_floats(int M, int N, int K) {
  const int mc = rdx_wgrad_chunk(M, N, K);
  const int64_t S = (M + mc - 1) / mc;
  return S * ((int64_t)N * K + N);
}

extern "C" int rdx_wgrad_acc(const void* dy, int64_t ldy, const void* x, int64_t ldx, int M, int N, int K, float* dw,
                             int64_t ldw, float* db, float* ws, int64_t ws_floats, void* stream) {
  RDX_REQUIRE(dy && x && dw && ws && M > 0 && N > 0 && K > 0 && ldy >= N && ldx >= K && ldw >= K);
  const int mc = rdx_wgrad_chunk(M, N, K);
  const int S = (M + mc - 1) / mc;
  RDX_REQUIRE(ws_floats >= rdx_wgrad_ws_floats(M, N, K) && S < 65536);
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_part_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 2 * WR_MAXMC * 128);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  WgradArgs a;
  a.dy = (const hst*)dy;
  a.x = (const hst*)x;
  a.ldy = ldy;
  a.ldx = ldx;
  a.part = ws;
  a.partb = db ? ws + (int64_t)S * N * K : nullptr;
  a.M = M;
  a.N = N;
  a.K = K;
  a.mc = mc;
  a.nbn = (N + 63) / 64;
  a.nbk = (K + 63) / 64;
  a.vy = (ldy % 8 == 0) && (((uintptr_t)dy & 15) == 0);
  a.vx = (ldx % 8 == 0) && (((uintptr_t)x & 15) == 0);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(wgrad_part_kernel, dim3((unsigned)(a.nbn * a.nbk), (unsigned)S), dim3(WR_T), 2 * WR_MAXMC * 128,
                     st, a);
  RDX_LAUNCH_CHECK();
  const int64_t tot = (int64_t)N * K + (db ? N : 0);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((tot + 63) / 64)), dim3(256), 0, st, ws, a.partb, S, N, K,
                     dw, ldw, db);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
