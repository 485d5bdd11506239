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

// ---- Batched form: every weight gradient of one backward pass in two launches (rdx_wgrad_acc_many). Launched one
// per linear, the pair above costs ~12 us per layer in a captured graph, nearly all of it launch boundary; 31 of
// them per detector-head backward. One workgroup owns (problem, 64 x 64 output block, run of R sub-chunks of 128
// token rows): the next sub-chunk's dY / X panels are loaded into registers while the current one's MFMAs run
// (accumulating in registers), so a run costs about one load latency per sub-chunk and leaves ONE fp32 partial.
constexpr int WGM_MC = 128;                        // token rows per sub-chunk (32 KB of LDS: several groups per CU)
constexpr int WGM_ITEMS = WGM_MC * 8 / WR_T;       // 16-byte items per thread per operand
constexpr int WGM_MAXP = 32;                       // problems per launch (the table is a kernel argument)
static_assert(WGM_MC == 4 * (WR_T / 8), "db: 32 row groups of 4 rows x 8 column chunks per sub-chunk");
struct WgmProb {
  const hst* dy;
  const hst* x;
  float* dw;
  float* db;
  float* part;    // [S][N][K]
  float* partb;   // [S][N] (db only)
  int ldy, ldx, ldw, M, N, K, S, R, nbn, nbk, vec, blk0, out0;
};
struct WgmTable {
  WgmProb p[WGM_MAXP];
  int n;
};

__device__ __forceinline__ void wgm_gather(uint4 (&v)[WGM_ITEMS], const hst* __restrict__ src, int64_t ld, int M,
                                           int C, int m0, int c0, bool vec) {
#pragma unroll
  for (int j = 0; j < WGM_ITEMS; ++j) {
    const int i = threadIdx.x + WR_T * j;
    const int row = i >> 3, ch = i & 7;
    const int m = m0 + row, c = c0 + 8 * ch;
    v[j] = make_uint4(0u, 0u, 0u, 0u);
    if (m < M) {
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
__device__ __forceinline__ void wgm_put(char* img, const uint4 (&v)[WGM_ITEMS]) {
#pragma unroll
  for (int j = 0; j < WGM_ITEMS; ++j) {
    const int i = threadIdx.x + WR_T * j;
    *reinterpret_cast<uint4*>(img + wr_img(i >> 3, i & 7)) = v[j];
  }
}
// the problem owning block b of a grid dealt as [problem 0's blocks | problem 1's | ...] (first[k] = its first block)
// (a fixed-count loop: the table's scalar loads issue together instead of one load latency per problem)
__device__ __forceinline__ int wgm_find(const WgmTable& t, int b, bool out) {
  int p = 0;
#pragma unroll
  for (int k = 1; k < WGM_MAXP; ++k) p = (k < t.n && b >= (out ? t.p[k].out0 : t.p[k].blk0)) ? k : p;
  return __builtin_amdgcn_readfirstlane(p);
}

__global__ __launch_bounds__(WR_T, 4) void wgrad_part_many_kernel(WgmTable t) {
  __shared__ __attribute__((aligned(16))) char iy[WGM_MC * 128], ix[WGM_MC * 128];
  const WgmProb& q = t.p[wgm_find(t, blockIdx.x, false)];
  const int nb = q.nbn * q.nbk, local = blockIdx.x - q.blk0;
  const int s = local / nb, blk = local - s * nb;
  const int bn = blk / q.nbk, bk = blk - bn * q.nbk;
  const int n0 = bn * 64, k0 = bk * 64;
  const int r0 = s * q.R * WGM_MC;
  const int nsub = min(q.R, (q.M - r0 + WGM_MC - 1) / WGM_MC);
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int tn = wv >> 1, tk = wv & 1;
  const bool bsum = q.partb && bk == 0;     // block-uniform: the whole group sums dY's columns
  wrf32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // columns 8 (tid & 7) .. + 7 over rows 4 (tid >> 3) .. + 3
  uint4 vy[WGM_ITEMS], vx[WGM_ITEMS];
  wgm_gather(vy, q.dy, q.ldy, q.M, q.N, r0, n0, q.vec & 1);
  wgm_gather(vx, q.x, q.ldx, q.M, q.K, r0, k0, q.vec & 2);
  for (int j = 0; j < nsub; ++j) {
    __syncthreads();                          // the previous sub-chunk's LDS reads are done
    wgm_put(iy, vy);
    wgm_put(ix, vx);
    if (j + 1 < nsub) {                       // the next sub-chunk's loads run under this one's MFMAs
      const int m1 = r0 + (j + 1) * WGM_MC;
      wgm_gather(vy, q.dy, q.ldy, q.M, q.N, m1, n0, q.vec & 1);
      wgm_gather(vx, q.x, q.ldx, q.M, q.K, m1, k0, q.vec & 2);
    }
    __syncthreads();
#pragma unroll
    for (int st = 0; st < WGM_MC / 16; ++st)
      acc = mfma32x32x16(wr_read_tr(iy, tn * 32, st, lane), wr_read_tr(ix, tk * 32, st, lane), acc);
    if (bsum) {     // db: this thread's 8 columns over its 4 rows of the sub-chunk (rows past M are zeros)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const uint4 v = *reinterpret_cast<const uint4*>(iy + wr_img(4 * (tid >> 3) + rr, tid & 7));
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bv[2 * e] += hlo(w[e]);
          bv[2 * e + 1] += hhi(w[e]);
        }
      }
    }
  }
  if (bsum) {       // the 32 row groups' sums of each column, added in row-group order
    __syncthreads();
    float* red = reinterpret_cast<float*>(ix);            // [32 row groups][64 columns]
#pragma unroll
    for (int e = 0; e < 8; ++e) red[(tid >> 3) * 64 + 8 * (tid & 7) + e] = bv[e];
    __syncthreads();
    if (tid < 64) {
      float t = 0.f;
      for (int g = 0; g < 32; ++g) t += red[g * 64 + tid];
      bv[0] = t;
    }
  }
  const int r = lane & 31, hh = lane >> 5;
  const int k = k0 + tk * 32 + r;
  float* out = q.part + (int64_t)s * q.N * q.K;
  if (k < q.K) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int n = n0 + tn * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
      if (n < q.N) out[(int64_t)n * q.K + k] = acc[i];
    }
  }
  if (bsum && tid < 64 && n0 + tid < q.N) q.partb[(int64_t)s * q.N + n0 + tid] = bv[0];
}

// dW += sum_s part[s], db += sum_s partb[s] for every problem: one output per thread, the runs added in run order
// (deterministic), 256 outputs per block
constexpr int WGM_RED = 256;
__global__ __launch_bounds__(WGM_RED) void wgrad_reduce_many_kernel(WgmTable t) {
  const WgmProb& q = t.p[wgm_find(t, blockIdx.x, true)];
  const int64_t nk = (int64_t)q.N * q.K;
  const int64_t tot = nk + (q.db ? q.N : 0);
  const int64_t i = (int64_t)(blockIdx.x - q.out0) * WGM_RED + threadIdx.x;
  if (i >= tot) return;
  const float* src = i < nk ? q.part + i : q.partb + (i - nk);
  const int64_t st = i < nk ? nk : (int64_t)q.N;
  float v[8];
  float acc = 0.f;
  for (int s0 = 0; s0 < q.S; s0 += 8) {      // 8 runs' loads in flight, then added in order
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = s0 + k < q.S ? src[(int64_t)(s0 + k) * st] : 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += v[k];
  }
  if (i < nk) {
    const int n = (int)(i / q.K), k = (int)(i - (int64_t)n * q.K);
    q.dw[(int64_t)n * q.ldw + k] += acc;
  } else {
    q.db[i - nk] += acc;
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

// Plan of a batched launch: every problem runs S runs of R sub-chunks (S, R from its token count and the group's
// total output blocks: about 4 workgroups per CU, its occupancy, over the whole group; at least 2 runs per block).
static void wgm_plan(int n, const int* M, const int* N, const int* K, int* S, int* R) {
  int64_t outb = 0;
  for (int k = 0; k < n; ++k) outb += (int64_t)((N[k] + 63) / 64) * ((K[k] + 63) / 64);
  int64_t runs = (4 * 256 + outb - 1) / (outb > 0 ? outb : 1);
  if (runs < 2) runs = 2;
  for (int k = 0; k < n; ++k) {
    const int nsub = (M[k] + WGM_MC - 1) / WGM_MC;
    R[k] = (int)((nsub + runs - 1) / runs);
    S[k] = (nsub + R[k] - 1) / R[k];
  }
}

extern "C" int64_t rdx_wgrad_many_ws_floats(int n, const int* M, const int* N, const int* K, const int* has_db) {
  if (n <= 0 || n > WGM_MAXP || !M || !N || !K || !has_db) return 0;
  int S[WGM_MAXP], R[WGM_MAXP];
  wgm_plan(n, M, N, K, S, R);
  int64_t f = 0;
  for (int k = 0; k < n; ++k) f += (int64_t)S[k] * ((int64_t)N[k] * K[k] + (has_db[k] ? N[k] : 0));
  return f;
}

extern "C" int rdx_wgrad_acc_many(int n, const void* const* dy, const int64_t* ldy, const void* const* x,
                                  const int64_t* ldx, const int* M, const int* N, const int* K, float* const* dw,
                                  const int64_t* ldw, float* const* db, float* ws, int64_t ws_floats, void* stream) {
  RDX_REQUIRE(n >= 0 && n <= WGM_MAXP);
  if (n == 0) return RDX_OK;
  RDX_REQUIRE(dy && ldy && x && ldx && M && N && K && dw && ldw && db && ws);
  int has_db[WGM_MAXP];
  for (int k = 0; k < n; ++k) {
    RDX_REQUIRE(dy[k] && x[k] && dw[k] && M[k] > 0 && N[k] > 0 && K[k] > 0 && ldy[k] >= N[k] && ldx[k] >= K[k] &&
                ldw[k] >= K[k] && ldy[k] < (1ll << 31) && ldx[k] < (1ll << 31) && ldw[k] < (1ll << 31));
    for (int j = 0; j < k; ++j) RDX_REQUIRE(dw[j] != dw[k] && (!db[k] || db[j] != db[k]));   // one add per output
    has_db[k] = db[k] != nullptr;
  }
  RDX_REQUIRE(ws_floats >= rdx_wgrad_many_ws_floats(n, M, N, K, has_db));
  int S[WGM_MAXP], R[WGM_MAXP];
  wgm_plan(n, M, N, K, S, R);
  WgmTable t{};
  t.n = n;
  int64_t blk = 0, outb = 0, off = 0;
  for (int k = 0; k < n; ++k) {
    WgmProb& q = t.p[k];
    q.dy = (const hst*)dy[k];
    q.x = (const hst*)x[k];
    q.dw = dw[k];
    q.db = db[k];
    q.part = ws + off;
    off += (int64_t)S[k] * N[k] * K[k];
    q.partb = db[k] ? ws + off : nullptr;
    off += db[k] ? (int64_t)S[k] * N[k] : 0;
    q.ldy = (int)ldy[k];
    q.ldx = (int)ldx[k];
    q.ldw = (int)ldw[k];
    q.M = M[k];
    q.N = N[k];
    q.K = K[k];
    q.S = S[k];
    q.R = R[k];
    q.nbn = (N[k] + 63) / 64;
    q.nbk = (K[k] + 63) / 64;
    q.vec = ((ldy[k] % 8 == 0) && (((uintptr_t)dy[k] & 15) == 0) ? 1 : 0) |
            ((ldx[k] % 8 == 0) && (((uintptr_t)x[k] & 15) == 0) ? 2 : 0);
    q.blk0 = (int)blk;
    q.out0 = (int)outb;
    blk += (int64_t)S[k] * q.nbn * q.nbk;
    outb += ((int64_t)N[k] * K[k] + (db[k] ? N[k] : 0) + WGM_RED - 1) / WGM_RED;
  }
  RDX_REQUIRE(blk < (1ll << 31) && outb < (1ll << 31));
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(wgrad_part_many_kernel, dim3((unsigned)blk), dim3(WR_T), 0, st, t);
  RDX_LAUNCH_CHECK();
  hipLaunchKernelGGL(wgrad_reduce_many_kernel, dim3((unsigned)outb), dim3(WGM_RED), 0, st, t);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
