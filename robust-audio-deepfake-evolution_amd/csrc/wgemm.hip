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
__device__ __forceinline__ uint32_t wg_pack2(float a, float b) {
  hst x = f2h(a), y = f2h(b);
  return (uint32_t)(*reinterpret_cast<uint16_t*>(&x)) | ((uint32_t)(*reinterpret_cast<uint16_t*>(&y)) << 16);
}

struct WgArgs {
  const hst* A;
  int64_t lda;
  const hst* B;
  int64_t ldb;
  hst* C;
  int64_t ldc;
  int M, N, K;
  const hst* bias;  // [N] or null
  const hst* aux;   // GELU_BWD: u [M, ldaux]
  int64_t ldaux;
  hst* aux_out;     // BIAS_GELU: gelu(u) [M, ldao]
  int64_t ldao;
  int tiles_m, tiles_n;
  int splits;                  // split-K factor (1: none); split s covers k-steps [s*nk/S, (s+1)*nk/S)
  float* ws;                   // split-K partial slabs: [tile][split][FM*FN][threads][4] fp32
  int* counters;               // split-K arrival tickets, one per tile, zero between launches
  int wide;                    // C / aux / aux_out rows 16-byte aligned (ld % 8 == 0): 16-byte row-phase accesses
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

template <int BM, int BN, int WM, int WN, int NST, int OCC, int EPI, int ABL = 0, int SEPI = 1>
__global__ __launch_bounds__(64 * WM * WN, OCC) void wgemm_kernel(WgArgs g) {
  constexpr int BK = WG_BK;
  constexpr int NW = WM * WN;
  constexpr int IMG_A = BM * 128, IMG_B = BN * 128, STAGE = IMG_A + IMG_B;
  constexpr int WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  constexpr int LPS = (BM + BN) / 8 / NW;  // LDS-DMA instructions per wave per stage
  static_assert(NST >= 2 && NST <= 4, "ring depth");
  extern __shared__ __attribute__((aligned(1024))) char lds[];

  // work id: XCD-contiguous runs of the column-panel-major (tile, split) order, so the splits of one tile share
  // an XCD (its L2 holds their operand panels and the partial slabs the last arriver reads)
  const int S = g.splits;
  const int nwg = g.tiles_m * g.tiles_n * S;
  int t;
  {
    const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int tile = t / S, split = t - tile * S;
  const int nt = tile / g.tiles_m, mt = tile - nt * g.tiles_m;
  const int m0 = mt * BM, n0 = nt * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int M = g.M, N = g.N, K = g.K;
  const int nk_all = K / BK;
  const int kb = split * nk_all / S, nk = (split + 1) * nk_all / S - kb;

  const int64_t lda_b = g.lda * 2, ldb_b = g.ldb * 2;
  const int rows_a = min(BM, M - m0), rows_b = min(BN, N - n0);
  const wi32x4 ra = wg_rsrc(g.A + (int64_t)m0 * g.lda, (uint32_t)((int64_t)(rows_a - 1) * lda_b + (int64_t)K * 2));
  const wi32x4 rb = wg_rsrc(g.B + (int64_t)n0 * g.ldb, (uint32_t)((int64_t)(rows_b - 1) * ldb_b + (int64_t)K * 2));

  auto issue = [&](int kt) {   // kt: k-step within this split's range
    char* st = lds + (kt % NST) * STAGE;
    wg_stage<BM, NW>(ra, lda_b, (kb + kt) * BK * 2, st, wave, lane);
    wg_stage<BN, NW>(rb, ldb_b, (kb + kt) * BK * 2, st + IMG_A, wave, lane);
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
      hx8 af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * WTM + i * 16 + fr;
        af[i] = *reinterpret_cast<const hx8*>(As + row * 128 + 16 * wg_swz(row, ch));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * WTN + j * 16 + fr;
        bf[j] = *reinterpret_cast<const hx8*>(Bs + row * 128 + 16 * wg_swz(row, ch));
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
            acc[i][j] = mfma16x16x32(bf[j], af[i], acc[i][j]);
      }
    }
  }

  // split-K keeps a second accumulator set for the ordered sum: only tiles of <= 64 accumulators per lane
  constexpr bool kSplitK = FM * FN * 4 <= 64;
  if (kSplitK && S > 1) {
    // Split-K: every split publishes its fp32 partial in fragment order (lane-contiguous 16-byte stores, the
    // reducer reads the same slots with the same thread mapping), then takes an arrival ticket; the last
    // arriver sums the S partials in split order (deterministic whoever arrives last) and runs the epilogue.
    // Publication (cdna_hip_programming.md Guideline 16 / "Projection GEMM at M = 256" item 2): plain stores,
    // every wave's vmcnt(0), barrier, one agent-scope release, vmcnt(0), relaxed agent ticket; the last arriver:
    // agent-scope acquire, vmcnt(0), barrier, plain loads. The ticket resets to 0 for the next launch.
    constexpr int NT = 64 * NW;
    float* slab = g.ws + (int64_t)tile * S * (FM * FN * NT * 4);
    {
      float* mine = slab + (int64_t)split * (FM * FN * NT * 4);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) *reinterpret_cast<wf32x4*>(mine + ((i * FN + j) * NT + tid) * 4) = acc[i][j];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(lds);
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int ticket = __hip_atomic_fetch_add(g.counters + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = ticket;
      if (ticket == S - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        g.counters[tile] = 0;
      }
    }
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(flag[0]) != S - 1) return;
    // the running sum in split order (the runtime loop stays outside the unrolled fragment loops: an acc index
    // under a runtime loop would put the accumulators in scratch)
    wf32x4 tot[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        tot[i][j] = split == 0 ? acc[i][j] : *reinterpret_cast<const wf32x4*>(slab + ((i * FN + j) * NT + tid) * 4);
    for (int s2 = 1; s2 < S; ++s2) {
      const float* ps = slab + (int64_t)s2 * (FM * FN * NT * 4);
      const bool own = s2 == split;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          tot[i][j] += own ? acc[i][j] : *reinterpret_cast<const wf32x4*>(ps + ((i * FN + j) * NT + tid) * 4);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = tot[i][j];
  }

  // epilogue: acc[i][j][e] = C[m0 + wm*WTM + i*16 + fr][n0 + wn*WTN + j*16 + 4*fq + e]
  if constexpr (SEPI) {
    // Staged through LDS: the fragment layout gives a lane 8 bytes in each of 16 rows per store instruction
    // (32-byte row pieces, store-issue-bound: MI355X_MICROARCH.md 'attention epilogue store tail'), so the
    // tile's bf16 values go to an LDS image first and leave it as whole rows, 16 bytes per lane. The row pitch
    // is padded by 16 bytes, so the 16 rows of one 16-lane ds_write_b64 group fall on distinct banks.
    // GELU_BWD and BIAS_GELU apply their element-wise part in the row phase, where aux is read coalesced.
    constexpr int PITCH = BN * 2 + 16;
    char* img = lds;
    wg_wait_barrier<0>();           // every wave's last fragment reads are done before the image overwrites the ring
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int r = wm * WTM + i * 16 + fr;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = wn * WTN + j * 16 + 4 * fq;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if (EPI != RDX_EPI_GELU_BWD && g.bias && n0 + c < N) {
          const uint2 bb = *reinterpret_cast<const uint2*>(g.bias + n0 + c);
          v[0] += hlo(bb.x);
          v[1] += hhi(bb.x);
          v[2] += hlo(bb.y);
          v[3] += hhi(bb.y);
        }
        *reinterpret_cast<uint2*>(img + r * PITCH + c * 2) = make_uint2(wg_pack2(v[0], v[1]), wg_pack2(v[2], v[3]));
      }
    }
    __syncthreads();
    constexpr int CPR = BN / 8;     // 16-byte chunks per tile row
#pragma unroll 4
    for (int idx = tid; idx < BM * CPR; idx += 64 * NW) {
      const int r = idx / CPR, c = (idx - r * CPR) * 8;
      const int m = m0 + r, n = n0 + c;
      if (m >= M || n >= N) continue;
      const bool full = n + 8 <= N;   // else 4 columns (N % 4 == 0)
      const bool wide = full && g.wide;
      // 8 columns as one 16-byte access, or two 8-byte halves (the second only when full)
      auto ld8 = [&](const hst* src) -> uint4 {
        if (wide) return *reinterpret_cast<const uint4*>(src);
        const uint2 lo = *reinterpret_cast<const uint2*>(src);
        const uint2 hi = full ? *reinterpret_cast<const uint2*>(src + 4) : make_uint2(0u, 0u);
        return make_uint4(lo.x, lo.y, hi.x, hi.y);
      };
      auto st8 = [&](hst* dst, uint4 v) {
        if (wide) { *reinterpret_cast<uint4*>(dst) = v; return; }
        *reinterpret_cast<uint2*>(dst) = make_uint2(v.x, v.y);
        if (full) *reinterpret_cast<uint2*>(dst + 4) = make_uint2(v.z, v.w);
      };
      uint4 q = *reinterpret_cast<const uint4*>(img + r * PITCH + c * 2);
      if (EPI == RDX_EPI_GELU_BWD) {
        const uint4 uu = ld8(g.aux + (int64_t)m * g.ldaux + n);
        const uint32_t qw[4] = {q.x, q.y, q.z, q.w}, uw[4] = {uu.x, uu.y, uu.z, uu.w};
        uint32_t o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a0 = hlo(qw[e]), a1 = hhi(qw[e]);
          const float u0 = hlo(uw[e]), u1 = hhi(uw[e]);
          o[e] = wg_pack2(a0 * wg_gelu_grad(u0), a1 * wg_gelu_grad(u1));
        }
        q = make_uint4(o[0], o[1], o[2], o[3]);
      }
      st8(g.C + (int64_t)m * g.ldc + n, q);
      if (EPI == RDX_EPI_BIAS_GELU) {
        const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
        uint32_t o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          o[e] = wg_pack2(wg_gelu(hlo(qw[e])), wg_gelu(hhi(qw[e])));
        st8(g.aux_out + (int64_t)m * g.ldao + n, make_uint4(o[0], o[1], o[2], o[3]));
      }
    }
    return;
  }
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
        v[0] += hlo(bb.x);
        v[1] += hhi(bb.x);
        v[2] += hlo(bb.y);
        v[3] += hhi(bb.y);
      }
      hst* cp = g.C + (int64_t)m * g.ldc + n;
      if (EPI == RDX_EPI_BIAS) {
        *reinterpret_cast<uint2*>(cp) = make_uint2(wg_pack2(v[0], v[1]), wg_pack2(v[2], v[3]));
      } else if (EPI == RDX_EPI_BIAS_GELU) {
        float u[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) u[e] = hround(v[e]);
        *reinterpret_cast<uint2*>(cp) = make_uint2(wg_pack2(u[0], u[1]), wg_pack2(u[2], u[3]));
        *reinterpret_cast<uint2*>(g.aux_out + (int64_t)m * g.ldao + n) =
            make_uint2(wg_pack2(wg_gelu(u[0]), wg_gelu(u[1])), wg_pack2(wg_gelu(u[2]), wg_gelu(u[3])));
      } else {  // RDX_EPI_GELU_BWD
        const uint2 uu = *reinterpret_cast<const uint2*>(g.aux + (int64_t)m * g.ldaux + n);
        const float u[4] = {hlo(uu.x), hhi(uu.x),
                            hlo(uu.y), hhi(uu.y)};
        float d[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) d[e] = hround(v[e]) * wg_gelu_grad(u[e]);
        *reinterpret_cast<uint2*>(cp) = make_uint2(wg_pack2(d[0], d[1]), wg_pack2(d[2], d[3]));
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, int NST, int OCC, int EPI, int ABL = 0, int SEPI = 1>
static int wg_launch(WgArgs g, hipStream_t st) {
  g.tiles_m = (g.M + BM - 1) / BM;
  g.tiles_n = (g.N + BN - 1) / BN;
  constexpr int ring = NST * (BM + BN) * 128, image = SEPI ? BM * (BN * 2 + 16) : 0;
  constexpr int lds = ring > image ? ring : image;
  static_assert(lds <= 160 * 1024, "LDS");
  static bool lds_ok = false;       // rings above the default 64 KB dynamic-LDS cap (160 KB per CU on gfx950)
  if (!lds_ok) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgemm_kernel<BM, BN, WM, WN, NST, OCC, EPI, ABL, SEPI>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int)e;
    lds_ok = true;
  }
  hipLaunchKernelGGL((wgemm_kernel<BM, BN, WM, WN, NST, OCC, EPI, ABL, SEPI>),
                     dim3((unsigned)(g.tiles_m * g.tiles_n * g.splits)),
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
    case 20: return wg_launch<128, 192, 2, 4, 3, 1, EPI>(g, st);
    case 21: return wg_launch<128, 192, 2, 4, 2, 1, EPI>(g, st);
    // timing probes (ABL 1: no refills in the loop, ABL 2: no MFMA) of tiles 12 and 5: wrong results by design
    case 90: return wg_launch<128, 256, 2, 4, 3, 1, EPI, 1>(g, st);
    case 91: return wg_launch<128, 256, 2, 4, 3, 1, EPI, 2>(g, st);
    case 92: return wg_launch<64, 64, 2, 2, 4, 1, EPI, 1>(g, st);
    case 93: return wg_launch<64, 64, 2, 2, 4, 1, EPI, 2>(g, st);
    // the same tiles with the unstaged (per-lane fragment) epilogue, for A/B
    case 45: return wg_launch<64, 64, 2, 2, 4, 1, EPI, 0, 0>(g, st);
    case 46: return wg_launch<128, 128, 2, 2, 2, 2, EPI, 0, 0>(g, st);
    case 52: return wg_launch<128, 256, 2, 4, 3, 1, EPI, 0, 0>(g, st);
    case 56: return wg_launch<128, 256, 2, 4, 2, 1, EPI, 0, 0>(g, st);
    default: return RDX_EINVAL;
  }
}

// Output tile of each tile code (the split-K workspace is sized from it).
static bool wg_geometry(int tile, int* bm, int* bn, int* nthreads) {
  switch (tile) {
    case 0: case 6: case 46: *bm = 128; *bn = 128; *nthreads = 256; return true;
    case 1: case 11: *bm = 64; *bn = 128; *nthreads = 256; return true;
    case 5: case 45: case 92: case 93: *bm = 64; *bn = 64; *nthreads = 256; return true;
    case 12: case 16: case 52: case 56: case 90: case 91: *bm = 128; *bn = 256; *nthreads = 512; return true;
    case 13: *bm = 256; *bn = 128; *nthreads = 512; return true;
    case 14: *bm = 128; *bn = 128; *nthreads = 512; return true;
    case 15: *bm = 64; *bn = 256; *nthreads = 512; return true;
    case 17: *bm = 64; *bn = 128; *nthreads = 512; return true;
    case 18: *bm = 256; *bn = 256; *nthreads = 512; return true;
    case 20: case 21: *bm = 128; *bn = 192; *nthreads = 512; return true;
    default: return false;
  }
}

}  // namespace rdx

using namespace rdx;

// -1 = the built-in choice for the shape (rdx_wgemm_pick).
extern "C" int rdx_wgemm_pick(int M, int N, int K) {
  (void)K;
  const int64_t t128 = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  if (t128 >= 256) return 0;
  const int64_t t64 = (int64_t)((M + 63) / 64) * ((N + 127) / 128);
  if (t64 >= 160) return 1;
  return 5;
}

extern "C" int64_t rdx_wgemm_ws_bytes(int M, int N, int tile, int splits) {
  int bm, bn, nt;
  if (splits <= 1) return 0;
  if (!wg_geometry(tile, &bm, &bn, &nt)) return -1;
  const int64_t tiles = (int64_t)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  return tiles * splits * (int64_t)bm * bn * 4;
}

extern "C" int64_t rdx_wgemm_counters(int M, int N, int tile) {
  int bm, bn, nt;
  if (!wg_geometry(tile, &bm, &bn, &nt)) return -1;
  return (int64_t)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
}

extern "C" int rdx_wgemm_bf16_ex(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M,
                                 int N, int K, const void* bias, int epilogue, const void* aux, int64_t ldaux,
                                 void* aux_out, int64_t ldao, int tile, int splits, void* ws, int64_t ws_bytes,
                                 int* counters, int64_t n_counters, void* stream) {
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
  RDX_REQUIRE(splits >= 1 && splits <= K / WG_BK && splits <= 64);
  if (splits > 1) {
    RDX_REQUIRE(tile < 90);   // the timing probes never split
    int bm, bn, nt;
    RDX_REQUIRE(wg_geometry(tile, &bm, &bn, &nt) && bm * bn / nt <= 64);   // kSplitK in the kernel
    const int64_t need = rdx_wgemm_ws_bytes(M, N, tile, splits), nc = rdx_wgemm_counters(M, N, tile);
    RDX_REQUIRE(need > 0 && ws && al(ws, 16) && ws_bytes >= need && counters && n_counters >= nc);
  }
  WgArgs g;
  g.A = (const hst*)A;
  g.lda = lda;
  g.B = (const hst*)B;
  g.ldb = ldb;
  g.C = (hst*)C;
  g.ldc = ldc;
  g.M = M;
  g.N = N;
  g.K = K;
  g.bias = (const hst*)bias;
  g.aux = (const hst*)aux;
  g.ldaux = ldaux;
  g.aux_out = (hst*)aux_out;
  g.ldao = ldao;
  g.tiles_m = g.tiles_n = 0;
  g.splits = splits;
  g.ws = (float*)ws;
  g.counters = counters;
  g.wide = al(C, 16) && ldc % 8 == 0;
  if (epilogue == RDX_EPI_BIAS_GELU) g.wide = g.wide && al(aux_out, 16) && ldao % 8 == 0;
  if (epilogue == RDX_EPI_GELU_BWD) g.wide = g.wide && al(aux, 16) && ldaux % 8 == 0;
  hipStream_t st = as_stream(stream);
  switch (epilogue) {
    case RDX_EPI_BIAS: return wg_dispatch<RDX_EPI_BIAS>(g, tile, st);
    case RDX_EPI_BIAS_GELU: return wg_dispatch<RDX_EPI_BIAS_GELU>(g, tile, st);
    default: return wg_dispatch<RDX_EPI_GELU_BWD>(g, tile, st);
  }
}

extern "C" int rdx_wgemm_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M,
                              int N, int K, const void* bias, int epilogue, const void* aux, int64_t ldaux,
                              void* aux_out, int64_t ldao, int tile, void* stream) {
  return rdx_wgemm_bf16_ex(A, lda, B, ldb, C, ldc, M, N, K, bias, epilogue, aux, ldaux, aux_out, ldao, tile, 1,
                           nullptr, 0, nullptr, 0, stream);
}
