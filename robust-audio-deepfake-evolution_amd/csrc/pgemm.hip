// Deep-pipelined bf16 MFMA GEMM for the WavLM encoder projections on gfx950 (the q/k/v, out_proj, FFN1, FFN2
// GEMMs of HF WavLMEncoderLayerStableLayerNorm and their input gradients, src/models/DualStreamSEMamba.py:292-439,
// at M = B x 201 token rows: 1608 at B = 8, 6432 at B = 32).
//
//   C[M, N] = A[M, K] . B[N, K]^T     (both operands K-contiguous; same epilogues as csrc/wgemm.hip)
//
// What differs from csrc/wgemm.hip (whose loop waits for the stage it reads right after the refill is issued, so
// the in-flight depth is one stage and the fragment reads of every K step stall the MFMAs):
//   * one 512-thread workgroup per CU, 8 waves as 2 (M) x 4 (N), wave tile (BM/2) x (BN/4) in 16x16 fragments;
//   * each 64-deep K step is cut into NPH phases along the wave's fragment rows; the A fragments of phase p + 1
//     are read from LDS while the MFMAs of phase p run (two register sets), and the B fragments of step k + 1 and
//     the A fragments of its phase 0 are read during the last phase of step k (two B register sets), so no MFMA
//     waits on an LDS read latency except behind the one barrier per K step;
//   * that barrier sits before the last phase: every wave has retired its reads of stage k (lgkmcnt(0)) and its
//     LDS-DMA share of stage k + 1 (a counted vmcnt that keeps stages k + 2 .. k + NST - 1 in flight), so right
//     after it stage k's slot is refilled with stage k + NST: NST - 1 stages stay in flight across each barrier;
//   * tiles are dealt to XCDs in contiguous runs and, inside a run, grouped GROUP_M row tiles x every column
//     tile, so the 32 workgroups of an XCD that run together share their A and B panels in that XCD's L2.
// LDS images and the LDS-DMA staging are csrc/wgemm.hip's (128-B rows, 16-byte chunks XOR-swizzled by
// (row >> 1) & 7 on the source side, rows past M read as zeros through the buffer range).
#include "common.h"

namespace rdx {
namespace pg {

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) int i32x4;

__device__ void buffer_load_lds(i32x4 rsrc, __attribute__((address_space(3))) uint32_t* lds, int size, int voffset,
                                int soffset, int offset, int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");

__device__ __forceinline__ i32x4 rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  i32x4 r;
  r.x = (int)(uint32_t)a;
  r.y = (int)(uint32_t)(a >> 32);
  r.z = (int)bytes;
  r.w = 0x00020000;
  return r;
}

constexpr int KALIGN = 64;   // K % 64 == 0 (both BK forms)
// LDS image rows are BKT bf16 = 2 * BKT bytes; the 16-byte chunks of a row are XOR-swizzled so that the 16 rows x
// 4 chunks one ds_read_b128 lane group reads fall on distinct 16-byte bank slots:
//   BKT 64 (128-B rows): chunk ^ ((row >> 1) & 7);  BKT 32 (64-B rows): chunk ^ ((-(row >> 2)) & 3)
template <int BKT>
__device__ __forceinline__ int swz(int row, int ch) {
  if constexpr (BKT == 64) return ch ^ ((row >> 1) & 7);
  else return ch ^ ((-(row >> 2)) & 3);
}
__device__ __forceinline__ float gelu(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad(float x) {
  return 0.5f * (1.0f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  hst x = f2h(a), y = f2h(b);
  return (uint32_t)(*reinterpret_cast<uint16_t*>(&x)) | ((uint32_t)(*reinterpret_cast<uint16_t*>(&y)) << 16);
}

struct Args {
  const hst* A;
  int64_t lda;
  const hst* B;
  int64_t ldb;
  hst* C;
  int64_t ldc;
  int M, N, K;
  const hst* bias;
  const hst* aux;
  int64_t ldaux;
  hst* aux_out;
  int64_t ldao;
  int tiles_m, tiles_n, group_m;
  int wide;
  uint64_t* prof;              // diagnostic builds (PROF): per workgroup 8 words (see rdx_pgemm_prof)
};

// Loop-invariant LDS-DMA source offsets of this lane for the ROWS x BKT image of one operand: each wave instruction
// moves 1 KB = 1024 / (2 BKT) rows, lane l landing at byte 16 l of the piece (row l / (BKT / 8), chunk l % (BKT / 8)),
// so the swizzle is applied to the SOURCE chunk. The ROWS * 2 BKT / 1024 pieces are dealt round-robin to the 8
// waves (NPW per wave); the K offset of a stage goes in the scalar soffset.
template <int ROWS, int BKT>
struct Stager {
  static constexpr int CPR = BKT / 8;                    // 16-byte chunks per row
  static constexpr int RPP = 64 / CPR;                   // rows per 1 KB piece
  static constexpr int NP = ROWS / RPP;                  // pieces per image
  static constexpr int NPW = NP / 8;                     // pieces per wave
  static_assert(NP % 8 == 0, "pieces must deal evenly over 8 waves");
  int voff[NPW];
  __device__ __forceinline__ void init(int64_t ld_bytes, int wave, int lane) {
    const int rr = lane / CPR, pos = lane % CPR;
#pragma unroll
    for (int j = 0; j < NPW; ++j) {
      const int row = (j * 8 + wave) * RPP + rr;
      voff[j] = (int)(row * ld_bytes) + swz<BKT>(row, pos) * 16;
    }
  }
  __device__ __forceinline__ void issue(i32x4 rs, int k0_bytes, char* img, int wave) const {
#pragma unroll
    for (int j = 0; j < NPW; ++j)
      buffer_load_lds(rs, (__attribute__((address_space(3))) uint32_t*)(img + (j * 8 + wave) * 1024), 16, voff[j],
                      k0_bytes, 0, 0);
  }
};

template <int N>
__device__ __forceinline__ void wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// s_waitcnt vmcnt(n * LPS) lgkmcnt(0) + s_barrier for a runtime n in [0, NST - 2]
template <int LPS, int NST>
__device__ __forceinline__ void wait_stages_barrier(int n) {
  if constexpr (NST >= 8) { if (n >= 6) { wait_barrier<6 * LPS>(); return; } }
  if constexpr (NST >= 7) { if (n >= 5) { wait_barrier<5 * LPS>(); return; } }
  if constexpr (NST >= 6) { if (n >= 4) { wait_barrier<4 * LPS>(); return; } }
  if constexpr (NST >= 5) { if (n >= 3) { wait_barrier<3 * LPS>(); return; } }
  if constexpr (NST >= 4) { if (n >= 2) { wait_barrier<2 * LPS>(); return; } }
  if constexpr (NST >= 3) { if (n >= 1) { wait_barrier<LPS>(); return; } }
  wait_barrier<0>();
}

// PROF: thread 0 stores, per workgroup, shader-clock stamps at entry / stage 0 landed / main loop done / exit, the
// 100 MHz real-time clock at entry and exit, and the XCC / hardware ids (vector stores to a buffer of its own)
__device__ __forceinline__ uint64_t pg_hwid() {
  uint32_t xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  return ((uint64_t)xcc << 32) | hw;
}

// K step of BKT (64 or 32) in NPH phases along the wave's fragment rows (NPH even): the A fragments of phase p + 1
// are read while the MFMAs of phase p run, all B fragments of a step are held (two B register sets: step k + 1's
// are read during the last phase of step k, after the barrier).
template <int BM, int BN, int BKT, int NST, int NPH, int EPI, int PRIO, int PROF = 0, int ABL = 0>
__global__ __launch_bounds__(512, 1) void pgemm_kernel(Args g) {
  uint64_t ts0 = 0, ts1 = 0, ts2 = 0, rt0 = 0;
  if (PROF) { ts0 = __builtin_amdgcn_s_memtime(); rt0 = __builtin_amdgcn_s_memrealtime(); }
  constexpr int WM = 2, WN = 4;
  constexpr int WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  constexpr int FMP = FM / NPH;                       // fragment rows per phase
  constexpr int KK = BKT / 32;                        // 16x16x32 MFMA k-chunks per step
  constexpr int ROWB = BKT * 2;                       // LDS image row bytes
  constexpr int IMG_A = BM * ROWB, STAGE = (BM + BN) * ROWB;
  using SA = Stager<BM, BKT>;
  using SB = Stager<BN, BKT>;
  constexpr int LPS = SA::NPW + SB::NPW;              // LDS-DMA instructions per wave per stage
  static_assert(FM % NPH == 0 && (NPH % 2) == 0 && NPH >= 2, "phases");
  static_assert(NST >= 2 && NST <= 8, "ring depth");
  extern __shared__ __attribute__((aligned(1024))) char lds[];

  // work id -> (mt, nt): XCD-contiguous runs, then GROUP_M row tiles x all column tiles per group
  const int nwg = g.tiles_m * g.tiles_n;
  int t;
  {
    const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  int mt, nt;
  {
    const int gm = g.group_m;
    if (PROF && gm < 0) {             // diagnostic: every workgroup on tile (0, 0) (L2-resident operands)
      mt = nt = 0;
    } else if (gm <= 0 || gm >= g.tiles_m) {
      nt = t / g.tiles_m;
      mt = t - nt * g.tiles_m;
    } else {
      const int per = gm * g.tiles_n, grp = t / per, first = grp * gm;
      const int gsz = min(g.tiles_m - first, gm), rem = t - grp * per;
      nt = rem / gsz;
      mt = first + (rem - nt * gsz);
    }
  }
  const int m0 = mt * BM, n0 = nt * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int M = g.M, N = g.N, K = g.K;
  const int nk = K / BKT;

  const int64_t lda_b = g.lda * 2, ldb_b = g.ldb * 2;
  const int rows_a = min(BM, M - m0), rows_b = min(BN, N - n0);
  const i32x4 ra = rsrc(g.A + (int64_t)m0 * g.lda, (uint32_t)((int64_t)(rows_a - 1) * lda_b + (int64_t)K * 2));
  const i32x4 rb = rsrc(g.B + (int64_t)n0 * g.ldb, (uint32_t)((int64_t)(rows_b - 1) * ldb_b + (int64_t)K * 2));
  SA sa;
  SB sb;
  sa.init(lda_b, wave, lane);
  sb.init(ldb_b, wave, lane);

  auto issue = [&](int kt) {
    char* st = lds + (kt % NST) * STAGE;
    sa.issue(ra, kt * ROWB, st, wave);
    sb.issue(rb, kt * ROWB, st + IMG_A, wave);
  };

  const int fr = lane & 15, fq = lane >> 4;
  // fragment reads of stage kt: A rows of phase p (FMP fragments x KK), all B columns (FN x KK)
  auto read_a = [&](int kt, int p, hx8 (&af)[KK][FMP]) {
    const char* As = lds + (kt % NST) * STAGE;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
#pragma unroll
      for (int i = 0; i < FMP; ++i) {
        const int row = wm * WTM + (p * FMP + i) * 16 + fr;
        af[kk][i] = *reinterpret_cast<const hx8*>(As + row * ROWB + 16 * swz<BKT>(row, kk * 4 + fq));
      }
  };
  auto read_b = [&](int kt, hx8 (&bf)[KK][FN]) {
    const char* Bs = lds + (kt % NST) * STAGE + IMG_A;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * WTN + j * 16 + fr;
        bf[kk][j] = *reinterpret_cast<const hx8*>(Bs + row * ROWB + 16 * swz<BKT>(row, kk * 4 + fq));
      }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mfma_phase = [&](int p, const hx8 (&af)[KK][FMP], const hx8 (&bf)[KK][FN]) {
    if (ABL == 2) {                   // diagnostic: fragments read, no MFMA
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
#pragma unroll
        for (int i = 0; i < FMP; ++i) asm volatile("" ::"v"(af[kk][i]));
#pragma unroll
        for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(bf[kk][j]));
      }
      return;
    }
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
#pragma unroll
      for (int i = 0; i < FMP; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[p * FMP + i][j] = mfma16x16x32(bf[kk][j], af[kk][i], acc[p * FMP + i][j]);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  };

  // prologue: stages 0 .. min(NST, nk) - 1 in flight, wait for stage 0
  const int pre = min(NST, nk);
#pragma unroll
  for (int s = 0; s < NST; ++s)
    if (s < pre) issue(s);
  wait_stages_barrier<LPS, NST + 1>(pre - 1);
  __builtin_amdgcn_sched_barrier(0);
  if (PROF) ts1 = __builtin_amdgcn_s_memtime();

  hx8 a0[KK][FMP], a1[KK][FMP], b0[KK][FN], b1[KK][FN];
  read_b(0, b0);
  read_a(0, 0, a0);

  // one K step with B fragments bc (this step) / bn (next step); the fences keep each phase's reads issued
  // before its MFMAs (the scheduler would otherwise sink them next to the barrier's lgkmcnt(0))
  auto step = [&](int kt, hx8 (&bc)[KK][FN], hx8 (&bn)[KK][FN]) {
#pragma unroll
    for (int p = 0; p < NPH - 1; ++p) {
      if (p & 1) {
        read_a(kt, p + 1, a0);
        __builtin_amdgcn_sched_barrier(0);
        mfma_phase(p, a1, bc);
      } else {
        read_a(kt, p + 1, a1);
        __builtin_amdgcn_sched_barrier(0);
        mfma_phase(p, a0, bc);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // every read of stage kt retired, this wave's share of stage kt + 1 landed; then the next step's fragment
    // reads and the refill of kt's slot with stage kt + NST
    if (kt + 1 < nk) {
      wait_stages_barrier<LPS, NST>(min(NST - 2, nk - 2 - kt));
      __builtin_amdgcn_sched_barrier(0);
      read_b(kt + 1, bn);
      read_a(kt + 1, 0, a0);
      if (ABL != 1 && kt + NST < nk) issue(kt + NST);   // ABL 1 (diagnostic): no refills
      __builtin_amdgcn_sched_barrier(0);
    }
    mfma_phase(NPH - 1, a1, bc);      // NPH is even: the last phase's A fragments are in a1
    __builtin_amdgcn_sched_barrier(0);
  };

  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    step(kt, b0, b1);
    step(kt + 1, b1, b0);
  }
  if (kt < nk) step(kt, b0, b1);
  if (PROF) ts2 = __builtin_amdgcn_s_memtime();

  // epilogue: the tile through an LDS image (rows padded by 16 B), then whole rows, 16 bytes per lane
  // acc[i][j][e] = C[m0 + wm*WTM + i*16 + fr][n0 + wn*WTN + j*16 + 4*fq + e]
  constexpr int PITCH = BN * 2 + 16;
  char* img = lds;
  wait_barrier<0>();
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
      *reinterpret_cast<uint2*>(img + r * PITCH + c * 2) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;
#pragma unroll 4
  for (int idx = tid; idx < BM * CPR; idx += 512) {
    const int r = idx / CPR, c = (idx - r * CPR) * 8;
    const int m = m0 + r, n = n0 + c;
    if (m >= M || n >= N) continue;
    const bool full = n + 8 <= N;
    const bool wide = full && g.wide;
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
        const float a0v = hlo(qw[e]), a1v = hhi(qw[e]);
        const float u0 = hlo(uw[e]), u1 = hhi(uw[e]);
        o[e] = pack2(a0v * gelu_grad(u0), a1v * gelu_grad(u1));
      }
      q = make_uint4(o[0], o[1], o[2], o[3]);
    }
    st8(g.C + (int64_t)m * g.ldc + n, q);
    if (EPI == RDX_EPI_BIAS_GELU) {
      const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
      uint32_t o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        o[e] = pack2(gelu(hlo(qw[e])), gelu(hhi(qw[e])));
      st8(g.aux_out + (int64_t)m * g.ldao + n, make_uint4(o[0], o[1], o[2], o[3]));
    }
  }
  if (PROF) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const uint64_t ts3 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
      uint64_t* o = g.prof + (int64_t)blockIdx.x * 8;
      o[0] = ts0; o[1] = ts1; o[2] = ts2; o[3] = ts3; o[4] = rt0; o[5] = rt1; o[6] = pg_hwid();
      o[7] = ((uint64_t)mt << 32) | (uint32_t)nt;
    }
  }
}

template <int BM, int BN, int BKT, int NST, int NPH, int EPI, int PRIO, int PROF = 0, int ABL = 0>
static int launch(Args g, hipStream_t st) {
  g.tiles_m = (g.M + BM - 1) / BM;
  g.tiles_n = (g.N + BN - 1) / BN;
  constexpr int ring = NST * (BM + BN) * BKT * 2, image = BM * (BN * 2 + 16);
  constexpr int lds = ring > image ? ring : image;
  static_assert(lds <= 160 * 1024, "LDS");
  auto kern = &pgemm_kernel<BM, BN, BKT, NST, NPH, EPI, PRIO, PROF, ABL>;
  static bool lds_ok = false;
  if (!lds_ok) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int)e;
    lds_ok = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)(g.tiles_m * g.tiles_n)), dim3(512), lds, st, g);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

// tile codes: BM x BN, K step, ring stages, phases per step; + 100: s_setprio(1) around the MFMA clusters
template <int EPI, int PRIO>
static int dispatch(const Args& g, int tile, hipStream_t st) {
  switch (tile) {
    case 0: return launch<256, 256, 32, 5, 2, EPI, PRIO>(g, st);
    case 1: return launch<256, 128, 32, 6, 2, EPI, PRIO>(g, st);
    case 2: return launch<128, 256, 32, 6, 2, EPI, PRIO>(g, st);
    case 3: return launch<128, 128, 32, 8, 2, EPI, PRIO>(g, st);
    case 4: return launch<128, 192, 64, 4, 2, EPI, PRIO>(g, st);
    case 5: return launch<128, 256, 64, 3, 2, EPI, PRIO>(g, st);
    case 6: return launch<256, 128, 64, 3, 4, EPI, PRIO>(g, st);
    case 7: return launch<128, 128, 64, 4, 2, EPI, PRIO>(g, st);
    case 8: return launch<256, 256, 32, 4, 2, EPI, PRIO>(g, st);
    case 9: return launch<256, 256, 32, 5, 4, EPI, PRIO>(g, st);
    default: return RDX_EINVAL;
  }
}

// diagnostic (PROF) instantiations, bias epilogue: tiles 0 / 2 / 4; + 10: no refills in the K loop; + 20: no MFMA
static int dispatch_prof(const Args& g, int tile, hipStream_t st) {
  switch (tile) {
    case 0: return launch<256, 256, 32, 5, 2, RDX_EPI_BIAS, 0, 1>(g, st);
    case 2: return launch<128, 256, 32, 6, 2, RDX_EPI_BIAS, 0, 1>(g, st);
    case 4: return launch<128, 192, 64, 4, 2, RDX_EPI_BIAS, 0, 1>(g, st);
    case 10: return launch<256, 256, 32, 5, 2, RDX_EPI_BIAS, 0, 1, 1>(g, st);
    case 12: return launch<128, 256, 32, 6, 2, RDX_EPI_BIAS, 0, 1, 1>(g, st);
    case 14: return launch<128, 192, 64, 4, 2, RDX_EPI_BIAS, 0, 1, 1>(g, st);
    case 20: return launch<256, 256, 32, 5, 2, RDX_EPI_BIAS, 0, 1, 2>(g, st);
    case 22: return launch<128, 256, 32, 6, 2, RDX_EPI_BIAS, 0, 1, 2>(g, st);
    case 24: return launch<128, 192, 64, 4, 2, RDX_EPI_BIAS, 0, 1, 2>(g, st);
    default: return RDX_EINVAL;
  }
}

static bool geometry(int tile, int* bm, int* bn) {
  switch (tile % 100) {
    case 0: case 8: case 9: *bm = 256; *bn = 256; return true;
    case 1: case 6: *bm = 256; *bn = 128; return true;
    case 2: case 5: *bm = 128; *bn = 256; return true;
    case 3: case 7: *bm = 128; *bn = 128; return true;
    case 4: *bm = 128; *bn = 192; return true;
    default: return false;
  }
}

}  // namespace pg
}  // namespace rdx

using namespace rdx;

static int pgemm_entry(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N,
                       int K, const void* bias, int epilogue, const void* aux, int64_t ldaux, void* aux_out,
                       int64_t ldao, int tile, int group_m, uint64_t* prof, void* stream) {
  auto al = [](const void* p, int a) { return ((uintptr_t)p & (a - 1)) == 0; };
  RDX_REQUIRE(A && B && C && M > 0 && N > 0 && K > 0 && al(A, 16) && al(B, 16) && al(C, 8));
  RDX_REQUIRE(K % pg::KALIGN == 0 && lda % 8 == 0 && ldb % 8 == 0 && lda >= K && ldb >= K && N % 4 == 0 && ldc >= N &&
              ldc % 4 == 0);
  RDX_REQUIRE((int64_t)256 * lda * 2 + (int64_t)K * 2 < 0x7fffffffLL && (int64_t)256 * ldb * 2 < 0x7fffffffLL);
  RDX_REQUIRE(!bias || al(bias, 8));
  RDX_REQUIRE(epilogue == RDX_EPI_BIAS || epilogue == RDX_EPI_BIAS_GELU || epilogue == RDX_EPI_GELU_BWD);
  if (epilogue == RDX_EPI_BIAS_GELU) RDX_REQUIRE(aux_out && ldao >= N && ldao % 4 == 0 && al(aux_out, 8));
  if (epilogue == RDX_EPI_GELU_BWD) RDX_REQUIRE(aux && ldaux >= N && ldaux % 4 == 0 && al(aux, 8));
  int bm, bn;
  RDX_REQUIRE(tile >= 0 && tile < 200 && (pg::geometry(tile, &bm, &bn) || prof));
  RDX_REQUIRE(group_m >= 0 || prof);
  pg::Args g;
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
  g.group_m = group_m;
  g.prof = prof;
  g.wide = al(C, 16) && ldc % 8 == 0;
  if (epilogue == RDX_EPI_BIAS_GELU) g.wide = g.wide && al(aux_out, 16) && ldao % 8 == 0;
  if (epilogue == RDX_EPI_GELU_BWD) g.wide = g.wide && al(aux, 16) && ldaux % 8 == 0;
  hipStream_t st = as_stream(stream);
  if (prof) {
    RDX_REQUIRE(epilogue == RDX_EPI_BIAS && tile < 30);
    return pg::dispatch_prof(g, tile, st);
  }
  const bool prio = tile >= 100;
  const int base = tile % 100;
  switch (epilogue) {
    case RDX_EPI_BIAS:
      return prio ? pg::dispatch<RDX_EPI_BIAS, 1>(g, base, st) : pg::dispatch<RDX_EPI_BIAS, 0>(g, base, st);
    case RDX_EPI_BIAS_GELU:
      return prio ? pg::dispatch<RDX_EPI_BIAS_GELU, 1>(g, base, st) : pg::dispatch<RDX_EPI_BIAS_GELU, 0>(g, base, st);
    default:
      return prio ? pg::dispatch<RDX_EPI_GELU_BWD, 1>(g, base, st) : pg::dispatch<RDX_EPI_GELU_BWD, 0>(g, base, st);
  }
}

extern "C" int rdx_pgemm_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M,
                              int N, int K, const void* bias, int epilogue, const void* aux, int64_t ldaux,
                              void* aux_out, int64_t ldao, int tile, int group_m, void* stream) {
  return pgemm_entry(A, lda, B, ldb, C, ldc, M, N, K, bias, epilogue, aux, ldaux, aux_out, ldao, tile, group_m, nullptr,
                     stream);
}

// Diagnostic form (bias epilogue, tiles 0 / 2 / 4; + 10 = no refills in the K loop, + 20 = no MFMA; group_m -1
// puts every workgroup on tile (0, 0)): also stores 8 words per workgroup into prof [grid][8]: shader-clock stamps at entry / stage 0 landed / main loop done / exit, 100 MHz real-time stamps at entry / exit, the
// (XCC id << 32 | HW_ID) word and (row tile << 32 | column tile).
extern "C" int rdx_pgemm_prof(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M,
                              int N, int K, const void* bias, int tile, int group_m, void* prof, void* stream) {
  RDX_REQUIRE(prof != nullptr);
  return pgemm_entry(A, lda, B, ldb, C, ldc, M, N, K, bias, RDX_EPI_BIAS, nullptr, 0, nullptr, 0, tile, group_m,
                     (uint64_t*)prof, stream);
}
