// Ping-pong MFMA GEMM for the WavLM encoder projections on gfx950: the q/k/v, out_proj, FFN1, FFN2 GEMMs of HF
// WavLMEncoderLayerStableLayerNorm and their input gradients (src/models/DualStreamSEMamba.py:292-439, run under
// autocast, src/main.py:1049), at M = B x 201 token rows (B = 8: 1608, B = 32: 6432).
//
//   C[M, N] = A[M, K] . B[N, K]^T     (both operands K-contiguous; the epilogues of csrc/wgemm.hip)
//
// Structure (cdna_hip_programming.md "The 256^2 8-phase template", MI355X_MICROARCH.md "Two waves per SIMD"):
//   * one 512-thread workgroup per CU: 8 waves as 2 (M) x 4 (N), two per SIMD. Waves 0-3 (row group 0) and 4-7
//     (row group 1) run staggered by one s_barrier, so on every SIMD one wave is in its MFMA segment while its
//     partner reads fragments from LDS and issues LDS-DMA loads;
//   * a 64-deep K step is cut into NPH = NPA x NPB phases, each the MFMAs of one (A part, B part) pair of the
//     wave's tile (snake order, so every fragment is read from LDS once per K step and stays in registers while
//     needed); a phase is [fragment reads, LDS-DMA issue, counted vmcnt + lgkmcnt(0)] s_barrier [MFMA] s_barrier;
//   * the LDS is a ring of S = U x SPK slabs of 64 rows x 64 k (8 KB, one buffer_load_dwordx4 ... lds per thread).
//     A K step's slabs are ordered by the phase that first reads them; a slab read in phase p is refilled in phase
//     p + 1 with the same slab of K step kt + U (the read was retired by lgkmcnt(0) before the barrier the refill
//     follows), so S - (slabs read in phases p and p + 1) slabs stay in flight across every barrier, and phase p's
//     counted vmcnt retires exactly the slabs phase p + 1 reads. Past the last K step the refills take a buffer
//     descriptor of zero records (no memory traffic; the count stays exact);
//   * LDS images are 128-B rows with the 16-byte chunk XOR-swizzled by (row >> 1) & 7 (conflict-free
//     ds_read_b128 for the 16x16x32 fragments), applied to the DMA's SOURCE chunk (the DMA writes lane-linear);
//     a slab's 64 image rows gather the tile rows its phase reads (any row order is free for the per-lane
//     source address); rows >= M / N read as zeros through the buffer range;
//   * v_mfma_f32_16x16x32 computing C^T: a lane ends with 4 consecutive output columns of one row;
//   * work ids are dealt to XCDs in contiguous runs (bijective remap), then GROUP_M row tiles x every column tile
//     per group; split-K (splits > 1): the splits of a tile are consecutive work ids, publish fp32 partials and
//     the last arriver sums them in split order (deterministic) and runs the epilogue;
//   * epilogue through an LDS image of the tile (16-byte padded rows), whole rows stored 16 bytes per lane.
#include <algorithm>
#include <utility>

#include "common.h"

namespace rdx {
namespace hg {

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

__device__ void buffer_load_lds(i32x4 rsrc, __attribute__((address_space(3))) uint32_t* lds, int size, int voffset,
                                int soffset, int offset, int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");

__device__ __forceinline__ i32x4 rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  i32x4 r;
  r.x = (int)(uint32_t)a;
  r.y = (int)(uint32_t)(a >> 32);
  r.z = (int)bytes;
  r.w = 0x00020000;  // raw buffer: dword-aligned, no swizzle, range-checked
  return r;
}

__device__ __forceinline__ int swz(int row, int ch) { return ch ^ ((row >> 1) & 7); }

__device__ __forceinline__ uint32_t pack2(float a, float b) { return hpack2(a, b); }

template <int N, class F, int... Is>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl<N>(f, std::make_integer_sequence<int, N>{});
}

struct Args {
  const hst* A;
  int64_t lda;
  const hst* B;
  int64_t ldb;
  hst* C;
  int64_t ldc;
  int M, N, K;
  const hst* bias;   // [N] or null
  const hst* aux;    // GELU_BWD: u [M, ldaux]
  int64_t ldaux;
  hst* aux_out;      // BIAS_GELU: gelu(u) [M, ldao]
  int64_t ldao;
  int tiles_m, tiles_n, group_m;
  int splits;        // split-K factor; split s covers k-steps [s*nk/S, (s+1)*nk/S); 0: stream-K
  int maxc;          // partial slots per tile in ws (splits, or the stream-K bound)
  int grid_sk;       // stream-K grid (host side)
  float* ws;         // split-K partial slabs [tile][split][FM*FN][512][4] fp32
  int* counters;     // split-K arrival tickets, one per tile, zero between launches
  int wide;          // C / aux / aux_out rows 16-byte aligned: 16-byte row-phase accesses
  // split-precision (X3) form, csrc/hgemm.hip rdx_hgemm_x3: A = A + A2, B = B + B2 (bf16 hi / lo planes of fp32
  // operands, same strides); the K loop runs 3 K passes, (A, B), (A2, B), (A, B2)
  const hst* A2;
  const hst* B2;
  int64_t sa, sc;    // batch strides (elements) of A / A2 and of C / aux_out (blockIdx.y = batch index)
};

// The phase / slab plan of a BM x BN tile with its A part split NPA ways and its B part NPB ways.
template <int BM, int BN, int NPA, int NPB>
struct Plan {
  static constexpr int FM = BM / 32, FN = BN / 64;        // 16x16 fragments per wave (2 x 4 waves)
  static constexpr int WTM = BM / 2, WTN = BN / 4;
  static constexpr int FMP = FM / NPA, FNP = FN / NPB;    // fragments of one part
  static constexpr int RA = WTM / NPA, RB = WTN / NPB;    // rows of one wave's part
  static constexpr int SA = BM / NPA / 64, SB = BN / NPB / 64;   // slabs of one part (both groups / all 4 waves)
  static constexpr int NPH = NPA * NPB;
  static constexpr int SPK = BM / 64 + BN / 64;           // slabs per K step
  static_assert(FM % NPA == 0 && FN % NPB == 0 && (BM / NPA) % 64 == 0 && (BN / NPB) % 64 == 0, "plan");
  static constexpr int pa(int q) { return q / NPB; }
  static constexpr int pb(int q) { return ((q / NPB) & 1) ? NPB - 1 - q % NPB : q % NPB; }
  static constexpr bool anew(int q) { return q % NPB == 0; }
  static constexpr bool bnew(int q) { return q < NPB; }
  static constexpr int reads(int q) { return (anew(q) ? SA : 0) + (bnew(q) ? SB : 0); }
  static constexpr int first(int q) { return q == 0 ? 0 : first(q - 1) + reads(q - 1); }
  // slab index (in the K step's read order) of A part a / B part b
  static constexpr int ja(int a) { return first(a * NPB); }
  static constexpr int jb(int b) { return first(b) + (anew(b) ? SA : 0); }
  // slab j -> (is B, part, slab within part)
  static constexpr int slab_isb(int j) {
    for (int q = 0; q < NPH; ++q) {
      const int f = first(q);
      if (j >= f && j < f + reads(q)) return (anew(q) && j < f + SA) ? 0 : 1;
    }
    return -1;
  }
  static constexpr int slab_part(int j) {
    for (int q = 0; q < NPH; ++q) {
      const int f = first(q);
      if (j >= f && j < f + reads(q)) return (anew(q) && j < f + SA) ? pa(q) : pb(q);
    }
    return -1;
  }
  static constexpr int slab_in_part(int j) {
    for (int q = 0; q < NPH; ++q) {
      const int f = first(q);
      if (j >= f && j < f + reads(q)) return (anew(q) && j < f + SA) ? j - f : j - f - (anew(q) ? SA : 0);
    }
    return -1;
  }
};

template <int N>
__device__ __forceinline__ void wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// output tile index -> (row tile, column tile): GROUP_M row tiles x every column tile per group (0: column-panel order)
__device__ __forceinline__ void tile_coords(const Args& g, int tile, int& mt, int& nt) {
  const int gm = g.group_m;
  if (gm <= 0 || gm >= g.tiles_m) {
    nt = tile / g.tiles_m;
    mt = tile - nt * g.tiles_m;
  } else {
    const int per = gm * g.tiles_n, grp = tile / per, first = grp * gm;
    const int gsz = min(g.tiles_m - first, gm), rem = tile - grp * per;
    nt = rem / gsz;
    mt = first + (rem - nt * gsz);
  }
}

// group_m < 0: the tiles as an R x (8 / R) grid of rectangular blocks (R = -group_m row groups, 8 / R column groups),
// one per XCD, laid out block after block: each XCD's L2 takes only the A rows of its row group and the B panels of
// its column group (over the chip A is fetched 8 / R times instead of 8 in column-panel order, B R times instead of
// once). Position t of that order -> (tile row, tile column, split); the XCD
// deal below hands each XCD a contiguous run of positions, so where the blocks' sizes differ by a few work ids the
// excess lands on a neighbour's XCD (a locality loss, never a correctness one).
__device__ __forceinline__ void grid_coords(const Args& g, int t, int spl, int& mt, int& nt, int& split) {
  const int R = -g.group_m, C = 8 / R;
  int pos = t;
  mt = nt = split = 0;
  for (int x = 0; x < 8; ++x) {
    const int rg = x / C, cg = x - rg * C;
    const int r0 = rg * g.tiles_m / R, r1 = (rg + 1) * g.tiles_m / R;
    const int c0 = cg * g.tiles_n / C, c1 = (cg + 1) * g.tiles_n / C;
    const int sz = (r1 - r0) * (c1 - c0) * spl;
    if (pos < sz) {
      const int tl = pos / spl, w = c1 - c0;
      split = pos - tl * spl;
      mt = r0 + tl / w;
      nt = c0 + tl % w;
      return;
    }
    pos -= sz;
  }
}

// bijective deal of n work ids onto the 8 XCDs in contiguous runs (blocks b and b + 8 share an XCD)
__device__ __forceinline__ int xcd_remap(int bid, int n) {
  const int xcd = bid & 7, q = n >> 3, r = n & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// One output tile's K steps [kb, kb + nk): the ring, the phases, then either the epilogue (nc == 1) or this
// contribution's fp32 partial in slot `slot` of the tile's nc and, for the last of them to arrive, the sum of the nc
// partials in slot order and the epilogue.
template <int BM, int BN, int NPA, int NPB, int U, int EPI, int PRIO, int ABL, int X3 = 0>
__device__ __forceinline__ void run_segment(const Args& g, char* lds, int mt, int nt, int tile, int kb, int nk,
                                            int slot, int nc, int maxc) {
  // batched form (rdx_hgemm_batched, rdx_hgemm_x3): blockIdx.y selects the problem, A (and A2) advanced by sa and
  // C / aux / aux_out by sc elements (gridDim.y == 1 otherwise)
  const int64_t yb = (int64_t)blockIdx.y;
  using P = Plan<BM, BN, NPA, NPB>;
  constexpr int FM = P::FM, FN = P::FN, WTM = P::WTM, WTN = P::WTN, FMP = P::FMP, FNP = P::FNP;
  constexpr int NPH = P::NPH, SPK = P::SPK, S = U * SPK;
  constexpr int SLAB = 8192;
  static_assert(S * SLAB <= 160 * 1024, "ring");
  __syncthreads();                                // the previous segment's epilogue is done with the LDS
  const int m0 = mt * BM, n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int M = g.M, N = g.N, K = g.K;

  const int64_t lda_b = g.lda * 2, ldb_b = g.ldb * 2;
  const int rows_a = min(BM, M - m0), rows_b = min(BN, N - n0);
  const i32x4 ra = rsrc(g.A + yb * g.sa + (int64_t)m0 * g.lda, (uint32_t)((int64_t)(rows_a - 1) * lda_b + (int64_t)K * 2));
  const i32x4 rb = rsrc(g.B + (int64_t)n0 * g.ldb, (uint32_t)((int64_t)(rows_b - 1) * ldb_b + (int64_t)K * 2));
  const i32x4 rnull = rsrc(g.A, 0u);
  // X3: the planes' base addresses (64-bit scalars: the descriptor of a refill is built from the pass's base, so
  // no descriptor is selected through memory), their buffer ranges, and the K steps per pass
  const uint64_t xa0 = (uint64_t)(g.A + yb * g.sa + (int64_t)m0 * g.lda);
  const uint64_t xa1 = X3 ? (uint64_t)(g.A2 + yb * g.sa + (int64_t)m0 * g.lda) : xa0;
  const uint64_t xb0 = (uint64_t)(g.B + (int64_t)n0 * g.ldb);
  const uint64_t xb1 = X3 ? (uint64_t)(g.B2 + (int64_t)n0 * g.ldb) : xb0;
  const uint32_t xra = (uint32_t)((int64_t)(rows_a - 1) * lda_b + (int64_t)K * 2);
  const uint32_t xrb = (uint32_t)((int64_t)(rows_b - 1) * ldb_b + (int64_t)K * 2);
  const int nkp = K / 64;

  // loop-invariant DMA source offsets of this lane, one per slab of a K step: image row ir = 8 * wave + lane / 8,
  // position lane % 8 holding source chunk swz(ir, lane % 8)
  int voff[SPK];
  {
    const int ir = 8 * wave + (lane >> 3), ch = swz(ir, lane & 7);
    static_for<SPK>([&](auto JC) {
      constexpr int j = decltype(JC)::value;
      constexpr int isb = P::slab_isb(j), part = P::slab_part(j), sip = P::slab_in_part(j);
      const int rr = sip * 64 + ir;
      int row;
      if constexpr (isb == 0) row = (rr / P::RA) * WTM + part * P::RA + rr % P::RA;
      else row = (rr / P::RB) * WTN + part * P::RB + rr % P::RB;
      voff[j] = (int)(row * (isb ? ldb_b : lda_b)) + ch * 16;
    });
  }
  // issue slab j of K step kst into ring position pos (slot pos * SPK + j)
  auto issue = [&](auto JC, int pos, int kst) {
    constexpr int j = decltype(JC)::value;
    constexpr int isb = P::slab_isb(j);
    const bool live = kst < nk;
    i32x4 rs;
    int kbytes;
    if constexpr (X3) {
      // pass p of global K step ks: (A, B), (A2, B), (A, B2)
      const int ks = kb + kst;
      const int p = (ks >= nkp) + (ks >= 2 * nkp);
      const uint64_t base = isb ? (p == 2 ? xb1 : xb0) : (p == 1 ? xa1 : xa0);
      rs = rsrc((const void*)base, live ? (isb ? xrb : xra) : 0u);
      kbytes = __builtin_amdgcn_readfirstlane(live ? (ks - p * nkp) * 128 : 0);   // uniform: keep it scalar
    } else {
      rs = live ? (isb ? rb : ra) : rnull;
      kbytes = live ? (kb + kst) * 128 : 0;
    }
    buffer_load_lds(rs, (__attribute__((address_space(3))) uint32_t*)(lds + (pos * SPK + j) * SLAB + wave * 1024),
                    16, voff[j], kbytes, 0, 0);
  };

  // per-lane fragment read offsets: row fr of a 16-row fragment, chunk kk * 4 + fq, swizzled by the row
  const int fr = lane & 15, fq = lane >> 4;
  const int sw = (fr >> 1) & 7;
  const int lofs0 = fr * 128 + 16 * ((0 * 4 + fq) ^ sw), lofs1 = fr * 128 + 16 * ((1 * 4 + fq) ^ sw);
  const int arow0 = wm * P::RA, brow0 = wn * P::RB;

  hx8 af[2][FM], bf[2][FN];
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the tile's bias columns: loaded ahead of the ring (older than every DMA, so the prologue's counted wait retires
  // it too), parked in LDS past the ring and the epilogue image for the epilogue's register phase
  constexpr int BIAS_OFF = (S * SLAB > BM * (BN * 2 + 16) ? S * SLAB : BM * (BN * 2 + 16));
  constexpr int FLAG_OFF = BIAS_OFF + BN * 2;     // the split / stream-K arrival broadcast
  static_assert(FLAG_OFF + 16 <= 160 * 1024, "bias slot");
  constexpr bool F32EPI = EPI == RDX_EPI_F32 || EPI == RDX_EPI_F32_GELU_SPLIT;
  const bool has_bias = EPI != RDX_EPI_GELU_BWD && !F32EPI && g.bias != nullptr;
  uint2 bias4 = make_uint2(0u, 0u);
  if (has_bias && tid < BN / 4 && n0 + 4 * tid < N) bias4 = *reinterpret_cast<const uint2*>(g.bias + n0 + 4 * tid);
  __builtin_amdgcn_sched_barrier(0);

  // prologue: the whole ring (K steps 0 .. U - 1), then retire what phase 0 reads
#pragma unroll
  for (int u = 0; u < U; ++u) static_for<SPK>([&](auto JC) { issue(JC, u, u); });
  wait_barrier<S - P::reads(0)>();
  __builtin_amdgcn_sched_barrier(0);
  if (tid < BN / 4) *reinterpret_cast<uint2*>(lds + BIAS_OFF + 8 * tid) = bias4;   // read after later barriers
  if (wm == 1) __builtin_amdgcn_s_barrier();     // row group 1 runs one barrier behind group 0
  __builtin_amdgcn_sched_barrier(0);
  if (PRIO == 2 && wm == 1) __builtin_amdgcn_s_setprio(1);

  // one phase q of K step kt held at ring position u
  auto phase = [&](auto UC, auto QC, int kt) {
    constexpr int u = decltype(UC)::value, q = decltype(QC)::value;
    constexpr int a = P::pa(q), b = P::pb(q);
    // 1. this phase's first reads
    if constexpr (P::anew(q)) {
      const char* base = lds + (u * SPK + P::ja(a)) * SLAB + arow0 * 128;
#pragma unroll
      for (int i = 0; i < FMP; ++i) {
        af[0][a * FMP + i] = *reinterpret_cast<const hx8*>(base + i * 2048 + lofs0);
        af[1][a * FMP + i] = *reinterpret_cast<const hx8*>(base + i * 2048 + lofs1);
      }
    }
    if constexpr (P::bnew(q)) {
      const char* base = lds + (u * SPK + P::jb(b)) * SLAB + brow0 * 128;
#pragma unroll
      for (int j = 0; j < FNP; ++j) {
        bf[0][b * FNP + j] = *reinterpret_cast<const hx8*>(base + j * 2048 + lofs0);
        bf[1][b * FNP + j] = *reinterpret_cast<const hx8*>(base + j * 2048 + lofs1);
      }
    }
    // 2. refill the slabs the previous phase read, with the same slabs U K steps later
    if constexpr (ABL == 1) {
    } else if constexpr (q >= 1) {
      constexpr int f = P::first(q - 1), n = P::reads(q - 1);
      static_for<n>([&](auto IC) { issue(std::integral_constant<int, f + decltype(IC)::value>{}, u, kt + U); });
    } else {
      constexpr int f = P::first(NPH - 1), n = P::reads(NPH - 1);
      constexpr int up = (u + U - 1) % U;
      if (n > 0 && kt > 0)
        static_for<n>([&](auto IC) { issue(std::integral_constant<int, f + decltype(IC)::value>{}, up, kt - 1 + U); });
    }
    // 3. retire this phase's reads and the slabs the next phase reads; meet the partner group
    if constexpr (ABL == 1) wait_barrier<0>();
    else wait_barrier<S - P::reads(q) - P::reads((q + 1) % NPH)>();
    __builtin_amdgcn_sched_barrier(0);
    // 4. MFMA segment
    if (PRIO == 1) __builtin_amdgcn_s_setprio(1);
    if constexpr (ABL == 2) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < FMP; ++i) asm volatile("" ::"v"(af[kk][a * FMP + i]));
#pragma unroll
        for (int j = 0; j < FNP; ++j) asm volatile("" ::"v"(bf[kk][b * FNP + j]));
      }
    } else
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < FMP; ++i)
#pragma unroll
        for (int j = 0; j < FNP; ++j)
          acc[a * FMP + i][b * FNP + j] =
              mfma16x16x32(bf[kk][b * FNP + j], af[kk][a * FMP + i], acc[a * FMP + i][b * FNP + j]);
    if (PRIO == 1) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto kstep = [&](auto UC, int kt) {
    static_for<NPH>([&](auto QC) { phase(UC, QC, kt); });
  };

  for (int kt = 0; kt < nk; kt += U) {
    kstep(std::integral_constant<int, 0>{}, kt);
    static_for<U - 1>([&](auto IC) {
      constexpr int u = decltype(IC)::value + 1;
      if (kt + u < nk) kstep(std::integral_constant<int, u>{}, kt + u);
    });
  }
  if (PRIO == 2 && wm == 1) __builtin_amdgcn_s_setprio(0);
  __builtin_amdgcn_sched_barrier(0);
  if (wm == 0) __builtin_amdgcn_s_barrier();     // group 0 catches up with group 1's last barrier
  __builtin_amdgcn_sched_barrier(0);
  wait_barrier<0>();                              // the trailing zero-record refills have landed too

  // split-K / stream-K: publish this contribution's fp32 partial (fragment order), take a ticket; the last arriver
  // sums the partials in slot (= K) order (cdna_hip_programming.md "Projection GEMM at M = 256" item 2)
  if (nc > 1) {
    constexpr int NT = 512;
    float* slab = g.ws + (int64_t)tile * maxc * (FM * FN * NT * 4);
    {
      // write-through (sc1) 16-byte stores: the partial reaches memory without an L2 write-back, so the ticket
      // needs no release fence (cdna_hip_programming.md Guideline 16, R1; a release fence here wrote the L2 back
      // and cost ~6 us per partial)
      float* mine = slab + (int64_t)slot * (FM * FN * NT * 4);
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(mine, 0, FM * FN * NT * 16, 0x00020000);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs, ((i * FN + j) * NT + tid) * 16,
                                                 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its write-through stores
    __syncthreads();
    int* flag = reinterpret_cast<int*>(lds + FLAG_OFF);
    if (tid == 0) {
#if !defined(__gfx950__) && !defined(__gfx942__)
      // the fence-free publish relies on gfx94x / gfx950's write-through (sc1) store encoding; any other target
      // releases the partials explicitly
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#endif
      const int ticket = __hip_atomic_fetch_add(g.counters + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = ticket;
      if (ticket == nc - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        g.counters[tile] = 0;
      }
    }
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(flag[0]) != nc - 1) return;
    // the sum in slot order, every partial (this one's included) read back from its slab
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = *reinterpret_cast<const f32x4*>(slab + ((i * FN + j) * NT + tid) * 4);
    for (int s2 = 1; s2 < nc; ++s2) {
      const float* ps = slab + (int64_t)s2 * (FM * FN * NT * 4);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] += *reinterpret_cast<const f32x4*>(ps + ((i * FN + j) * NT + tid) * 4);
    }
  }

  if constexpr (ABL == 3) {                       // timing probe: no epilogue (the accumulators kept live)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  // epilogue: acc[i][j][e] = C[m0 + wm*WTM + i*16 + fr][n0 + wn*WTN + j*16 + 4*fq + e], through an LDS image
  // (fp32 acc + bias rounded once, as the unfused layer rounds), then whole rows, 16 bytes per lane
  constexpr int PITCH = BN * 2 + 16;
  if constexpr (F32EPI) {
    // split-precision epilogues: fp32 bias; RDX_EPI_F32 stores C fp32 from the registers (16 bytes per lane, 64-byte
    // row pieces); RDX_EPI_F32_GELU_SPLIT forms v = gelu(acc + bias) and leaves it as the bf16 pair hi = bf16(v)
    // (C), lo = bf16(v - hi) (aux_out), each through the LDS image and whole-row stores
    const float* biasf = reinterpret_cast<const float*>(g.bias);
    f32x4 bv[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = n0 + wn * WTN + j * 16 + 4 * fq;
      bv[j] = (biasf != nullptr && c < N) ? *reinterpret_cast<const f32x4*>(biasf + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (EPI == RDX_EPI_F32) {
      float* Cf = reinterpret_cast<float*>(g.C) + yb * g.sc;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = m0 + wm * WTM + i * 16 + fr;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int c = n0 + wn * WTN + j * 16 + 4 * fq;
          if (r < M && c < N) *reinterpret_cast<f32x4*>(Cf + (int64_t)r * g.ldc + c) = acc[i][j] + bv[j];
        }
      }
      return;
    } else {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][e] = gelu(acc[i][j][e] + bv[j][e]);
      constexpr int CPR = BN / 8, ITER = BM * CPR / 512;
      static_assert((BM * CPR) % 512 == 0, "row phase");
      char* img = lds;
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
        __syncthreads();                          // the ring (pass 0) / the previous pass's row phase is done
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int r = wm * WTM + i * 16 + fr;
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int c = wn * WTN + j * 16 + 4 * fq;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = pass == 0 ? acc[i][j][e] : acc[i][j][e] - hround(acc[i][j][e]);
            *reinterpret_cast<uint2*>(img + r * PITCH + c * 2) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
          }
        }
        __syncthreads();
        hst* dst = (pass == 0 ? g.C : g.aux_out) + yb * g.sc;
        const int64_t ld = pass == 0 ? g.ldc : g.ldao;
        if (m0 + BM <= M && n0 + BN <= N && g.wide) {
          uint4 qv[ITER];
#pragma unroll
          for (int it = 0; it < ITER; ++it) {
            const int idx = tid + it * 512, r = idx / CPR, c = (idx - r * CPR) * 8;
            qv[it] = *reinterpret_cast<const uint4*>(img + r * PITCH + c * 2);
          }
#pragma unroll
          for (int it = 0; it < ITER; ++it) {
            const int idx = tid + it * 512, r = idx / CPR, c = (idx - r * CPR) * 8;
            *reinterpret_cast<uint4*>(dst + (int64_t)(m0 + r) * ld + n0 + c) = qv[it];
          }
        } else {
          for (int idx = tid; idx < BM * CPR; idx += 512) {
            const int r = idx / CPR, c = (idx - r * CPR) * 8;
            const int m = m0 + r, n = n0 + c;
            if (m >= M || n >= N) continue;
            const uint4 q = *reinterpret_cast<const uint4*>(img + r * PITCH + c * 2);
            hst* o = dst + (int64_t)m * ld + n;
            if (n + 8 <= N && g.wide) {
              *reinterpret_cast<uint4*>(o) = q;
            } else {
              *reinterpret_cast<uint2*>(o) = make_uint2(q.x, q.y);
              if (n + 8 <= N) *reinterpret_cast<uint2*>(o + 4) = make_uint2(q.z, q.w);
            }
          }
        }
      }
      return;
    }
  }
  static_assert(BM * PITCH <= 160 * 1024, "epilogue image");
  char* img = lds;
  uint2 bb[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j)
    bb[j] = has_bias ? *reinterpret_cast<const uint2*>(lds + BIAS_OFF + 2 * (wn * WTN + j * 16 + 4 * fq))
                     : make_uint2(0u, 0u);
  __syncthreads();                                // bias read before the image overwrites nothing (own slot)
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int r = wm * WTM + i * 16 + fr;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = wn * WTN + j * 16 + 4 * fq;
      const float v0 = acc[i][j][0] + hlo(bb[j].x), v1 = acc[i][j][1] + hhi(bb[j].x);
      const float v2 = acc[i][j][2] + hlo(bb[j].y), v3 = acc[i][j][3] + hhi(bb[j].y);
      *reinterpret_cast<uint2*>(img + r * PITCH + c * 2) = make_uint2(pack2(v0, v1), pack2(v2, v3));
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;                     // 16-byte chunks per tile row
  constexpr int ITER = BM * CPR / 512;
  static_assert((BM * CPR) % 512 == 0, "row phase");
  auto gelu8 = [&](uint4 q) -> uint4 {
    const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2(gelu(hlo(qw[e])), gelu(hhi(qw[e])));
    return make_uint4(o[0], o[1], o[2], o[3]);
  };
  auto gelu_bwd8 = [&](uint4 q, uint4 u) -> uint4 {
    const uint32_t qw[4] = {q.x, q.y, q.z, q.w}, uw[4] = {u.x, u.y, u.z, u.w};
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2(hlo(qw[e]) * gelu_grad(hlo(uw[e])), hhi(qw[e]) * gelu_grad(hhi(uw[e])));
    return make_uint4(o[0], o[1], o[2], o[3]);
  };
  if (m0 + BM <= M && n0 + BN <= N && g.wide) {
    // whole tile in range, 16-byte aligned rows: every load issued before any store, no per-element branch
    uint4 qv[ITER], ux[ITER];
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int idx = tid + it * 512, r = idx / CPR, c = (idx - r * CPR) * 8;
      if (EPI == RDX_EPI_GELU_BWD) ux[it] = *reinterpret_cast<const uint4*>(g.aux + yb * g.sc + (int64_t)(m0 + r) * g.ldaux + n0 + c);
      qv[it] = *reinterpret_cast<const uint4*>(img + r * PITCH + c * 2);
    }
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int idx = tid + it * 512, r = idx / CPR, c = (idx - r * CPR) * 8;
      const uint4 q = EPI == RDX_EPI_GELU_BWD ? gelu_bwd8(qv[it], ux[it]) : qv[it];
      *reinterpret_cast<uint4*>(g.C + yb * g.sc + (int64_t)(m0 + r) * g.ldc + n0 + c) = q;
      if (EPI == RDX_EPI_BIAS_GELU) *reinterpret_cast<uint4*>(g.aux_out + yb * g.sc + (int64_t)(m0 + r) * g.ldao + n0 + c) = gelu8(q);
    }
    return;
  }
  // ragged tile or 8-byte rows
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
    uint4 qv = *reinterpret_cast<const uint4*>(img + r * PITCH + c * 2);
    if (EPI == RDX_EPI_GELU_BWD) qv = gelu_bwd8(qv, ld8(g.aux + yb * g.sc + (int64_t)m * g.ldaux + n));
    st8(g.C + yb * g.sc + (int64_t)m * g.ldc + n, qv);
    if (EPI == RDX_EPI_BIAS_GELU) st8(g.aux_out + yb * g.sc + (int64_t)m * g.ldao + n, gelu8(qv));
  }
}

// splits >= 1: work id (XCD-dealt) = tile * splits + split; splits == 0 (stream-K): the grid's workgroups take
// equal contiguous runs of the (tile, K step) units in tile order, a tile shared by several runs summed by the last
// of them to arrive (its partial slots in K order).
template <int BM, int BN, int NPA, int NPB, int U, int EPI, int PRIO, int ABL = 0, int SK = 0, int X3 = 0>
__global__ __launch_bounds__(512, 1) void hgemm_kernel(const Args g) {
  extern __shared__ __attribute__((aligned(1024))) char lds[];
  const int nk_all = (X3 ? 3 : 1) * (g.K / 64);

  const int tiles = g.tiles_m * g.tiles_n;
  if constexpr (SK == 0) {
    const int SPL = g.splits;
    const int t = xcd_remap(blockIdx.x, tiles * SPL);
    int tile = t / SPL, split = t - tile * SPL;
    int mt, nt;
    if (g.group_m < 0) {
      grid_coords(g, t, SPL, mt, nt, split);
      tile = nt * g.tiles_m + mt;     // the tile's id for its split-K slots and ticket (column-panel numbering)
    } else {
      tile_coords(g, tile, mt, nt);
    }
    const int kb = split * nk_all / SPL, nk = (split + 1) * nk_all / SPL - kb;
    run_segment<BM, BN, NPA, NPB, U, EPI, PRIO, ABL, X3>(g, lds, mt, nt, tile, kb, nk, split, SPL, SPL);
    return;
  }
  if (g.splits != 0) return;
  const int G = gridDim.x;
  const int64_t UT = (int64_t)tiles * nk_all;
  const int w = xcd_remap(blockIdx.x, G);
  const int64_t u1 = (int64_t)(w + 1) * UT / G;
  auto owner = [&](int64_t x) { return (int)(((x + 1) * G - 1) / UT); };   // the run holding unit x
  for (int64_t u = (int64_t)w * UT / G; u < u1;) {
    const int tile = (int)(u / nk_all);
    const int kb = (int)(u - (int64_t)tile * nk_all);
    const int ke = (int)min((int64_t)nk_all, kb + (u1 - u));
    const int wf = owner((int64_t)tile * nk_all), wl = owner((int64_t)tile * nk_all + nk_all - 1);
    int mt, nt;
    tile_coords(g, tile, mt, nt);
    run_segment<BM, BN, NPA, NPB, U, EPI, PRIO, ABL>(g, lds, mt, nt, tile, kb, ke - kb, w - wf, wl - wf + 1,
                                                     g.maxc);
    u += ke - kb;
  }
}

template <int BM, int BN, int NPA, int NPB, int U, int EPI, int PRIO, int ABL = 0, int SK = 0, int X3 = 0>
static int launch(Args g, hipStream_t st, int batch = 1) {
  g.tiles_m = (g.M + BM - 1) / BM;
  g.tiles_n = (g.N + BN - 1) / BN;
  constexpr int ring = U * (BM / 64 + BN / 64) * 8192, image = BM * (BN * 2 + 16);
  constexpr int lds = (ring > image ? ring : image) + BN * 2 + 16;   // + the bias slot and the arrival flag
  static_assert(lds <= 160 * 1024, "LDS");
  auto kern = &hgemm_kernel<BM, BN, NPA, NPB, U, EPI, PRIO, ABL, SK, X3>;
  static bool lds_ok = false;
  if (!lds_ok) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int)e;
    lds_ok = true;
  }
  const unsigned grid = g.splits >= 1 ? (unsigned)(g.tiles_m * g.tiles_n * g.splits) : (unsigned)g.grid_sk;
  hipLaunchKernelGGL(kern, dim3(grid, batch), dim3(512), lds, st, g);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

// tile codes (BM x BN, A / B parts, ring K steps); + 100: s_setprio(1) around each MFMA segment; + 200: static
// priority 1 for row group 1
template <int EPI, int PRIO>
static int dispatch(const Args& g, int tile, hipStream_t st, int batch = 1) {
  if (g.splits == 0) {                           // stream-K: the ingest-bound tiles of the N = 1024 shapes
    switch (tile) {
      case 2: return launch<128, 256, 1, 2, 3, EPI, PRIO, 0, 1>(g, st);
      case 3: return launch<128, 192, 2, 1, 3, EPI, PRIO, 0, 1>(g, st);
      case 4: return launch<128, 128, 1, 1, 4, EPI, PRIO, 0, 1>(g, st);
      default: return RDX_EINVAL;
    }
  }
  switch (tile) {
    case 0: return launch<256, 256, 2, 2, 2, EPI, PRIO>(g, st, batch);   // 16 slabs, 128 KB
    case 1: return launch<256, 192, 2, 1, 2, EPI, PRIO>(g, st, batch);   // 14 slabs
    case 2: return launch<128, 256, 1, 2, 3, EPI, PRIO>(g, st, batch);   // 18 slabs
    case 3: return launch<128, 192, 2, 1, 3, EPI, PRIO>(g, st, batch);   // 15 slabs
    case 4: return launch<128, 128, 1, 1, 4, EPI, PRIO>(g, st, batch);   // 16 slabs
    case 5: return launch<256, 128, 2, 1, 3, EPI, PRIO>(g, st, batch);   // 18 slabs
    case 6: return launch<64, 128, 1, 1, 4, EPI, PRIO>(g, st, batch);    // 12 slabs: twice the tiles of 128 x 128
    case 7: return launch<64, 256, 1, 1, 3, EPI, PRIO>(g, st, batch);    // 15 slabs
    default: return RDX_EINVAL;
  }
}

#ifndef RDX_F16
// split-precision (X3) launches: the eval tiles (bf16 planes only)
template <int EPI>
static int dispatch_x3(const Args& g, int tile, int batch, hipStream_t st) {
  switch (tile) {
    case 0: return launch<256, 256, 2, 2, 2, EPI, 0, 0, 0, 1>(g, st, batch);
    case 1: return launch<256, 192, 2, 1, 2, EPI, 0, 0, 0, 1>(g, st, batch);
    case 2: return launch<128, 256, 1, 2, 3, EPI, 0, 0, 0, 1>(g, st, batch);
    case 3: return launch<128, 192, 2, 1, 3, EPI, 0, 0, 0, 1>(g, st, batch);
    case 4: return launch<128, 128, 1, 1, 4, EPI, 0, 0, 0, 1>(g, st, batch);
    case 5: return launch<256, 128, 2, 1, 3, EPI, 0, 0, 0, 1>(g, st, batch);
    default: return RDX_EINVAL;
  }
}
#endif

// timing probes (bias epilogue, wrong results by design): 1000 + tile without refills in the K loop, 2000 + tile
// without MFMA, 3000 + tile without the epilogue
static int dispatch_probe(const Args& g, int code, hipStream_t st) {
  switch (code) {
    case 1000: return launch<256, 256, 2, 2, 2, RDX_EPI_BIAS, 0, 1>(g, st);
    case 1002: return launch<128, 256, 1, 2, 3, RDX_EPI_BIAS, 0, 1>(g, st);
    case 1004: return launch<128, 128, 1, 1, 4, RDX_EPI_BIAS, 0, 1>(g, st);
    case 2000: return launch<256, 256, 2, 2, 2, RDX_EPI_BIAS, 0, 2>(g, st);
    case 2002: return launch<128, 256, 1, 2, 3, RDX_EPI_BIAS, 0, 2>(g, st);
    case 2004: return launch<128, 128, 1, 1, 4, RDX_EPI_BIAS, 0, 2>(g, st);
    case 3000: return launch<256, 256, 2, 2, 2, RDX_EPI_BIAS, 0, 3>(g, st);
    case 3002: return launch<128, 256, 1, 2, 3, RDX_EPI_BIAS, 0, 3>(g, st);
    case 3004: return launch<128, 128, 1, 1, 4, RDX_EPI_BIAS, 0, 3>(g, st);
    default: return RDX_EINVAL;
  }
}

static bool geometry(int tile, int* bm, int* bn) {
  switch (tile % 100) {
    case 0: *bm = 256; *bn = 256; return true;
    case 1: *bm = 256; *bn = 192; return true;
    case 2: *bm = 128; *bn = 256; return true;
    case 3: *bm = 128; *bn = 192; return true;
    case 4: *bm = 128; *bn = 128; return true;
    case 5: *bm = 256; *bn = 128; return true;
    case 6: *bm = 64; *bn = 128; return true;
    case 7: *bm = 64; *bn = 256; return true;
    default: return false;
  }
}

}  // namespace hg
}  // namespace rdx

using namespace rdx;

namespace {
int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) ==
                                                 hipSuccess && v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}
// stream-K geometry: grid (one workgroup per CU, at most one per unit) and the partial slots a tile can need
void sk_geometry(int64_t tiles, int nk_all, int* grid, int* maxc) {
  const int64_t ut = tiles * nk_all;
  const int G = (int)std::min<int64_t>(cu_count(), ut);
  const int64_t per = ut / G;                   // every run holds per or per + 1 units
  int mc = per >= 1 ? (int)((nk_all - 1) / per + 2) : nk_all;
  *grid = G;
  *maxc = std::min(mc, G);
}
}  // namespace

extern "C" int64_t rdx_hgemm_sk_ws_bytes(int M, int N, int K, int tile) {
  int bm, bn;
  if (tile < 0 || tile >= 300 || !hg::geometry(tile, &bm, &bn) || K < 64) return -1;
  const int64_t tiles = (int64_t)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  int grid, maxc;
  sk_geometry(tiles, K / 64, &grid, &maxc);
  return tiles * maxc * (int64_t)bm * bn * 4;
}

extern "C" int64_t rdx_hgemm_ws_bytes(int M, int N, int tile, int splits) {
  int bm, bn;
  if (splits <= 1) return 0;
  if (tile < 0 || tile >= 300 || !hg::geometry(tile, &bm, &bn)) return -1;
  const int64_t tiles = (int64_t)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  return tiles * splits * (int64_t)bm * bn * 4;
}

extern "C" int64_t rdx_hgemm_counters(int M, int N, int tile) {
  int bm, bn;
  if (tile < 0 || tile >= 300 || !hg::geometry(tile, &bm, &bn)) return -1;
  return (int64_t)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
}

extern "C" int rdx_hgemm(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N,
                         int K, const void* bias, int epilogue, const void* aux, int64_t ldaux, void* aux_out,
                         int64_t ldao, int tile, int splits, int group_m, void* ws, int64_t ws_bytes, int* counters,
                         int64_t n_counters, void* stream) {
  auto al = [](const void* p, int a) { return ((uintptr_t)p & (a - 1)) == 0; };
  RDX_REQUIRE(A && B && C && M > 0 && N > 0 && K > 0 && al(A, 16) && al(B, 16) && al(C, 8));
  RDX_REQUIRE(K % 64 == 0 && lda % 8 == 0 && ldb % 8 == 0 && lda >= K && ldb >= K && N % 4 == 0 && ldc >= N &&
              ldc % 4 == 0);
  // 32-bit buffer ranges and source offsets
  RDX_REQUIRE((int64_t)M * lda * 2 < 0x7fffffffLL && (int64_t)N * ldb * 2 < 0x7fffffffLL);
  RDX_REQUIRE(!bias || al(bias, 8));
  RDX_REQUIRE(epilogue == RDX_EPI_BIAS || epilogue == RDX_EPI_BIAS_GELU || epilogue == RDX_EPI_GELU_BWD);
  if (epilogue == RDX_EPI_BIAS_GELU) RDX_REQUIRE(aux_out && ldao >= N && ldao % 4 == 0 && al(aux_out, 8));
  if (epilogue == RDX_EPI_GELU_BWD) RDX_REQUIRE(aux && ldaux >= N && ldaux % 4 == 0 && al(aux, 8));
  int bm, bn;
  const bool probe = tile >= 1000;
  RDX_REQUIRE(probe ? (tile < 4000 && epilogue == RDX_EPI_BIAS && splits == 1)
                    : (tile >= 0 && tile < 300 && hg::geometry(tile, &bm, &bn)));
  RDX_REQUIRE(group_m >= 0 || ((group_m == -1 || group_m == -2 || group_m == -4 || group_m == -8) && splits != 0));
  RDX_REQUIRE(splits >= 0 && splits <= 16 && splits <= K / 64);
  RDX_REQUIRE(splits >= 1 || !probe);
  if (splits != 1) {
    const int64_t need = splits > 1 ? rdx_hgemm_ws_bytes(M, N, tile, splits) : rdx_hgemm_sk_ws_bytes(M, N, K, tile);
    const int64_t nc = rdx_hgemm_counters(M, N, tile);
    RDX_REQUIRE(need > 0 && ws && al(ws, 16) && ws_bytes >= need && counters && n_counters >= nc);
  }
  hg::Args g;
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
  g.splits = splits;
  g.maxc = splits;
  g.grid_sk = 0;
  if (splits == 0) {
    const int64_t tiles = (int64_t)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
    sk_geometry(tiles, K / 64, &g.grid_sk, &g.maxc);
  }
  g.ws = (float*)ws;
  g.counters = counters;
  g.A2 = g.B2 = nullptr;
  g.sa = g.sc = 0;
  g.wide = al(C, 16) && ldc % 8 == 0;
  if (epilogue == RDX_EPI_BIAS_GELU) g.wide = g.wide && al(aux_out, 16) && ldao % 8 == 0;
  if (epilogue == RDX_EPI_GELU_BWD) g.wide = g.wide && al(aux, 16) && ldaux % 8 == 0;
  hipStream_t st = as_stream(stream);
  if (probe) return hg::dispatch_probe(g, tile, st);
  const int prio = tile / 100, base = tile % 100;
  switch (epilogue) {
    case RDX_EPI_BIAS:
      return prio == 0 ? hg::dispatch<RDX_EPI_BIAS, 0>(g, base, st)
           : prio == 1 ? hg::dispatch<RDX_EPI_BIAS, 1>(g, base, st) : hg::dispatch<RDX_EPI_BIAS, 2>(g, base, st);
    case RDX_EPI_BIAS_GELU:
      return prio == 0 ? hg::dispatch<RDX_EPI_BIAS_GELU, 0>(g, base, st)
           : prio == 1 ? hg::dispatch<RDX_EPI_BIAS_GELU, 1>(g, base, st)
                       : hg::dispatch<RDX_EPI_BIAS_GELU, 2>(g, base, st);
    default:
      return prio == 0 ? hg::dispatch<RDX_EPI_GELU_BWD, 0>(g, base, st)
           : prio == 1 ? hg::dispatch<RDX_EPI_GELU_BWD, 1>(g, base, st)
                       : hg::dispatch<RDX_EPI_GELU_BWD, 2>(g, base, st);
  }
}

extern "C" int rdx_hgemm_x3(const void* A, const void* A_lo, int64_t lda, int64_t sa, const void* B, const void* B_lo,
                            int64_t ldb, void* C, void* C_lo, int64_t ldc, int64_t sc, int M, int N, int K, int batch,
                            const float* bias, int epilogue, int tile, int splits, int group_m, void* ws,
                            int64_t ws_bytes, int* counters, int64_t n_counters, void* stream) {
#ifdef RDX_F16
  (void)A; (void)A_lo; (void)lda; (void)sa; (void)B; (void)B_lo; (void)ldb; (void)C; (void)C_lo; (void)ldc; (void)sc;
  (void)M; (void)N; (void)K; (void)batch; (void)bias; (void)epilogue; (void)tile; (void)splits; (void)group_m;
  (void)ws; (void)ws_bytes; (void)counters; (void)n_counters; (void)stream;
  return RDX_EINVAL;                              // bf16 planes only (libradhip.so)
#else
  auto al = [](const void* p, int a) { return ((uintptr_t)p & (a - 1)) == 0; };
  RDX_REQUIRE(A && A_lo && B && B_lo && C && M > 0 && N > 0 && K > 0 && batch >= 1);
  RDX_REQUIRE(al(A, 16) && al(A_lo, 16) && al(B, 16) && al(B_lo, 16) && al(C, 16));
  // A rows may overlap (lda < K: a strided convolution's im2col rows, never materialised)
  RDX_REQUIRE(K % 64 == 0 && lda % 8 == 0 && ldb % 8 == 0 && lda > 0 && ldb >= K && N % 4 == 0 && ldc >= N);
  RDX_REQUIRE(((int64_t)(M - 1) * lda + K) * 2 < 0x7fffffffLL && (int64_t)N * ldb * 2 < 0x7fffffffLL);
  RDX_REQUIRE(batch == 1 || (sa % 8 == 0 && sc % 8 == 0 && sa >= 0 && sc >= 0 && splits == 1));
  RDX_REQUIRE(!bias || al(bias, 16));
  RDX_REQUIRE(epilogue == RDX_EPI_F32 || epilogue == RDX_EPI_F32_GELU_SPLIT);
  if (epilogue == RDX_EPI_F32) RDX_REQUIRE(ldc % 4 == 0);
  else RDX_REQUIRE(C_lo && al(C_lo, 16) && ldc % 8 == 0);
  int bm, bn;
  RDX_REQUIRE(tile >= 0 && tile <= 5 && hg::geometry(tile, &bm, &bn));
  RDX_REQUIRE(group_m >= 0 || ((group_m == -1 || group_m == -2 || group_m == -4 || group_m == -8) && splits != 0));
  RDX_REQUIRE(splits >= 1 && splits <= 16 && splits <= 3 * (K / 64));
  if (splits > 1) {
    const int64_t need = rdx_hgemm_ws_bytes(M, N, tile, splits);
    const int64_t nc = rdx_hgemm_counters(M, N, tile);
    RDX_REQUIRE(need > 0 && ws && al(ws, 16) && ws_bytes >= need && counters && n_counters >= nc);
  }
  hg::Args g;
  g.A = (const hst*)A;
  g.A2 = (const hst*)A_lo;
  g.lda = lda;
  g.B = (const hst*)B;
  g.B2 = (const hst*)B_lo;
  g.ldb = ldb;
  g.C = (hst*)C;
  g.ldc = ldc;
  g.M = M;
  g.N = N;
  g.K = K;
  g.bias = (const hst*)bias;                      // fp32 [N], read as such by the F32 epilogues
  g.aux = nullptr;
  g.ldaux = 0;
  g.aux_out = (hst*)C_lo;
  g.ldao = ldc;
  g.tiles_m = g.tiles_n = 0;
  g.group_m = group_m;
  g.splits = splits;
  g.maxc = splits;
  g.grid_sk = 0;
  g.ws = (float*)ws;
  g.counters = counters;
  g.sa = sa;
  g.sc = sc;
  g.wide = ldc % 8 == 0 && (batch == 1 || sc % 8 == 0);
  hipStream_t st = as_stream(stream);
  return epilogue == RDX_EPI_F32 ? hg::dispatch_x3<RDX_EPI_F32>(g, tile, batch, st)
                                 : hg::dispatch_x3<RDX_EPI_F32_GELU_SPLIT>(g, tile, batch, st);
#endif
}

// Batched 16-bit form: `batch` problems C_y = A_y . B^T (+ bias) in one launch (blockIdx.y), A_y = A + y sa with rows
// that may overlap (lda < K: the token-major input of a strided convolution read as its im2col matrix), C_y = C + y sc.
// The frozen WavLM CNN's layers 1-6 (csrc/featconv.hip's token-major layout) run here.
extern "C" int rdx_hgemm_batched(const void* A, int64_t lda, int64_t sa, const void* B, int64_t ldb, void* C,
                                 int64_t ldc, int64_t sc, int M, int N, int K, int batch, const void* bias, int tile,
                                 int group_m, void* stream) {
  auto al = [](const void* p, int a) { return ((uintptr_t)p & (a - 1)) == 0; };
  RDX_REQUIRE(A && B && C && M > 0 && N > 0 && K > 0 && batch >= 1 && batch <= 65535);
  RDX_REQUIRE(al(A, 16) && al(B, 16) && al(C, 8) && (!bias || al(bias, 8)));
  RDX_REQUIRE(K % 64 == 0 && lda % 8 == 0 && ldb % 8 == 0 && lda > 0 && ldb >= K && N % 4 == 0 && ldc >= N &&
              ldc % 4 == 0 && sa >= 0 && sa % 8 == 0 && sc >= 0 && sc % 4 == 0);
  RDX_REQUIRE(((int64_t)(M - 1) * lda + K) * 2 < 0x7fffffffLL && (int64_t)N * ldb * 2 < 0x7fffffffLL);
  RDX_REQUIRE(batch == 1 || (sc >= (int64_t)(M - 1) * ldc + N));    // the problems' outputs do not overlap
  int bm, bn;
  RDX_REQUIRE(tile >= 0 && tile < 8 && hg::geometry(tile, &bm, &bn));
  RDX_REQUIRE(group_m >= 0);
  hg::Args g;
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
  g.aux = nullptr;
  g.ldaux = 0;
  g.aux_out = nullptr;
  g.ldao = 0;
  g.tiles_m = g.tiles_n = 0;
  g.group_m = group_m;
  g.splits = 1;
  g.maxc = 1;
  g.grid_sk = 0;
  g.ws = nullptr;
  g.counters = nullptr;
  g.A2 = g.B2 = nullptr;
  g.sa = sa;
  g.sc = sc;
  g.wide = al(C, 16) && ldc % 8 == 0 && sc % 8 == 0;
  return hg::dispatch<RDX_EPI_BIAS, 0>(g, tile, as_stream(stream), batch);
}
