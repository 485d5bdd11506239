// WavLM self-attention with the gated relative-position bias, fused, on gfx950 MFMA (bf16 in, fp32
// accumulate), forward and backward.
//
// Reference: HF WavLMAttention (transformers modeling_wavlm.py) as used by WavLMFrontend
// (src/models/DualStreamSEMamba.py:292-439): per head h
//     bias[b,h,i,j] = gate[b,i,h] * pb[h,i,j]      (gated rel-pos bias; gate depends on the layer input)
//     P = softmax(Q K^T / sqrt(64) + bias),  O = dropout(P) V
// The [B,H,T,T] bias is never materialised: it is formed in registers from gate and the shared
// position bias pb, and the backward returns d gate = sum_j dS[i,j] pb[h,i,j] directly (pb comes from
// the frozen rel_attn_embed table). Dropout keeps element (b,h,i,j) iff a counter hash of
// (seed, index) >= p * 2^32, so the backward regenerates the same mask; the seed is read from device
// memory, which keeps the launch replayable inside a HIP graph.
//
// Structure (T <= 256, i.e. at most 8 tiles of 32 rows; the WavLM stream at 64 600 samples has T = 201).
// A workgroup is 4 waves of one (b, h). It first stages the whole sequence of the two operands it sweeps
// into LDS images (K and V for the query-stationary forward and dQ kernels, Q and dO for the
// key-stationary dK/dV kernel); then each wave owns one 32-row tile and loops over every tile of the other
// side with no barrier and no global load but the position-bias row. MFMA is mfma_f32_32x32x16_bf16
// (A: lane (r, h) holds A[r][8h + j]; B: B[8h + j][r]; C: col = lane & 31, row = (i & 3) + 8 (i >> 2) + 4h).
// A fragment that runs along a row of an image is one 16-byte ds_read; a fragment that runs down a column
// (V^T, K^T, Q^T, dO^T in the k order of an accumulator fed back as an operand) is two
// ds_read_b64_tr_b16 hardware-transposed reads. The images use 8-row x 32-column subtiles with the 16-byte
// chunk XOR-swizzled by (row >> 2) & 3, which keeps both kinds of read conflict-free with no padding.
//   forward  S^T = K Q^T (query on the lane), online softmax over the key tiles, O^T += V^T P^T.
//   dQ       query-stationary; also writes D = rowsum(dO o O) for its rows. S^T and dP^T = V dO^T as the
//            forward, dQ^T += K^T dS^T; d gate is a lane-local sum plus one cross-half exchange.
//   dK, dV   key-stationary: S = Q K^T, dP = dO V^T (query rows from the images), dV += P^T dO and
//            dK += dS^T Q; gate, lse and D of every query row are staged in LDS with Q and dO.
#include "common.h"

namespace rdx {

typedef __attribute__((ext_vector_type(16))) float f32x16;
constexpr int AT_DH = 64;                  // head dim
constexpr int AT_TILE = 32;                // rows per wave
constexpr int AT_MAXNT = 8;                // tiles per sequence: T <= 256
constexpr int AT_WAVES = 4;                // waves (tiles) per workgroup
constexpr int AT_TILE_BYTES = AT_TILE * AT_DH * 2;  // one 32-row tile of an image: 4 KB
constexpr float kLog2e = 1.4426950408889634f;

// Diagnostic build only (tools/attn_probe.cpp defines RDX_ATTN_PROBE): per-wave s_memtime stamps at phase
// boundaries into a buffer of their own; no output value depends on them. Empty in the library.
#ifdef RDX_ATTN_PROBE
__device__ uint64_t rdx_probe[1 << 16];
#define RDX_PROBE(k)                                                                                          \
  do {                                                                                                        \
    if ((threadIdx.x & 63) == 0)                                                                              \
      rdx_probe[((size_t)blockIdx.x * 8 + (threadIdx.x >> 6)) * 8 + (k)] = __builtin_amdgcn_s_memtime();      \
  } while (0)
#else
#define RDX_PROBE(k) \
  do {              \
  } while (0)
#endif

__device__ __forceinline__ f32x16 mfma32(hx8 a, hx8 b, f32x16 c) {
  return mfma32x32x16(a, b, c);
}
// C/D row held in accumulator register i by lane half h
__device__ __forceinline__ int crow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

__device__ __forceinline__ hx8 pack8(const float* x) {
  hx8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (hel)x[j];
  return r;
}
__device__ __forceinline__ hx8 load8(const hst* p, bool ok) {
  if (!ok) {
    hx8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = (hel)0.f;
    return z;
  }
  return *reinterpret_cast<const hx8*>(p);
}
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// Relative-position bias. WavLM's bias of (query i, key j) depends on j - i only (bucketed relative
// position, compute_bias), so the kernels take it as a table rel[h][j - i + T - 1] of 2T - 1 values per
// head and stage the head's row in LDS, padded so that every (row, column) of the 32-padded tiles indexes
// inside it: tab[j - i + (T - 1) + pad] with pad = tp - T, 2 tp entries, zeros outside |j - i| < T.
__device__ __forceinline__ int rel_tab_bytes(int tp) { return 2 * tp * 4; }
__device__ __forceinline__ void stage_rel(float* tab, const float* rel, int head, int T, int tp) {
  const int pad = tp - T;
  for (int i = threadIdx.x; i < 2 * tp; i += blockDim.x) {
    const int d = i - pad - (T - 1);
    tab[i] = (d > -T && d < T) ? rel[(int64_t)head * (2 * T - 1) + d + T - 1] : 0.f;
  }
}
// query on the lane (row q), keys kb*32 + crow(i, hh): v[i] = bias(q, key)
__device__ __forceinline__ void rel16_q(const float* tab, int q, int T, int tp, int kb, int hh, float* v) {
  const float* t = tab + (tp - T) + (T - 1) - q + kb * AT_TILE;
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = t[crow(i, hh)];
}
// key on the lane, query rows qb*32 + crow(i, hh): v[i] = bias(query, key)
__device__ __forceinline__ void rel16_k(const float* tab, int key, int T, int tp, int qb, int hh, float* v) {
  const float* t = tab + (tp - T) + (T - 1) + key - qb * AT_TILE;
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = t[-crow(i, hh)];
}

// Byte offset of 16-byte chunk ch (0..7, columns 8 ch .. 8 ch + 7) of image row `row`: 8-row x 32-column
// subtiles of 512 B, chunk XOR-swizzled by (row >> 2) & 3 (MI355X guide T10, layout (a), on 64-column rows).
__device__ __forceinline__ int img_off(int row, int ch) {
  return 1024 * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}

// rows [0, 32 nt) of the head slice (columns col0 .. col0 + 63) of a [B, T, ld] bf16 tensor into an LDS
// image; rows past T are zero. Every thread of the workgroup takes part.
__device__ __forceinline__ void stage_image(char* img, const hst* src, int64_t ld, int b, int T,
                                            int64_t col0, int nt, int nthreads = AT_WAVES * 64) {
  for (int i = threadIdx.x; i < nt * AT_TILE * 8; i += nthreads) {
    const int row = i >> 3, ch = i & 7;
    *reinterpret_cast<hx8*>(img + img_off(row, ch)) =
        load8(src + ((int64_t)b * T + row) * ld + col0 + 8 * ch, row < T);
  }
}
// fragment along a row: element j = X[row][16 s + 8 h + j]
__device__ __forceinline__ hx8 read_row(const char* img, int row, int s, int h) {
  return *reinterpret_cast<const hx8*>(img + img_off(row, 2 * s + h));
}
// fragment down a column in the k order of an accumulator fed back as an operand:
//   element j = X[r0 + 16 s + 8 (j >> 2) + 4 h + (j & 3)][c0 + (lane & 31)].
// Each ds_read_b64_tr_b16 gives 16-lane group g the 4 x 16 block at rows r0 + 16 s + 4 (g >> 1) (+ 8 for
// elements 4..7), columns c0 + 16 (g & 1) .. + 15, column-major (lane i of the group gets column i, row q in
// element q); lane 4q + p of the group supplies the address of row q, columns 4p .. 4p + 3.
__device__ __forceinline__ hx8 read_tr(char* img, int r0, int c0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int row = r0 + 16 * s + 4 * (g >> 1) + (i >> 2);
  const int col = c0 + 16 * (g & 1) + 4 * (i & 3);
  const int sub = 2 * (col & 7);  // 0 or 8 bytes into the chunk
  const hx4v lo = ds_tr4((img + img_off(row, col >> 3) + sub));
  const hx4v hi =
      ds_tr4((img + img_off(row + 8, col >> 3) + sub));
  hx8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = lo[j];
    r[4 + j] = hi[j];
  }
  return r;
}

struct AttnArgs {
  const hst *q, *k, *v;
  int64_t ldq, ldk, ldv;
  const float* gate;  // [B, T, H]
  const float* rel;   // [H, 2T - 1] relative-position bias table
  const int64_t* seed_dev;
  int salt;
  uint32_t thr;   // p * 2^16, the 16-bit threshold of the paired hash (0: no dropout)
  float inv_keep;  // 1 / (1 - p)
  float scale;
  int B, T, H;
};

struct AttnBwdArgs {
  const hst* dO;
  int64_t lddo;
  const float* lse;  // [B, H, T]
  float* D;          // [B, H, T]: written by the dQ kernel, read by the dK/dV kernel
};

// Keep factors of the 16 scores a lane holds in the query-on-lane layout (keys kb*32 + crow(i, hh) of
// row `row`): keys crow(i) and crow(i) + 1 (i even) form one hash pair. Returns the 16 keep bits.
template <bool kIdx32>
__device__ __forceinline__ uint32_t row_keep16(uint64_t seed, DropKey32 k32, uint64_t prow, int kb, int hh,
                                               uint32_t thr, float inv_keep, float* mk) {
  uint32_t bits = 0;
#pragma unroll
  for (int i = 0; i < 16; i += 2) {
    const uint64_t pid = prow + (uint64_t)((kb * AT_TILE + crow(i, hh)) >> 1);
    const uint32_t h = kIdx32 ? pair_hash32(k32, (uint32_t)pid) : pair_hash(seed, pid);
    const bool k0 = half_keep(h, false, thr), k1 = half_keep(h, true, thr);
    mk[i] = k0 ? inv_keep : 0.f;
    mk[i + 1] = k1 ? inv_keep : 0.f;
    bits |= ((uint32_t)k0 << i) | ((uint32_t)k1 << (i + 1));
  }
  return bits;
}

// mask word layout shared by the forward (writer) and the fused backward (reader): word (bh, kb, q) holds
// the keep bits of query q for the 32 keys of tile kb, bit i + 16 hh = key kb*32 + crow(i, hh)
__device__ __forceinline__ int64_t mask_word(int64_t bh, int nt, int tp, int kb, int q) {
  return (bh * nt + kb) * tp + q;
}

// Forward: a workgroup owns AT_WAVES query tiles of one (b, h), one wave per query tile sweeping every key tile.
// kSplit (small batches, where the grid would leave most SIMDs with one wave): 8 waves, the two waves of a query
// tile split its key tiles (the first takes ceil(nt / 2), the second the rest), each with its own online-softmax
// state (m, l, O^T), and the second hands its state to the first through LDS for the merge: 2 waves per SIMD at
// the same K / V staging (B = 8: 14.0 -> 11.7 us; at B = 32 the unsplit kernel is faster, 42 vs 48 us).
constexpr int AT_MERGE_STRIDE = 2 * 16 + 2;   // floats per lane: O^T (2 x 16), m, l
template <bool kSplit>
constexpr int at_fwd_threads() { return (kSplit ? 2 : 1) * AT_WAVES * 64; }
template <bool kDrop, bool kIdx32, bool kSplit>
__global__ __launch_bounds__(at_fwd_threads<kSplit>()) void attn_fwd_kernel(AttnArgs a, hst* __restrict__ o,
                                                                 int64_t ldo, float* __restrict__ lse,
                                                                 uint32_t* __restrict__ mask) {
  extern __shared__ __attribute__((aligned(16))) char at_lds[];
  const int T = a.T, H = a.H, nt = (T + AT_TILE - 1) / AT_TILE, tp = nt * AT_TILE;
  const int head = blockIdx.y, b = blockIdx.z;
  const int64_t col0 = (int64_t)head * AT_DH;
  // images sized for AT_MAXNT tiles whatever T (the host allocates at_fwd_lds): every staged chunk has a slot, so the
  // stores below are unconditional and the compiler keeps all the loads ahead of the first wait
  char* Ks = at_lds;
  char* Vs = at_lds + AT_MAXNT * AT_TILE_BYTES;
  float* tab = reinterpret_cast<float*>(at_lds + 2 * AT_MAXNT * AT_TILE_BYTES);
  float* mrg = tab + 2 * AT_MAXNT * AT_TILE;  // [AT_WAVES][64][AT_MERGE_STRIDE]
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int qw = w % AT_WAVES, half = w / AT_WAVES;
  const int qb = blockIdx.x * AT_WAVES + qw;
  const bool active = qb < nt;                // no early return: the merge below has a barrier
  const int kmid = kSplit ? (nt + 1) >> 1 : nt;
  const int kb0 = half ? kmid : 0, kb1 = half ? nt : kmid;
  const int qi = qb * AT_TILE + r;
  const bool qvalid = active && qi < T;
  const int qc = qvalid ? qi : T - 1;
  // Every global load of the workgroup in flight at once before the first wait: the K / V images (PER 16-byte
  // chunks of each per thread, from row-clamped addresses, zeroed past T), the relative-bias row, this lane's Q
  // fragments and gate. A staging loop that stored each chunk as it arrived waited out one load round trip per
  // iteration (7 at T = 201 with 512 threads, 14 with 256).
  constexpr int NTHR = at_fwd_threads<kSplit>();
  constexpr int PER = AT_MAXNT * AT_TILE * 8 / NTHR;
  hx8 kc[PER], vc[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = threadIdx.x + j * NTHR, row = i >> 3, ch = i & 7;
    const int64_t o = (int64_t)b * T + (row < T ? row : T - 1);
    kc[j] = *reinterpret_cast<const hx8*>(a.k + o * a.ldk + col0 + 8 * ch);
    vc[j] = *reinterpret_cast<const hx8*>(a.v + o * a.ldv + col0 + 8 * ch);
  }
  constexpr int TPER = (2 * AT_MAXNT * AT_TILE + NTHR - 1) / NTHR;
  float tv[TPER];
  {
    const int pad = tp - T;
#pragma unroll
    for (int j = 0; j < TPER; ++j) {
      const int i = threadIdx.x + j * NTHR, d = i - pad - (T - 1);
      const int dc = d > -T ? (d < T ? d : T - 1) : 1 - T;
      tv[j] = a.rel[(int64_t)head * (2 * T - 1) + dc + T - 1];
      tv[j] = (d > -T && d < T) ? tv[j] : 0.f;
    }
  }
  hx8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const hx8*>(a.q + ((int64_t)b * T + qc) * a.ldq + col0 + 16 * s + 8 * hh);
  const float graw = a.gate[((int64_t)b * T + qc) * H + head];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = threadIdx.x + j * NTHR, row = i >> 3, ch = i & 7;
    hx8 kv = kc[j], vv = vc[j];
    const bool z = row >= T;   // rows past T read as zeros
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      kv[e] = z ? (hel)0.f : kv[e];
      vv[e] = z ? (hel)0.f : vv[e];
    }
    *reinterpret_cast<hx8*>(Ks + img_off(row, ch)) = kv;
    *reinterpret_cast<hx8*>(Vs + img_off(row, ch)) = vv;
  }
#pragma unroll
  for (int j = 0; j < TPER; ++j) {
    const int i = threadIdx.x + j * NTHR;
    if (TPER * NTHR == 2 * AT_MAXNT * AT_TILE || i < 2 * AT_MAXNT * AT_TILE) tab[i] = tv[j];
  }
  __syncthreads();
  float m = -INFINITY, l = 0.f;
  f32x16 oacc[2] = {zero16(), zero16()};
  const int64_t bh = (int64_t)b * H + head;
  if (active) {
    if (!qvalid) {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) qf[s][e] = (hel)0.f;
    }
    const float g2 = graw * kLog2e;   // base-2 domain: exp2 of log2e-scaled scores
    const float scale2 = a.scale * kLog2e;
    const uint64_t seed = kDrop ? attn_seed(a.seed_dev, a.salt) : 0;
    const DropKey32 k32 = drop_key32(seed);
    const uint64_t prow = ((uint64_t)bh * T + qc) * (uint64_t)((T + 1) >> 1);
    for (int kb = kb0; kb < kb1; ++kb) {
      float sv[16], pbv[16];
      rel16_q(tab, qc, T, tp, kb, hh, pbv);
      f32x16 sacc = zero16();
#pragma unroll
      for (int s = 0; s < 4; ++s) sacc = mfma32(read_row(Ks, kb * AT_TILE + r, s, hh), qf[s], sacc);
      float mloc = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = kb * AT_TILE + crow(i, hh);
        const float x = fmaf(sacc[i], scale2, g2 * pbv[i]);
        sv[i] = key < T ? x : -INFINITY;
        mloc = fmaxf(mloc, sv[i]);
      }
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      const float mnew = fmaxf(m, mloc);  // finite: every tile holds at least one key < T
      const float alpha = __builtin_amdgcn_exp2f(m - mnew);
      float mk[16];
      if (kDrop) {
        const uint32_t bits = row_keep16<kIdx32>(seed, k32, prow, kb, hh, a.thr, a.inv_keep, mk);
        if (mask) {
          const uint32_t other = (uint32_t)__shfl_xor((int)bits, 32, 64);
          if (hh == 0) mask[mask_word(bh, nt, tp, kb, qi)] = bits | (other << 16);
        }
      }
      float lsum = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = __builtin_amdgcn_exp2f(sv[i] - mnew);  // exp2(-inf) = 0 for keys past T
        lsum += p;
        sv[i] = kDrop ? p * mk[i] : p;
      }
      lsum += __shfl_xor(lsum, 32, 64);
      l = l * alpha + lsum;
      m = mnew;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        oacc[0][i] *= alpha;
        oacc[1][i] *= alpha;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const hx8 pf = pack8(sv + 8 * s);
#pragma unroll
        for (int db = 0; db < 2; ++db) oacc[db] = mfma32(read_tr(Vs, kb * AT_TILE, db * 32, s, lane), pf, oacc[db]);
      }
    }
  }
  // merge the key halves: the second wave of the tile hands (O^T, m, l) to the first
  float* slot = mrg + ((size_t)qw * 64 + lane) * AT_MERGE_STRIDE;
  if constexpr (kSplit) {
  if (half == 1 && active) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      slot[i] = oacc[0][i];
      slot[16 + i] = oacc[1][i];
    }
    slot[32] = m;
    slot[33] = l;
  }
  __syncthreads();
  if (half == 1 || !active) return;
  {
    const float m2 = slot[32], l2 = slot[33];
    const float mn = fmaxf(m, m2);            // finite: the first half holds at least one key < T
    const float a1 = __builtin_amdgcn_exp2f(m - mn), a2 = __builtin_amdgcn_exp2f(m2 - mn);  // a2 = 0: empty half
    l = l * a1 + l2 * a2;
    m = mn;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      oacc[0][i] = oacc[0][i] * a1 + slot[i] * a2;
      oacc[1][i] = oacc[1][i] * a1 + slot[16 + i] * a2;
    }
  }
  }
  if (qvalid) {
    const float inv = 1.f / l;
    hst* orow = o + ((int64_t)b * T + qi) * ldo + col0;
    // registers 4k .. 4k + 3 hold the 4 consecutive columns crow(4k, hh) .. + 3 of the lane's row: one 8-byte store
    // each (ldo and col0 keep them 8-byte aligned: rdx_attn_fwd requires ldo % 4 == 0)
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        *reinterpret_cast<uint2*>(orow + db * 32 + crow(4 * k4, hh)) =
            make_uint2(hpack2(oacc[db][4 * k4] * inv, oacc[db][4 * k4 + 1] * inv),
                       hpack2(oacc[db][4 * k4 + 2] * inv, oacc[db][4 * k4 + 3] * inv));
      }
    if (hh == 0) lse[bh * T + qi] = (m + __log2f(l)) * 0.69314718055994531f;  // natural-log LSE
  }
}

// query-stationary: dQ, d gate and D = rowsum(dO o O) of the wave's 32 query rows
template <bool kDrop>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnArgs a, AttnBwdArgs g,
                                                          const hst* __restrict__ O, int64_t ldo,
                                                          hst* __restrict__ dq, int64_t ldg,
                                                          float* __restrict__ dgate) {
  extern __shared__ __attribute__((aligned(16))) char at_lds[];
  const int T = a.T, H = a.H, nt = (T + AT_TILE - 1) / AT_TILE;
  const int head = blockIdx.y, b = blockIdx.z;
  const int64_t col0 = (int64_t)head * AT_DH;
  char* Ks = at_lds;
  char* Vs = at_lds + nt * AT_TILE_BYTES;
  float* tab = reinterpret_cast<float*>(at_lds + 2 * nt * AT_TILE_BYTES);
  stage_image(Ks, a.k, a.ldk, b, T, col0, nt);
  stage_image(Vs, a.v, a.ldv, b, T, col0, nt);
  stage_rel(tab, a.rel, head, T, nt * AT_TILE);
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int qb = blockIdx.x * AT_WAVES + w;
  if (qb >= nt) return;
  const int qi = qb * AT_TILE + r;
  const bool qvalid = qi < T;
  const int qc = qvalid ? qi : T - 1;
  const int64_t trow = (int64_t)b * T + qc;
  hx8 qf[4], dof[4];
  float dpart = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = load8(a.q + trow * a.ldq + col0 + 16 * s + 8 * hh, qvalid);
    dof[s] = load8(g.dO + trow * g.lddo + col0 + 16 * s + 8 * hh, qvalid);
    const hx8 of = load8(O + trow * ldo + col0 + 16 * s + 8 * hh, qvalid);
#pragma unroll
    for (int j = 0; j < 8; ++j) dpart = fmaf((float)dof[s][j], (float)of[j], dpart);
  }
  const float Dq = dpart + __shfl_xor(dpart, 32, 64);
  const int64_t bh = (int64_t)b * H + head;
  if (hh == 0 && qvalid) g.D[bh * T + qi] = Dq;
  const float gq = a.gate[trow * H + head];
  const float lq = g.lse[bh * T + qc];
  const uint64_t seed = kDrop ? attn_seed(a.seed_dev, a.salt) : 0;
  const uint64_t prow = ((uint64_t)bh * T + qc) * (uint64_t)((T + 1) >> 1);
  f32x16 dqacc[2] = {zero16(), zero16()};
  float dg = 0.f;
  for (int kb = 0; kb < nt; ++kb) {
    f32x16 S = zero16(), dP = zero16();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      S = mfma32(read_row(Ks, kb * AT_TILE + r, s, hh), qf[s], S);
      dP = mfma32(read_row(Vs, kb * AT_TILE + r, s, hh), dof[s], dP);
    }
    float dS[16], pbt[16], mk[16];
    rel16_q(tab, qc, T, nt * AT_TILE, kb, hh, pbt);
    if (kDrop) row_keep16<false>(seed, drop_key32(seed), prow, kb, hh, a.thr, a.inv_keep, mk);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = kb * AT_TILE + crow(i, hh);
      float ds = 0.f;
      if (key < T && qvalid) {
        const float p = __expf(fmaf(S[i], a.scale, gq * pbt[i]) - lq);
        ds = p * (dP[i] * (kDrop ? mk[i] : 1.f) - Dq);
        dg = fmaf(ds, pbt[i], dg);
      }
      dS[i] = ds;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const hx8 xs = pack8(dS + 8 * s);
#pragma unroll
      for (int db = 0; db < 2; ++db) dqacc[db] = mfma32(read_tr(Ks, kb * AT_TILE, db * 32, s, lane), xs, dqacc[db]);
    }
  }
  dg += __shfl_xor(dg, 32, 64);
  if (qvalid) {
    hst* row = dq + ((int64_t)b * T + qi) * ldg + col0;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int i = 0; i < 16; ++i) row[db * 32 + crow(i, hh)] = f2h(dqacc[db][i] * a.scale);
    if (hh == 0) dgate[((int64_t)b * T + qi) * H + head] = dg;
  }
}

// key-stationary: dK and dV of the wave's 32 keys
template <bool kDrop>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(AttnArgs a, AttnBwdArgs g,
                                                            hst* __restrict__ dk,
                                                            hst* __restrict__ dv, int64_t ldg) {
  extern __shared__ __attribute__((aligned(16))) char at_lds[];
  const int T = a.T, H = a.H, nt = (T + AT_TILE - 1) / AT_TILE, tp = nt * AT_TILE;
  const int head = blockIdx.y, b = blockIdx.z;
  const int64_t col0 = (int64_t)head * AT_DH;
  const int64_t bh = (int64_t)b * H + head;
  char* Qs = at_lds;
  char* dOs = at_lds + nt * AT_TILE_BYTES;
  float* s_gate = reinterpret_cast<float*>(at_lds + 2 * nt * AT_TILE_BYTES);  // [tp] gate, then lse, then D
  float* s_lse = s_gate + tp;
  float* s_D = s_lse + tp;
  float* tab = s_D + tp;
  stage_image(Qs, a.q, a.ldq, b, T, col0, nt);
  stage_image(dOs, g.dO, g.lddo, b, T, col0, nt);
  stage_rel(tab, a.rel, head, T, tp);
  for (int i = threadIdx.x; i < tp; i += AT_WAVES * 64) {
    const bool ok = i < T;
    s_gate[i] = ok ? a.gate[((int64_t)b * T + i) * H + head] : 0.f;
    s_lse[i] = ok ? g.lse[bh * T + i] : 0.f;
    s_D[i] = ok ? g.D[bh * T + i] : 0.f;
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int kb = blockIdx.x * AT_WAVES + w;
  if (kb >= nt) return;
  const int key = kb * AT_TILE + r;  // this lane's key column
  const bool kvalid = key < T;
  hx8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = load8(a.k + ((int64_t)b * T + key) * a.ldk + col0 + 16 * s + 8 * hh, kvalid);
    vf[s] = load8(a.v + ((int64_t)b * T + key) * a.ldv + col0 + 16 * s + 8 * hh, kvalid);
  }
  const uint64_t seed = kDrop ? attn_seed(a.seed_dev, a.salt) : 0;
  const float* tcol = tab + (tp - T) + (T - 1) + key;  // bias(q, key) = tcol[-q]
  f32x16 dkacc[2] = {zero16(), zero16()}, dvacc[2] = {zero16(), zero16()};
  for (int qb = 0; qb < nt; ++qb) {
    f32x16 S = zero16(), dP = zero16();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      S = mfma32(read_row(Qs, qb * AT_TILE + r, s, hh), kf[s], S);
      dP = mfma32(read_row(dOs, qb * AT_TILE + r, s, hh), vf[s], dP);
    }
    float P[16], dS[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int q0 = qb * AT_TILE + 8 * c + 4 * hh;  // rows crow(4c + e, hh) = q0 + e
      const float4 g4 = *reinterpret_cast<const float4*>(s_gate + q0);
      const float4 l4 = *reinterpret_cast<const float4*>(s_lse + q0);
      const float4 d4 = *reinterpret_cast<const float4*>(s_D + q0);
      const float gv[4] = {g4.x, g4.y, g4.z, g4.w}, lv[4] = {l4.x, l4.y, l4.z, l4.w};
      const float dd[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * c + e, qi = q0 + e;
        float p = 0.f, ds = 0.f;
        if (qi < T && kvalid) {
          const float sc = fmaf(S[i], a.scale, gv[e] * tcol[-qi]);
          p = __expf(sc - lv[e]);
          float mk = 1.f;
          if (kDrop) {
            const uint32_t hsh = pair_hash(seed, ((uint64_t)bh * T + qi) * (uint64_t)((T + 1) >> 1) + (key >> 1));
            mk = half_keep(hsh, key & 1, a.thr) ? a.inv_keep : 0.f;
          }
          ds = p * (dP[i] * mk - dd[e]);
          p *= mk;
        }
        P[i] = p;
        dS[i] = ds;
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const hx8 xp = pack8(P + 8 * s), xs = pack8(dS + 8 * s);
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        dvacc[db] = mfma32(xp, read_tr(dOs, qb * AT_TILE, db * 32, s, lane), dvacc[db]);
        dkacc[db] = mfma32(xs, read_tr(Qs, qb * AT_TILE, db * 32, s, lane), dkacc[db]);
      }
    }
  }
  // Z[key][d]: col = d (lane), row = key (registers)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int kk = kb * AT_TILE + crow(i, hh);
    if (kk < T) {
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const int64_t off = ((int64_t)b * T + kk) * ldg + col0 + db * 32 + r;
        dk[off] = f2h(dkacc[db][i] * a.scale);
        dv[off] = f2h(dvacc[db][i]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------------
// Fused backward: ONE workgroup per (b, h), one wave per 32-row tile (T <= 224: nt <= 7 waves), every
// S / dP tile computed once (5 matmul units per (query tile, key tile) pair instead of the 7 of the
// two-kernel path), K/V/Q/dO staged once per (b, h).
//   phase 0  all threads: Q and dO images, gate / lse of every query row, D = rowsum(dO o O) -> LDS.
//   phase 1  wave kb (key-stationary): S = Q K^T, dP = dO V^T per query tile, dV += P^T dO, dK += dS^T Q;
//            dS (bf16) goes to an LDS image [key][query] of 32-column panels, one panel per query tile.
//   phase 2  K image over the Q image; wave qb (query-stationary): dQ = dS K with both operands read by
//            ds_read_b64_tr_b16 from LDS (the same permuted k order on both sides), d gate = sum over
//            keys of dS * pb from the same fragments.
// LDS at nt = 7: Q 28 KB + dO 28 KB + dS 98 KB + row scalars 2.6 KB = 157 KB (one workgroup per CU).
// The relative-position bias row of the head lives in LDS too (2 tp floats).
// untransposed (pb[h][q][key]); both are L2-resident (blocks of one head are steered to one XCD).
constexpr int AT_FUSED_MAXNT = 7;

// byte offset of 16-byte chunk ch (0..3) of row `row` in a 32-column panel image: 8-row x 32-column
// subtiles of 512 B with the same (row >> 2) & 3 chunk swizzle as img_off
__device__ __forceinline__ int pan_off(int row, int ch) {
  return 512 * (row >> 3) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}
// read_tr on a 32-column panel: element j = X[r0 + 16 s + 8 (j >> 2) + 4 h + (j & 3)][lane & 31]
__device__ __forceinline__ hx8 read_tr_pan(char* pan, int r0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int row = r0 + 16 * s + 4 * (g >> 1) + (i >> 2);
  const int col = 16 * (g & 1) + 4 * (i & 3);
  const int sub = 2 * (col & 7);
  const hx4v lo = ds_tr4((pan + pan_off(row, col >> 3) + sub));
  const hx4v hi = ds_tr4((pan + pan_off(row + 8, col >> 3) + sub));
  hx8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = lo[j];
    r[4 + j] = hi[j];
  }
  return r;
}

// Fixed LDS map of the fused backward (T <= 224): images at compile-time offsets, so every fragment read
// is one lane-offset VGPR + an immediate. Image tile t starts at t * 4096.
constexpr int FB_Q = 0;                                              // Q image; phase 2: K image
constexpr int FB_DO = AT_FUSED_MAXNT * AT_TILE_BYTES;                // dO image
constexpr int FB_DS = 2 * AT_FUSED_MAXNT * AT_TILE_BYTES;            // dS panels, panel qb at qb * tp * 64
constexpr int FB_SC = FB_DS + AT_FUSED_MAXNT * AT_FUSED_MAXNT * AT_TILE * 64;   // gate, lse, D rows
constexpr int FB_TAB = FB_SC + 3 * AT_FUSED_MAXNT * AT_TILE * 4;    // relative-position bias row
constexpr int FB_LDS = FB_TAB + 2 * AT_FUSED_MAXNT * AT_TILE * 4;   // 162176 B

// lane part of read_row(img, 32 t + r, s, hh) = img_off(r, 2 (s & 1) + hh) + 512 (s >> 1) + 4096 t
__device__ __forceinline__ int fb_row_off(int r, int hh, int sodd) { return img_off(r, 2 * sodd + hh); }
// lane part of read_tr(img, 32 t, 32 db, s, lane) (half hi = 0 / 1): + 4096 t + 2048 s + 512 db
__device__ __forceinline__ int fb_tr_off(int lane, int hi) {
  const int g = lane >> 4, i = lane & 15;
  const int row = 4 * (g >> 1) + (i >> 2) + 8 * hi, col = 16 * (g & 1) + 4 * (i & 3);
  return img_off(row, col >> 3) + 2 * (col & 7);
}
// lane part of read_tr_pan(panel, 32 t, s, lane) (half hi): + 2048 t + 1024 s
__device__ __forceinline__ int fb_pan_off(int lane, int hi) {
  const int g = lane >> 4, i = lane & 15;
  const int row = 4 * (g >> 1) + (i >> 2) + 8 * hi, col = 16 * (g & 1) + 4 * (i & 3);
  return pan_off(row, col >> 3) + 2 * (col & 7);
}
__device__ __forceinline__ hx8 lds8(const char* p) { return *reinterpret_cast<const hx8*>(p); }
__device__ __forceinline__ hx8 lds_tr(const char* lo, const char* hi) {
  const hx4v a = ds_tr4(lo);
  const hx4v b = ds_tr4(hi);
  hx8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = a[j];
    r[4 + j] = b[j];
  }
  return r;
}

// kSplit (grids of fewer (b, h) than CUs, B = 8): TWO workgroups per (b, h), part p taking the key tiles
// [kbeg, kend) (the first ceil(nt / 2), the rest) in phase 1 and in phase 2's sum over keys; each writes its
// partial dQ / d gate (fp32) to ws, and the second to arrive (agent-scope release / acquire, a self-resetting
// ticket) adds the two in part order and stores dQ and d gate. Per CU: half the phase-1 MFMAs, 4 / 7 of phase 2.
constexpr int FB_WSP = AT_FUSED_MAXNT * AT_TILE * (AT_DH + 1);   // fp32 per (b, h, part): dQ [tp][64], d gate [tp]

template <bool kDrop, bool kSplit = false>
__global__ __launch_bounds__(AT_FUSED_MAXNT * 64) void attn_bwd_fused_kernel(
    AttnArgs a, AttnBwdArgs g, const uint32_t* __restrict__ mask,
    const hst* __restrict__ O, int64_t ldo,
    hst* __restrict__ dq, hst* __restrict__ dk, hst* __restrict__ dv, int64_t ldg,
    float* __restrict__ dgate, float* __restrict__ ws, int* __restrict__ counters) {
  extern __shared__ __attribute__((aligned(16))) char at_lds[];
  char* const L = at_lds;
  const int T = a.T, H = a.H, nt = (T + AT_TILE - 1) / AT_TILE, tp = nt * AT_TILE;
  // blocks of one head on one XCD (blocks b and b + 8 share an XCD): the head's bias row stays in that XCD's L2.
  // A speed choice only; any placement is correct.
  int head, b, part = 0;
  {
    int bid = blockIdx.x;
    if (kSplit) {   // the two parts of a (b, h) are blocks bid and bid + 8 (one XCD)
      part = (bid >> 3) & 1;
      bid = (bid & 7) | ((bid >> 4) << 3);
    }
    if ((H & 7) == 0) {
      const int xcd = bid & 7, j = bid >> 3, hpx = H >> 3;
      head = xcd + 8 * (j % hpx);
      b = j / hpx;
    } else {
      head = bid % H;
      b = bid / H;
    }
  }
  const int64_t col0 = (int64_t)head * AT_DH;
  const int64_t bh = (int64_t)b * H + head;
  const int64_t row0 = (int64_t)b * T;
  float* s_gate = reinterpret_cast<float*>(L + FB_SC);
  float* s_lse = s_gate + AT_FUSED_MAXNT * AT_TILE;
  float* s_D = s_lse + AT_FUSED_MAXNT * AT_TILE;
  float* tab = reinterpret_cast<float*>(L + FB_TAB);
  const int nthr = nt * 64;                            // every image is exactly 4 chunks per thread
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  RDX_PROBE(0);
  // ---- phase 0: every global load of the phase in flight at once (Q and dO images, the O row and
  // scalars of this thread's query row, this wave's K / V fragments), then the LDS writes; D =
  // rowsum(dO o O) after a barrier, from the dO image (dO is read from HBM once)
  const int kbeg = kSplit && part ? (nt + 1) / 2 : 0, kend = kSplit && !part ? (nt + 1) / 2 : nt;
  const int kb = __builtin_amdgcn_readfirstlane(w) + kbeg;
  const bool kact = kb < kend;       // this wave has a key tile in phase 1
  const int key = kb * AT_TILE + r;
  const bool kvalid = kact && key < T;
  hx8 kf[4], vf[4];
  {
    hx8 qv[4], ov[4], xo[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = threadIdx.x + j * nthr, row = i >> 3, ch = i & 7;
      qv[j] = load8(a.q + (row0 + row) * a.ldq + col0 + 8 * ch, row < T);
      ov[j] = load8(g.dO + (row0 + row) * g.lddo + col0 + 8 * ch, row < T);
    }
    const int t = threadIdx.x;
    const bool trow = t < T;
    const int64_t tr = row0 + (trow ? t : 0);
#pragma unroll
    for (int c = 0; c < 8; ++c) xo[c] = load8(O + tr * ldo + col0 + 8 * c, trow);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[s] = load8(a.k + (row0 + key) * a.ldk + col0 + 16 * s + 8 * hh, kvalid);
      vf[s] = load8(a.v + (row0 + key) * a.ldv + col0 + 16 * s + 8 * hh, kvalid);
    }
    // base-2 domain: p = exp2(S * scale * log2e + gate * log2e * pb - lse * log2e); a padded row
    // (t >= T) gets lse = +inf, so its p (and dS) are exactly 0 with no per-element test
    const float gq = trow ? a.gate[tr * H + head] * kLog2e : 0.f;
    const float lq = trow ? g.lse[bh * T + t] * kLog2e : INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = threadIdx.x + j * nthr, row = i >> 3, ch = i & 7;
      *reinterpret_cast<hx8*>(L + FB_Q + img_off(row, ch)) = qv[j];
      *reinterpret_cast<hx8*>(L + FB_DO + img_off(row, ch)) = ov[j];
    }
    if (t < tp) {
      s_gate[t] = gq;
      s_lse[t] = lq;
    }
    stage_rel(tab, a.rel, head, T, tp);
    RDX_PROBE(6);
    __syncthreads();
    if (t < tp) {
      float dd = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const hx8 xd = lds8(L + FB_DO + img_off(t, c));
#pragma unroll
        for (int j = 0; j < 8; ++j) dd = fmaf((float)xd[j], (float)xo[c][j], dd);
      }
      if (trow && part == 0) g.D[bh * T + t] = dd;
      s_D[t] = dd;
    }
  }
  const int ro0 = fb_row_off(r, hh, 0), ro1 = fb_row_off(r, hh, 1);
  const int tr0 = fb_tr_off(lane, 0), tr1 = fb_tr_off(lane, 1);
  __syncthreads();
  RDX_PROBE(1);
  // ---- phase 1: wave w owns key tile kb = kbeg + w
  if (kact) {
    // this lane's key in a mask word of the forward: bit i + 16 h with crow(i, h) = r
    const int bitpos = (r & 3) + 4 * (r >> 3) + 16 * ((r >> 2) & 1);
    const float scale2 = a.scale * kLog2e;
    // dS image rows of this lane's key: chunk 2s + t of the row (plus 8 hh bytes) in every panel
    int dso[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) dso[c] = FB_DS + pan_off(kb * AT_TILE + r, c) + 8 * hh;
    f32x16 dkacc[2] = {zero16(), zero16()}, dvacc[2] = {zero16(), zero16()};
    // the keep words of this lane's 16 query rows (crow(4c + e, hh) = 8c + 4hh + e, the same addresses
    // across each half-wave) are loaded one tile ahead, so their HBM latency runs under the previous
    // tile's work
    const uint32_t* mbase = mask + mask_word(bh, nt, tp, kb, 0) + 4 * hh;
    uint4 mwn[4];
    if (kDrop) {
#pragma unroll
      for (int c = 0; c < 4; ++c) mwn[c] = *reinterpret_cast<const uint4*>(mbase + 8 * c);
    }
    for (int qb = 0; qb < nt; ++qb) {
      float pbv[16];
      uint4 mw[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) mw[c] = mwn[c];
      if (kDrop && qb + 1 < nt) {
#pragma unroll
        for (int c = 0; c < 4; ++c) mwn[c] = *reinterpret_cast<const uint4*>(mbase + (qb + 1) * AT_TILE + 8 * c);
      }
      asm volatile("" ::: "memory");
      rel16_k(tab, key, T, tp, qb, hh, pbv);
      const char* R0 = L + qb * AT_TILE_BYTES + ro0;
      const char* R1 = L + qb * AT_TILE_BYTES + ro1;
      f32x16 S = zero16(), dP = zero16();
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const char* R = (s & 1) ? R1 : R0;
        S = mfma32(lds8(R + FB_Q + 512 * (s >> 1)), kf[s], S);
        dP = mfma32(lds8(R + FB_DO + 512 * (s >> 1)), vf[s], dP);
      }
      float P[16], dS[16];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int q0 = qb * AT_TILE + 8 * c + 4 * hh;  // rows crow(4c + e, hh) = q0 + e
        const float4 g4 = *reinterpret_cast<const float4*>(s_gate + q0);
        const float4 l4 = *reinterpret_cast<const float4*>(s_lse + q0);
        const float4 d4 = *reinterpret_cast<const float4*>(s_D + q0);
        const float gv[4] = {g4.x, g4.y, g4.z, g4.w}, lv[4] = {l4.x, l4.y, l4.z, l4.w};
        const float dd[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * c + e;
          // no per-element test: rows past T have lse = +inf (p = 0); a key past T has finite p and dS that
          // only reach its own (unwritten) dK / dV row, or meet a zero K row / zero pb entry in phase 2
          const float p = __builtin_amdgcn_exp2f(fmaf(S[i], scale2, fmaf(gv[e], pbv[i], -lv[e])));
          float mk = 1.f;
          if (kDrop) {
            const uint32_t word = e == 0 ? mw[c].x : e == 1 ? mw[c].y : e == 2 ? mw[c].z : mw[c].w;
            mk = ((word >> bitpos) & 1u) ? a.inv_keep : 0.f;
          }
          dS[i] = p * fmaf(dP[i], mk, -dd[e]);
          P[i] = p * mk;
        }
      }
      const char* T0 = L + qb * AT_TILE_BYTES + tr0;
      const char* T1 = L + qb * AT_TILE_BYTES + tr1;
      char* pan = L + qb * tp * 64;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const hx8 xp = pack8(P + 8 * s), xs = pack8(dS + 8 * s);
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          const int o = 2048 * s + 512 * db;
          dvacc[db] = mfma32(xp, lds_tr(T0 + FB_DO + o, T1 + FB_DO + o), dvacc[db]);
          dkacc[db] = mfma32(xs, lds_tr(T0 + FB_Q + o, T1 + FB_Q + o), dkacc[db]);
        }
        // dS rows crow(8s + 4t + e, hh) = 16 s + 8 t + 4 hh + e of the query panel -> [key][q] image
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          hx4v v4;
#pragma unroll
          for (int e = 0; e < 4; ++e) v4[e] = xs[4 * t + e];
          *reinterpret_cast<hx4v*>(pan + dso[2 * s + t]) = v4;
        }
      }
    }
    RDX_PROBE(2);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kk = kb * AT_TILE + crow(i, hh);
      if (kk < T) {
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          const int64_t off = (row0 + kk) * ldg + col0 + db * 32 + r;
          dk[off] = f2h(dkacc[db][i] * a.scale);
          dv[off] = f2h(dvacc[db][i]);
        }
      }
    }
  }
  const int qb2 = __builtin_amdgcn_readfirstlane(w);
  const int qi2 = qb2 * AT_TILE + r;
  // the K image over the Q image, from the K fragments already in registers: lane (r, hh) holds key row
  // kb*32 + r, columns 16 s + 8 hh .. + 7 = chunk 2 s + hh (zero rows past T)
  RDX_PROBE(7);
  __syncthreads();  // every dS panel is complete; the Q image is free
  if (kact) {
#pragma unroll
    for (int s = 0; s < 4; ++s) *reinterpret_cast<hx8*>(L + FB_Q + img_off(kb * AT_TILE + r, 2 * s + hh)) = kf[s];
  }
  __syncthreads();
  RDX_PROBE(3);
  // ---- phase 2: wave w owns query tile qb = w
  {
    const int qb = qb2;
    const int qi = qi2;  // this lane's query row in the A fragments
    const bool qvalid = qi < T;
    const char* P0 = L + FB_DS + qb * tp * 64 + fb_pan_off(lane, 0);
    const char* P1 = L + FB_DS + qb * tp * 64 + fb_pan_off(lane, 1);
    f32x16 dqacc[2] = {zero16(), zero16()};
    float dg = 0.f;
    for (int kb2 = kbeg; kb2 < kend; ++kb2) {
      float pbv[16];
      rel16_q(tab, qi, T, tp, kb2, hh, pbv);
      // dS of a key past T is finite but meaningless (phase 1 does not mask keys): its bias weight is 0
      if (kb2 == nt - 1) {
#pragma unroll
        for (int i = 0; i < 16; ++i) pbv[i] = kb2 * AT_TILE + crow(i, hh) < T ? pbv[i] : 0.f;
      }
      const char* K0 = L + FB_Q + kb2 * AT_TILE_BYTES + tr0;
      const char* K1 = L + FB_Q + kb2 * AT_TILE_BYTES + tr1;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int po = 2048 * kb2 + 1024 * s;
        const hx8 xs = lds_tr(P0 + po, P1 + po);  // dS[qi][keys of step s]
#pragma unroll
        for (int j = 0; j < 8; ++j) dg = fmaf((float)xs[j], pbv[8 * s + j], dg);
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          const int o = 2048 * s + 512 * db;
          dqacc[db] = mfma32(xs, lds_tr(K0 + o, K1 + o), dqacc[db]);
        }
      }
    }
    RDX_PROBE(4);
    dg += __shfl_xor(dg, 32, 64);
    if (kSplit) {   // partials of this part: dQ [tp][64] then d gate [tp], stored write-through (sc1)
      float* wp = ws + (bh * 2 + part) * FB_WSP;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(wp, 0, FB_WSP * 4, 0x00020000);
      if (qvalid && hh == 0)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dg), rs, (AT_FUSED_MAXNT * AT_TILE * AT_DH + qi) * 4, 0,
                                              16);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qq = qb * AT_TILE + crow(i, hh);
        if (qq < T) {
#pragma unroll
          for (int db = 0; db < 2; ++db)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dqacc[db][i]), rs, (qq * AT_DH + db * 32 + r) * 4,
                                                  0, 16);
        }
      }
    } else {
      if (qvalid && hh == 0) dgate[(row0 + qi) * H + head] = dg;
      // C[q][d]: col = d (lane), row = q (registers)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qq = qb * AT_TILE + crow(i, hh);
        if (qq < T) {
#pragma unroll
          for (int db = 0; db < 2; ++db)
            dq[(row0 + qq) * ldg + col0 + db * 32 + r] = f2h(dqacc[db][i] * a.scale);
        }
      }
    }
  }
  if (kSplit) {
    // publish: the partials were stored write-through, so every wave's stores retired then the ticket, with no
    // release fence (an agent-scope release wrote the L2 back, µs per block); the second arriver acquires and
    // combines (cdna_hip_programming.md Guideline 16, R1); the ticket is left at zero
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(L + FB_SC);   // the row-scalar area is free in phase 2
    if (threadIdx.x == 0) {
#if !defined(__gfx950__) && !defined(__gfx942__)
      // the fence-free publish relies on gfx94x / gfx950's write-through (sc1) store encoding; any other target
      // releases the partials explicitly
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#endif
      const int t = __hip_atomic_fetch_add(counters + bh, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = t;
      if (t == 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        counters[bh] = 0;
      }
    }
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(flag[0]) == 1) {
      const float* w0 = ws + (bh * 2) * FB_WSP;
      const float* w1 = w0 + FB_WSP;
      for (int i = threadIdx.x; i < T * (AT_DH / 4); i += nthr) {
        const int qq = i / (AT_DH / 4), c4 = (i - qq * (AT_DH / 4)) * 4;
        const float4 x0 = *reinterpret_cast<const float4*>(w0 + qq * AT_DH + c4);
        const float4 x1 = *reinterpret_cast<const float4*>(w1 + qq * AT_DH + c4);
        hst* dst = dq + (row0 + qq) * ldg + col0 + c4;
        dst[0] = f2h((x0.x + x1.x) * a.scale);
        dst[1] = f2h((x0.y + x1.y) * a.scale);
        dst[2] = f2h((x0.z + x1.z) * a.scale);
        dst[3] = f2h((x0.w + x1.w) * a.scale);
      }
      for (int t = threadIdx.x; t < T; t += nthr)
        dgate[(row0 + t) * H + head] = w0[AT_FUSED_MAXNT * AT_TILE * AT_DH + t] + w1[AT_FUSED_MAXNT * AT_TILE * AT_DH + t];
    }
  }
  RDX_PROBE(5);
}

// element-wise dropout mask of the same paired hash (tests only): keep[row, key] in {0, 1} for rows
// (b*H + h)*T + q of length T
__global__ void attn_mask_kernel(const int64_t* seed_dev, int salt, uint32_t thr, uint8_t* keep, int64_t n, int T) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) {
    const int64_t row = t / T;
    const int key = (int)(t - row * T);
    const uint32_t h = pair_hash(attn_seed(seed_dev, salt), (uint64_t)row * (uint64_t)((T + 1) >> 1) + (key >> 1));
    keep[t] = half_keep(h, key & 1, thr) ? 1 : 0;
  }
}

// element-wise dropout mask of the per-element hash drop_keep (the fused WavLM layer's hidden / LoRA
// dropouts, csrc/wavlm_layer.hip; tests only): keep[t] for element index t
__global__ void elem_mask_kernel(const int64_t* seed_dev, int salt, uint32_t thr, uint8_t* keep, int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) keep[t] = drop_keep(attn_seed(seed_dev, salt), (uint64_t)t, thr) ? 1 : 0;
}

inline AttnArgs make_args(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                          const float* gate, const float* rel, const int64_t* seed_dev, int salt,
                          float p_drop, float scale, int B, int T, int H) {
  AttnArgs a;
  a.q = (const hst*)q;
  a.k = (const hst*)k;
  a.v = (const hst*)v;
  a.ldq = ldq;
  a.ldk = ldk;
  a.ldv = ldv;
  a.gate = gate;
  a.rel = rel;
  a.seed_dev = seed_dev;
  a.salt = salt;
  const double t = (double)p_drop * 65536.0 + 0.5;   // 16-bit threshold of the paired hash
  a.thr = p_drop > 0.f ? (uint32_t)(t >= 65535.0 ? 65535.0 : (t < 1.0 ? 1.0 : t)) : 0u;
  a.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  a.scale = scale;
  a.B = B;
  a.T = T;
  a.H = H;
  return a;
}

}  // namespace rdx

using namespace rdx;

static bool attn_ok(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv, int B,
                    int T, int H) {
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  return q && k && v && al(q) && al(k) && al(v) && B > 0 && T > 0 && H > 0 && B <= 65535 && H <= 65535 &&
         ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldq >= (int64_t)H * AT_DH && ldk >= (int64_t)H * AT_DH &&
         ldv >= (int64_t)H * AT_DH;
}

static inline size_t rel_bytes(int T) { return (size_t)2 * ((T + AT_TILE - 1) / AT_TILE) * AT_TILE * sizeof(float); }

// the dK/dV kernel's images and row scalars exceed the default 64 KB dynamic-LDS cap at T = 256
static int attn_allow_lds(const void* fn, bool& done) {
  if (done) return RDX_OK;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return (int)e;
  done = true;
  return RDX_OK;
}

template <bool kDrop, bool kIdx32, bool kSplit>
static int launch_fwd(dim3 grid, size_t lds, hipStream_t st, const AttnArgs& a, hst* o, int64_t ldo,
                      float* lse, uint32_t* mask) {
  static bool done = false;
  const int rc = attn_allow_lds(reinterpret_cast<const void*>(&attn_fwd_kernel<kDrop, kIdx32, kSplit>), done);
  if (rc != RDX_OK) return rc;
  if (kSplit) lds += (size_t)AT_WAVES * 64 * AT_MERGE_STRIDE * 4;
  hipLaunchKernelGGL((attn_fwd_kernel<kDrop, kIdx32, kSplit>), grid, dim3(at_fwd_threads<kSplit>()), lds, st, a, o,
                     ldo, lse, mask);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

template <bool kDrop>
static int launch_bwd(dim3 grid, size_t lds_dq, size_t lds_kv, hipStream_t st, const AttnArgs& a,
                      const AttnBwdArgs& g, const hst* o, int64_t ldo, hst* dq,
                      hst* dk, hst* dv, int64_t ldg, float* dgate) {
  static bool done_dq = false, done_kv = false;
  int rc = attn_allow_lds(reinterpret_cast<const void*>(&attn_bwd_dq_kernel<kDrop>), done_dq);
  if (rc != RDX_OK) return rc;
  rc = attn_allow_lds(reinterpret_cast<const void*>(&attn_bwd_dkdv_kernel<kDrop>), done_kv);
  if (rc != RDX_OK) return rc;
  hipLaunchKernelGGL((attn_bwd_dq_kernel<kDrop>), grid, dim3(AT_WAVES * 64), lds_dq, st, a, g, o, ldo, dq, ldg,
                     dgate);
  RDX_LAUNCH_CHECK();
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<kDrop>), grid, dim3(AT_WAVES * 64), lds_kv, st, a, g, dk, dv, ldg);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_attn_fwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                            const float* gate, const float* rel_bias, const int64_t* seed_dev,
                            int salt, float p_drop, float scale, void* o, int64_t ldo, float* lse,
                            uint32_t* keep_mask, int B, int T, int H, int head_dim, void* stream) {
  RDX_REQUIRE(attn_ok(q, ldq, k, ldk, v, ldv, B, T, H) && gate && rel_bias && o && lse && ldo >= (int64_t)H * AT_DH);
  RDX_REQUIRE(ldo % 4 == 0 && ((uintptr_t)o & 7) == 0);   // 8-byte output stores
  RDX_REQUIRE(p_drop >= 0.f && p_drop < 1.f && (p_drop == 0.f || seed_dev));
  if (head_dim != AT_DH || T > AT_MAXNT * AT_TILE) return RDX_EUNSUPPORTED;
  const AttnArgs a = make_args(q, ldq, k, ldk, v, ldv, gate, rel_bias, seed_dev, salt, p_drop, scale, B, T, H);
  const int nt = (T + AT_TILE - 1) / AT_TILE;
  const dim3 grid((nt + AT_WAVES - 1) / AT_WAVES, H, B);
  const size_t lds = 2 * (size_t)AT_MAXNT * AT_TILE_BYTES + 2 * AT_MAXNT * AT_TILE * sizeof(float);   // see the kernel
  hipStream_t st = as_stream(stream);
  hst* ob = (hst*)o;
  // key-split kernel while the unsplit grid is at most 2 workgroups per CU (one wave per SIMD each)
  const bool split = (int64_t)grid.x * grid.y * grid.z <= 512;
  if (!a.thr)
    return split ? launch_fwd<false, true, true>(grid, lds, st, a, ob, ldo, lse, nullptr)
                 : launch_fwd<false, true, false>(grid, lds, st, a, ob, ldo, lse, nullptr);
  const bool idx32 = (uint64_t)B * H * (uint64_t)T * (uint64_t)((T + 1) >> 1) <= 0xffffffffull;
  if (split)
    return idx32 ? launch_fwd<true, true, true>(grid, lds, st, a, ob, ldo, lse, keep_mask)
                 : launch_fwd<true, false, true>(grid, lds, st, a, ob, ldo, lse, keep_mask);
  return idx32 ? launch_fwd<true, true, false>(grid, lds, st, a, ob, ldo, lse, keep_mask)
               : launch_fwd<true, false, false>(grid, lds, st, a, ob, ldo, lse, keep_mask);
}

extern "C" int64_t rdx_attn_keep_mask_words(int B, int T, int H) {
  const int64_t nt = (T + AT_TILE - 1) / AT_TILE;
  return (int64_t)B * H * nt * nt * AT_TILE;
}

extern "C" int rdx_attn_bwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                            const float* gate, const float* rel_bias, const int64_t* seed_dev,
                            int salt, float p_drop, float scale, const void* o, int64_t ldo, const float* lse,
                            const void* dout, int64_t lddo, float* D, void* dq, void* dk, void* dv, int64_t ldg,
                            float* dgate, int B, int T, int H, int head_dim, void* stream) {
  RDX_REQUIRE(attn_ok(q, ldq, k, ldk, v, ldv, B, T, H) && gate && rel_bias && o && lse && dout && D);
  RDX_REQUIRE(dq && dk && dv && dgate && ldg >= (int64_t)H * AT_DH && ldg % 8 == 0 && lddo % 8 == 0 && ldo % 8 == 0);
  RDX_REQUIRE(((uintptr_t)o & 15) == 0 && ((uintptr_t)dout & 15) == 0);
  RDX_REQUIRE(p_drop >= 0.f && p_drop < 1.f && (p_drop == 0.f || seed_dev));
  if (head_dim != AT_DH || T > AT_MAXNT * AT_TILE) return RDX_EUNSUPPORTED;
  const AttnArgs a = make_args(q, ldq, k, ldk, v, ldv, gate, rel_bias, seed_dev, salt, p_drop, scale, B, T, H);
  const AttnBwdArgs g{(const hst*)dout, lddo, lse, D};
  const int nt = (T + AT_TILE - 1) / AT_TILE;
  const dim3 grid((nt + AT_WAVES - 1) / AT_WAVES, H, B);
  const size_t lds_dq = 2 * (size_t)nt * AT_TILE_BYTES + rel_bytes(T);
  const size_t lds_kv = 2 * (size_t)nt * AT_TILE_BYTES + 3 * (size_t)nt * AT_TILE * sizeof(float) + rel_bytes(T);
  return a.thr ? launch_bwd<true>(grid, lds_dq, lds_kv, as_stream(stream), a, g, (const hst*)o, ldo,
                                  (hst*)dq, (hst*)dk, (hst*)dv, ldg, dgate)
               : launch_bwd<false>(grid, lds_dq, lds_kv, as_stream(stream), a, g, (const hst*)o, ldo,
                                   (hst*)dq, (hst*)dk, (hst*)dv, ldg, dgate);
}

template <bool kDrop, bool kSplit>
static int launch_bwd_fused(dim3 grid, dim3 block, size_t lds, hipStream_t st, const AttnArgs& a,
                            const AttnBwdArgs& g, const uint32_t* mask, const void* o, int64_t ldo,
                            void* dq, void* dk, void* dv, int64_t ldg, float* dgate, float* ws, int* counters) {
  static bool done = false;
  const int rc = attn_allow_lds(reinterpret_cast<const void*>(&attn_bwd_fused_kernel<kDrop, kSplit>), done);
  if (rc != RDX_OK) return rc;
  hipLaunchKernelGGL((attn_bwd_fused_kernel<kDrop, kSplit>), grid, block, lds, st, a, g, mask,
                     (const hst*)o, ldo, (hst*)dq, (hst*)dk, (hst*)dv, ldg,
                     dgate, ws, counters);
  return RDX_OK;
}

extern "C" int rdx_attn_bwd_fused(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                                  int64_t ldv, const float* gate, const float* rel_bias,
                                  const uint32_t* keep_mask, float p_drop, float scale, const void* o,
                                  int64_t ldo, const float* lse, const void* dout, int64_t lddo, float* D, void* dq,
                                  void* dk, void* dv, int64_t ldg, float* dgate, int B, int T, int H, int head_dim,
                                  void* stream) {
  RDX_REQUIRE(attn_ok(q, ldq, k, ldk, v, ldv, B, T, H) && gate && rel_bias && o && lse && dout && D);
  RDX_REQUIRE(dq && dk && dv && dgate && ldg >= (int64_t)H * AT_DH && ldg % 8 == 0 && lddo % 8 == 0 && ldo % 8 == 0);
  RDX_REQUIRE(((uintptr_t)o & 15) == 0 && ((uintptr_t)dout & 15) == 0);
  RDX_REQUIRE(p_drop >= 0.f && p_drop < 1.f && (p_drop == 0.f || keep_mask));
  RDX_REQUIRE((int64_t)B * H <= 0x7fffffff);
  if (head_dim != AT_DH || T > AT_FUSED_MAXNT * AT_TILE) return RDX_EUNSUPPORTED;
  const AttnArgs a = make_args(q, ldq, k, ldk, v, ldv, gate, rel_bias, nullptr, 0, p_drop, scale, B, T, H);
  const AttnBwdArgs g{(const hst*)dout, lddo, lse, D};
  const int nt = (T + AT_TILE - 1) / AT_TILE, tp = nt * AT_TILE;
  const size_t lds = FB_LDS;   // fixed map (immediate-offset LDS addressing)
  const dim3 grid((unsigned)(B * H)), block(nt * 64);
  (void)tp;
  hipStream_t st = as_stream(stream);
  const int rc = a.thr ? launch_bwd_fused<true, false>(grid, block, lds, st, a, g, keep_mask, o, ldo, dq, dk, dv,
                                                       ldg, dgate, nullptr, nullptr)
                       : launch_bwd_fused<false, false>(grid, block, lds, st, a, g, keep_mask, o, ldo, dq, dk,
                                                        dv, ldg, dgate, nullptr, nullptr);
  if (rc != RDX_OK) return rc;
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int64_t rdx_attn_bwd_split_ws(int B, int H) { return (int64_t)B * H * 2 * FB_WSP; }

extern "C" int rdx_attn_bwd_fused_split(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                                        int64_t ldv, const float* gate, const float* rel_bias,
                                        const uint32_t* keep_mask, float p_drop, float scale, const void* o,
                                        int64_t ldo, const float* lse, const void* dout, int64_t lddo, float* D,
                                        void* dq, void* dk, void* dv, int64_t ldg, float* dgate, float* ws,
                                        int64_t ws_floats, int* counters, int64_t n_counters, int B, int T, int H,
                                        int head_dim, void* stream) {
  RDX_REQUIRE(attn_ok(q, ldq, k, ldk, v, ldv, B, T, H) && gate && rel_bias && o && lse && dout && D);
  RDX_REQUIRE(dq && dk && dv && dgate && ldg >= (int64_t)H * AT_DH && ldg % 8 == 0 && lddo % 8 == 0 && ldo % 8 == 0);
  RDX_REQUIRE(((uintptr_t)o & 15) == 0 && ((uintptr_t)dout & 15) == 0);
  RDX_REQUIRE(p_drop >= 0.f && p_drop < 1.f && (p_drop == 0.f || keep_mask));
  RDX_REQUIRE(ws && counters && ((uintptr_t)ws & 15) == 0 && ws_floats >= rdx_attn_bwd_split_ws(B, H) &&
              n_counters >= (int64_t)B * H);
  RDX_REQUIRE(((int64_t)B * H) % 8 == 0 && (int64_t)B * H * 2 <= 0x7fffffff);   // the block -> part map
  if (head_dim != AT_DH || T > AT_FUSED_MAXNT * AT_TILE) return RDX_EUNSUPPORTED;
  const AttnArgs a = make_args(q, ldq, k, ldk, v, ldv, gate, rel_bias, nullptr, 0, p_drop, scale, B, T, H);
  const AttnBwdArgs g{(const hst*)dout, lddo, lse, D};
  const int nt = (T + AT_TILE - 1) / AT_TILE;
  const dim3 grid((unsigned)(2 * B * H)), block(nt * 64);
  hipStream_t st = as_stream(stream);
  const int rc = a.thr ? launch_bwd_fused<true, true>(grid, block, FB_LDS, st, a, g, keep_mask, o, ldo, dq, dk, dv,
                                                      ldg, dgate, ws, counters)
                       : launch_bwd_fused<false, true>(grid, block, FB_LDS, st, a, g, keep_mask, o, ldo, dq, dk, dv,
                                                       ldg, dgate, ws, counters);
  if (rc != RDX_OK) return rc;
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_attn_dropout_mask(const int64_t* seed_dev, int salt, float p_drop, uint8_t* keep, int64_t n,
                                     int T, void* stream) {
  RDX_REQUIRE(seed_dev && keep && n > 0 && T > 0 && n % T == 0 && p_drop >= 0.f && p_drop < 1.f);
  const AttnArgs a = make_args(nullptr, 0, nullptr, 0, nullptr, 0, nullptr, nullptr, seed_dev, salt, p_drop, 1.f, 1, 1, 1);
  hipLaunchKernelGGL(attn_mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), seed_dev,
                     salt, a.thr, keep, n, T);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_dropout_mask(const int64_t* seed_dev, int salt, float p_drop, uint8_t* keep, int64_t n,
                                void* stream) {
  RDX_REQUIRE(seed_dev && keep && n > 0 && p_drop >= 0.f && p_drop < 1.f);
  const double t = (double)p_drop * 4294967296.0;
  const uint32_t thr = p_drop > 0.f ? (uint32_t)(t >= 4294967295.0 ? 4294967295.0 : t) : 0u;
  hipLaunchKernelGGL(elem_mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), seed_dev,
                     salt, thr, keep, n);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
