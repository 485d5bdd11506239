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

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((__vector_size__(4 * sizeof(__bf16)))) __bf16 bf16x4v;
typedef __attribute__((address_space(3))) bf16x4v lds_bf16x4v;
constexpr int AT_DH = 64;                  // head dim
constexpr int AT_TILE = 32;                // rows per wave
constexpr int AT_MAXNT = 8;                // tiles per sequence: T <= 256
constexpr int AT_WAVES = 4;                // waves (tiles) per workgroup
constexpr int AT_TILE_BYTES = AT_TILE * AT_DH * 2;  // one 32-row tile of an image: 4 KB

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// C/D row held in accumulator register i by lane half h
__device__ __forceinline__ int crow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

__device__ __forceinline__ bf16x8 pack8(const float* x) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)x[j];
  return r;
}
__device__ __forceinline__ bf16x8 load8(const __hip_bfloat16* p, bool ok) {
  if (!ok) {
    bf16x8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = (__bf16)0.f;
    return z;
  }
  return *reinterpret_cast<const bf16x8*>(p);
}
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// the 16 position-bias values of key tile kb this lane needs (keys kb*32 + crow(i, hh)): four float4
// loads from a row padded to a multiple of 32
__device__ __forceinline__ void load_pb16(const float* pbrow, int kb, int hh, float* v) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float4 t = *reinterpret_cast<const float4*>(pbrow + kb * AT_TILE + 8 * c + 4 * hh);
    v[4 * c] = t.x;
    v[4 * c + 1] = t.y;
    v[4 * c + 2] = t.z;
    v[4 * c + 3] = t.w;
  }
}

// Byte offset of 16-byte chunk ch (0..7, columns 8 ch .. 8 ch + 7) of image row `row`: 8-row x 32-column
// subtiles of 512 B, chunk XOR-swizzled by (row >> 2) & 3 (MI355X guide T10, layout (a), on 64-column rows).
__device__ __forceinline__ int img_off(int row, int ch) {
  return 1024 * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}

// rows [0, 32 nt) of the head slice (columns col0 .. col0 + 63) of a [B, T, ld] bf16 tensor into an LDS
// image; rows past T are zero. Every thread of the workgroup takes part.
__device__ __forceinline__ void stage_image(char* img, const __hip_bfloat16* src, int64_t ld, int b, int T,
                                            int64_t col0, int nt) {
  for (int i = threadIdx.x; i < nt * AT_TILE * 8; i += AT_WAVES * 64) {
    const int row = i >> 3, ch = i & 7;
    *reinterpret_cast<bf16x8*>(img + img_off(row, ch)) =
        load8(src + ((int64_t)b * T + row) * ld + col0 + 8 * ch, row < T);
  }
}
// fragment along a row: element j = X[row][16 s + 8 h + j]
__device__ __forceinline__ bf16x8 read_row(const char* img, int row, int s, int h) {
  return *reinterpret_cast<const bf16x8*>(img + img_off(row, 2 * s + h));
}
// fragment down a column in the k order of an accumulator fed back as an operand:
//   element j = X[r0 + 16 s + 8 (j >> 2) + 4 h + (j & 3)][c0 + (lane & 31)].
// Each ds_read_b64_tr_b16 gives 16-lane group g the 4 x 16 block at rows r0 + 16 s + 4 (g >> 1) (+ 8 for
// elements 4..7), columns c0 + 16 (g & 1) .. + 15, column-major (lane i of the group gets column i, row q in
// element q); lane 4q + p of the group supplies the address of row q, columns 4p .. 4p + 3.
__device__ __forceinline__ bf16x8 read_tr(char* img, int r0, int c0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int row = r0 + 16 * s + 4 * (g >> 1) + (i >> 2);
  const int col = c0 + 16 * (g & 1) + 4 * (i & 3);
  const int sub = 2 * (col & 7);  // 0 or 8 bytes into the chunk
  const bf16x4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4v*)(img + img_off(row, col >> 3) + sub));
  const bf16x4v hi =
      __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4v*)(img + img_off(row + 8, col >> 3) + sub));
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = lo[j];
    r[4 + j] = hi[j];
  }
  return r;
}

struct AttnArgs {
  const __hip_bfloat16 *q, *k, *v;
  int64_t ldq, ldk, ldv;
  const float* gate;  // [B, T, H]
  const float* pb;    // [H, T, ldpb], ldpb >= 32 * ceil(T / 32), rows 16-byte aligned
  int64_t ldpb;
  const int64_t* seed_dev;
  int salt;
  uint32_t thr;   // p * 2^32 (0: no dropout)
  float inv_keep;  // 1 / (1 - p)
  float scale;
  int B, T, H;
};

struct AttnBwdArgs {
  const __hip_bfloat16* dO;
  int64_t lddo;
  const float* lse;  // [B, H, T]
  float* D;          // [B, H, T]: written by the dQ kernel, read by the dK/dV kernel
};

template <bool kDrop>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a, __hip_bfloat16* __restrict__ o, int64_t ldo,
                                                       float* __restrict__ lse) {
  extern __shared__ __attribute__((aligned(16))) char at_lds[];
  const int T = a.T, H = a.H, nt = (T + AT_TILE - 1) / AT_TILE;
  const int head = blockIdx.y, b = blockIdx.z;
  const int64_t col0 = (int64_t)head * AT_DH;
  char* Ks = at_lds;
  char* Vs = at_lds + nt * AT_TILE_BYTES;
  stage_image(Ks, a.k, a.ldk, b, T, col0, nt);
  stage_image(Vs, a.v, a.ldv, b, T, col0, nt);
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int qb = blockIdx.x * AT_WAVES + w;
  if (qb >= nt) return;  // no barrier follows
  const int qi = qb * AT_TILE + r;
  const bool qvalid = qi < T;
  const int qc = qvalid ? qi : T - 1;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = load8(a.q + ((int64_t)b * T + qc) * a.ldq + col0 + 16 * s + 8 * hh, qvalid);
  const float g = a.gate[((int64_t)b * T + qc) * H + head];
  const float* pbrow = a.pb + ((int64_t)head * T + qc) * a.ldpb;
  const uint64_t seed = kDrop ? attn_seed(a.seed_dev, a.salt) : 0;
  const uint64_t ibase = (((uint64_t)b * H + head) * T + qc) * (uint64_t)T;
  float m = -INFINITY, l = 0.f;
  f32x16 oacc[2] = {zero16(), zero16()};
  for (int kb = 0; kb < nt; ++kb) {
    f32x16 sacc = zero16();
#pragma unroll
    for (int s = 0; s < 4; ++s) sacc = mfma32(read_row(Ks, kb * AT_TILE + r, s, hh), qf[s], sacc);
    float sv[16], pbv[16];
    load_pb16(pbrow, kb, hh, pbv);
    float mloc = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = kb * AT_TILE + crow(i, hh);
      float x = -INFINITY;
      if (key < T) x = fmaf(sacc[i], a.scale, g * pbv[i]);
      sv[i] = x;
      mloc = fmaxf(mloc, x);
    }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float mnew = fmaxf(m, mloc);
    const float alpha = mnew == -INFINITY ? 1.f : __expf(m - mnew);
    float lsum = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = sv[i] == -INFINITY ? 0.f : __expf(sv[i] - mnew);
      lsum += p;
      if (kDrop) {
        const int key = kb * AT_TILE + crow(i, hh);
        sv[i] = drop_keep(seed, ibase + key, a.thr) ? p * a.inv_keep : 0.f;
      } else {
        sv[i] = p;
      }
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
      const bf16x8 pf = pack8(sv + 8 * s);
#pragma unroll
      for (int db = 0; db < 2; ++db) oacc[db] = mfma32(read_tr(Vs, kb * AT_TILE, db * 32, s, lane), pf, oacc[db]);
    }
  }
  if (qvalid) {
    const float inv = 1.f / l;
    __hip_bfloat16* orow = o + ((int64_t)b * T + qi) * ldo + col0;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int i = 0; i < 16; ++i) orow[db * 32 + crow(i, hh)] = __float2bfloat16(oacc[db][i] * inv);
    if (hh == 0) lse[((int64_t)b * H + head) * T + qi] = m + __logf(l);
  }
}

// query-stationary: dQ, d gate and D = rowsum(dO o O) of the wave's 32 query rows
template <bool kDrop>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnArgs a, AttnBwdArgs g,
                                                          const __hip_bfloat16* __restrict__ O, int64_t ldo,
                                                          __hip_bfloat16* __restrict__ dq, int64_t ldg,
                                                          float* __restrict__ dgate) {
  extern __shared__ __attribute__((aligned(16))) char at_lds[];
  const int T = a.T, H = a.H, nt = (T + AT_TILE - 1) / AT_TILE;
  const int head = blockIdx.y, b = blockIdx.z;
  const int64_t col0 = (int64_t)head * AT_DH;
  char* Ks = at_lds;
  char* Vs = at_lds + nt * AT_TILE_BYTES;
  stage_image(Ks, a.k, a.ldk, b, T, col0, nt);
  stage_image(Vs, a.v, a.ldv, b, T, col0, nt);
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int qb = blockIdx.x * AT_WAVES + w;
  if (qb >= nt) return;
  const int qi = qb * AT_TILE + r;
  const bool qvalid = qi < T;
  const int qc = qvalid ? qi : T - 1;
  const int64_t trow = (int64_t)b * T + qc;
  bf16x8 qf[4], dof[4];
  float dpart = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = load8(a.q + trow * a.ldq + col0 + 16 * s + 8 * hh, qvalid);
    dof[s] = load8(g.dO + trow * g.lddo + col0 + 16 * s + 8 * hh, qvalid);
    const bf16x8 of = load8(O + trow * ldo + col0 + 16 * s + 8 * hh, qvalid);
#pragma unroll
    for (int j = 0; j < 8; ++j) dpart = fmaf((float)dof[s][j], (float)of[j], dpart);
  }
  const float Dq = dpart + __shfl_xor(dpart, 32, 64);
  const int64_t bh = (int64_t)b * H + head;
  if (hh == 0 && qvalid) g.D[bh * T + qi] = Dq;
  const float gq = a.gate[trow * H + head];
  const float lq = g.lse[bh * T + qc];
  const float* pbrow = a.pb + ((int64_t)head * T + qc) * a.ldpb;
  const uint64_t seed = kDrop ? attn_seed(a.seed_dev, a.salt) : 0;
  const uint64_t ibase = ((uint64_t)bh * T + qc) * (uint64_t)T;
  f32x16 dqacc[2] = {zero16(), zero16()};
  float dg = 0.f;
  for (int kb = 0; kb < nt; ++kb) {
    f32x16 S = zero16(), dP = zero16();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      S = mfma32(read_row(Ks, kb * AT_TILE + r, s, hh), qf[s], S);
      dP = mfma32(read_row(Vs, kb * AT_TILE + r, s, hh), dof[s], dP);
    }
    float dS[16], pbt[16];
    load_pb16(pbrow, kb, hh, pbt);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = kb * AT_TILE + crow(i, hh);
      float ds = 0.f;
      if (key < T && qvalid) {
        const float p = __expf(fmaf(S[i], a.scale, gq * pbt[i]) - lq);
        float mk = 1.f;
        if (kDrop) mk = drop_keep(seed, ibase + key, a.thr) ? a.inv_keep : 0.f;
        ds = p * (dP[i] * mk - Dq);
        dg = fmaf(ds, pbt[i], dg);
      }
      dS[i] = ds;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 xs = pack8(dS + 8 * s);
#pragma unroll
      for (int db = 0; db < 2; ++db) dqacc[db] = mfma32(read_tr(Ks, kb * AT_TILE, db * 32, s, lane), xs, dqacc[db]);
    }
  }
  dg += __shfl_xor(dg, 32, 64);
  if (qvalid) {
    __hip_bfloat16* row = dq + ((int64_t)b * T + qi) * ldg + col0;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int i = 0; i < 16; ++i) row[db * 32 + crow(i, hh)] = __float2bfloat16(dqacc[db][i] * a.scale);
    if (hh == 0) dgate[((int64_t)b * T + qi) * H + head] = dg;
  }
}

// key-stationary: dK and dV of the wave's 32 keys
template <bool kDrop>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(AttnArgs a, AttnBwdArgs g,
                                                            __hip_bfloat16* __restrict__ dk,
                                                            __hip_bfloat16* __restrict__ dv, int64_t ldg) {
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
  stage_image(Qs, a.q, a.ldq, b, T, col0, nt);
  stage_image(dOs, g.dO, g.lddo, b, T, col0, nt);
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
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = load8(a.k + ((int64_t)b * T + key) * a.ldk + col0 + 16 * s + 8 * hh, kvalid);
    vf[s] = load8(a.v + ((int64_t)b * T + key) * a.ldv + col0 + 16 * s + 8 * hh, kvalid);
  }
  const uint64_t seed = kDrop ? attn_seed(a.seed_dev, a.salt) : 0;
  const uint64_t kbase = (uint64_t)bh * T * (uint64_t)T + (uint64_t)key;
  const float* pbcol = a.pb + (int64_t)head * T * a.ldpb + key;
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
          const float sc = fmaf(S[i], a.scale, gv[e] * pbcol[(int64_t)qi * a.ldpb]);
          p = __expf(sc - lv[e]);
          float mk = 1.f;
          if (kDrop) mk = drop_keep(seed, kbase + (uint64_t)(qi * T), a.thr) ? a.inv_keep : 0.f;
          ds = p * (dP[i] * mk - dd[e]);
          p *= mk;
        }
        P[i] = p;
        dS[i] = ds;
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 xp = pack8(P + 8 * s), xs = pack8(dS + 8 * s);
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
        dk[off] = __float2bfloat16(dkacc[db][i] * a.scale);
        dv[off] = __float2bfloat16(dvacc[db][i]);
      }
    }
  }
}

// element-wise dropout mask of the same hash (tests only): keep[b, h, i, j] in {0, 1}
__global__ void attn_mask_kernel(const int64_t* seed_dev, int salt, uint32_t thr, uint8_t* keep, int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) keep[t] = drop_keep(attn_seed(seed_dev, salt), (uint64_t)t, thr) ? 1 : 0;
}

inline AttnArgs make_args(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                          const float* gate, const float* pb, int64_t ldpb, const int64_t* seed_dev, int salt,
                          float p_drop, float scale, int B, int T, int H) {
  AttnArgs a;
  a.q = (const __hip_bfloat16*)q;
  a.k = (const __hip_bfloat16*)k;
  a.v = (const __hip_bfloat16*)v;
  a.ldq = ldq;
  a.ldk = ldk;
  a.ldv = ldv;
  a.gate = gate;
  a.pb = pb;
  a.ldpb = ldpb;
  a.seed_dev = seed_dev;
  a.salt = salt;
  const double t = (double)p_drop * 4294967296.0;
  a.thr = p_drop > 0.f ? (uint32_t)(t >= 4294967295.0 ? 4294967295.0 : t) : 0u;
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

static bool pb_ok(const float* pb, int64_t ldpb, int T) {
  return ((uintptr_t)pb & 15) == 0 && ldpb >= (int64_t)((T + AT_TILE - 1) / AT_TILE) * AT_TILE && ldpb % 4 == 0;
}

// the dK/dV kernel's images and row scalars exceed the default 64 KB dynamic-LDS cap at T = 256
static int attn_allow_lds(const void* fn, bool& done) {
  if (done) return RDX_OK;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return (int)e;
  done = true;
  return RDX_OK;
}

template <bool kDrop>
static int launch_fwd(dim3 grid, size_t lds, hipStream_t st, const AttnArgs& a, __hip_bfloat16* o, int64_t ldo,
                      float* lse) {
  static bool done = false;
  const int rc = attn_allow_lds(reinterpret_cast<const void*>(&attn_fwd_kernel<kDrop>), done);
  if (rc != RDX_OK) return rc;
  hipLaunchKernelGGL((attn_fwd_kernel<kDrop>), grid, dim3(AT_WAVES * 64), lds, st, a, o, ldo, lse);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

template <bool kDrop>
static int launch_bwd(dim3 grid, size_t lds_dq, size_t lds_kv, hipStream_t st, const AttnArgs& a,
                      const AttnBwdArgs& g, const __hip_bfloat16* o, int64_t ldo, __hip_bfloat16* dq,
                      __hip_bfloat16* dk, __hip_bfloat16* dv, int64_t ldg, float* dgate) {
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
                            const float* gate, const float* pos_bias, int64_t ldpb, const int64_t* seed_dev,
                            int salt, float p_drop, float scale, void* o, int64_t ldo, float* lse, int B, int T, int H,
                            int head_dim, void* stream) {
  RDX_REQUIRE(attn_ok(q, ldq, k, ldk, v, ldv, B, T, H) && gate && pos_bias && o && lse && ldo >= (int64_t)H * AT_DH);
  RDX_REQUIRE(pb_ok(pos_bias, ldpb, T));
  RDX_REQUIRE(p_drop >= 0.f && p_drop < 1.f && (p_drop == 0.f || seed_dev));
  if (head_dim != AT_DH || T > AT_MAXNT * AT_TILE) return RDX_EUNSUPPORTED;
  const AttnArgs a = make_args(q, ldq, k, ldk, v, ldv, gate, pos_bias, ldpb, seed_dev, salt, p_drop, scale, B, T, H);
  const int nt = (T + AT_TILE - 1) / AT_TILE;
  const dim3 grid((nt + AT_WAVES - 1) / AT_WAVES, H, B);
  const size_t lds = 2 * (size_t)nt * AT_TILE_BYTES;
  return a.thr ? launch_fwd<true>(grid, lds, as_stream(stream), a, (__hip_bfloat16*)o, ldo, lse)
               : launch_fwd<false>(grid, lds, as_stream(stream), a, (__hip_bfloat16*)o, ldo, lse);
}

extern "C" int rdx_attn_bwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                            const float* gate, const float* pos_bias, int64_t ldpb, const int64_t* seed_dev,
                            int salt, float p_drop, float scale, const void* o, int64_t ldo, const float* lse,
                            const void* dout, int64_t lddo, float* D, void* dq, void* dk, void* dv, int64_t ldg,
                            float* dgate, int B, int T, int H, int head_dim, void* stream) {
  RDX_REQUIRE(attn_ok(q, ldq, k, ldk, v, ldv, B, T, H) && gate && pos_bias && o && lse && dout && D);
  RDX_REQUIRE(pb_ok(pos_bias, ldpb, T));
  RDX_REQUIRE(dq && dk && dv && dgate && ldg >= (int64_t)H * AT_DH && ldg % 8 == 0 && lddo % 8 == 0 && ldo % 8 == 0);
  RDX_REQUIRE(((uintptr_t)o & 15) == 0 && ((uintptr_t)dout & 15) == 0);
  RDX_REQUIRE(p_drop >= 0.f && p_drop < 1.f && (p_drop == 0.f || seed_dev));
  if (head_dim != AT_DH || T > AT_MAXNT * AT_TILE) return RDX_EUNSUPPORTED;
  const AttnArgs a = make_args(q, ldq, k, ldk, v, ldv, gate, pos_bias, ldpb, seed_dev, salt, p_drop, scale, B, T, H);
  const AttnBwdArgs g{(const __hip_bfloat16*)dout, lddo, lse, D};
  const int nt = (T + AT_TILE - 1) / AT_TILE;
  const dim3 grid((nt + AT_WAVES - 1) / AT_WAVES, H, B);
  const size_t lds_dq = 2 * (size_t)nt * AT_TILE_BYTES;
  const size_t lds_kv = lds_dq + 3 * (size_t)nt * AT_TILE * sizeof(float);
  return a.thr ? launch_bwd<true>(grid, lds_dq, lds_kv, as_stream(stream), a, g, (const __hip_bfloat16*)o, ldo,
                                  (__hip_bfloat16*)dq, (__hip_bfloat16*)dk, (__hip_bfloat16*)dv, ldg, dgate)
               : launch_bwd<false>(grid, lds_dq, lds_kv, as_stream(stream), a, g, (const __hip_bfloat16*)o, ldo,
                                   (__hip_bfloat16*)dq, (__hip_bfloat16*)dk, (__hip_bfloat16*)dv, ldg, dgate);
}

extern "C" int rdx_attn_dropout_mask(const int64_t* seed_dev, int salt, float p_drop, uint8_t* keep, int64_t n,
                                     void* stream) {
  RDX_REQUIRE(seed_dev && keep && n > 0 && p_drop >= 0.f && p_drop < 1.f);
  const AttnArgs a = make_args(nullptr, 0, nullptr, 0, nullptr, 0, nullptr, nullptr, 0, seed_dev, salt, p_drop, 1.f, 1, 1, 1);
  hipLaunchKernelGGL(attn_mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), seed_dev,
                     salt, a.thr, keep, n);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
