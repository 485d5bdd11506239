// Fused pieces of the detector head (src/models/DualStreamSEMamba.py:492-531, SELayer inside DualStreamFusion) for
// the training passes under autocast: the squeeze-excitation over time as one launch forward and two backward.
//
//   m = mean_t(x)              [B, C]   (AdaptiveAvgPool1d(1) of the 16-bit x: fp32 sum, one rounding)
//   h = relu(m W1^T)           [B, R]   (fc1, R = C / 16, no bias; the GEMM rounds once to 16 bits)
//   s = sigmoid(h W2^T)        [B, C]   (fc2, no bias; rounded, sigmoid rounded)
//   y = x * s                  [B, T, C]
// Every value autocast keeps in 16 bits is rounded to the storage type where autocast's op would round it, so the
// launches reproduce the module path's values up to the order of fp32 sums. Backward (one workgroup per utterance,
// then a fixed-order reduction): ds = sum_t round(dy x), dz = round(ds s (1 - s)), dh = round(dz W2) (relu'),
// dm = round(dh W1), dx = round(dy s) + round(dm / T) (the two branches' gradients added in 16 bits, as autograd
// adds them); dW2 = sum_b dz^T h and dW1 = sum_b dh^T m in fp32, per-utterance partial rows summed in utterance
// order and ADDED into the caller's fp32 .grad buffers.
// The torch ops this replaces (mean, two small GEMMs, relu, sigmoid, the product; their backward kernels, the
// broadcast-sum and cast, the two-branch add) were ~20 launches per pass for ~58 KB of activations per utterance.
#include "common.h"

namespace rdx {

constexpr int SE_T = 256;        // threads
constexpr int SE_CMAX = 256;     // channels
constexpr int SE_RMAX = 16;      // squeeze width
constexpr int SE_CH = 8;         // channels per 16-byte chunk

struct SeArgs {
  const hst* x;     // [B, T, C]
  const hst* w1;    // [R, C] (16-bit, autocast's cast of fc1.weight)
  const hst* w2;    // [C, R]
  hst* y;           // [B, T, C]
  hst* m;           // [B, C] saved for the backward
  hst* h;           // [B, R]
  hst* s;           // [B, C]
  int B, T, C, R;
};

// column sums over t of rows [T, C] (16-byte chunks): thread (chunk q, row group g) sums rows g, g + G, ...; the
// G partial sums of a chunk reduced through LDS. f(t, chunk j) -> 8 fp32 values added.
template <class F>
__device__ __forceinline__ void se_colsum(float* red, float* out, int T, int C, F f) {
  const int nq = C / SE_CH, G = SE_T / nq;   // nq <= 32 chunks, G >= 8 row groups
  const int q = threadIdx.x % nq, g = threadIdx.x / nq;
  float acc[SE_CH];
#pragma unroll
  for (int k = 0; k < SE_CH; ++k) acc[k] = 0.f;
  if (g < G)
    for (int t = g; t < T; t += G) f(t, q, acc);
  __syncthreads();
  if (g < G)
#pragma unroll
    for (int k = 0; k < SE_CH; ++k) red[(g * nq + q) * SE_CH + k] = acc[k];
  __syncthreads();
  if (threadIdx.x < C) {
    const int c = threadIdx.x, qq = c / SE_CH, k = c % SE_CH;
    float sum = 0.f;
    for (int gg = 0; gg < G; ++gg) sum += red[(gg * nq + qq) * SE_CH + k];
    out[c] = sum;
  }
  __syncthreads();
}

__device__ __forceinline__ void se_unpack(uint4 u, float* v) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = hlo(w[j]);
    v[2 * j + 1] = hhi(w[j]);
  }
}

// the utterance's [T, C] 16-bit rows into an LDS image (256 threads; every 16-byte load of a batch of 8 per thread
// in flight before its LDS stores, from clamped addresses): the passes over the rows then read LDS, not one
// dependent global round trip per row group or per row
__device__ __forceinline__ void head_stage(char* img, const hst* fb, int T, int C) {
  const int n = T * C / 8;
  const uint4* src = reinterpret_cast<const uint4*>(fb);
  for (int base = 0; base < n; base += 8 * 256) {
    uint4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = base + j * 256 + threadIdx.x;
      v[j] = src[i < n ? i : n - 1];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = base + j * 256 + threadIdx.x;
      if (i < n) reinterpret_cast<uint4*>(img)[i] = v[j];
    }
  }
}
__global__ __launch_bounds__(SE_T) void se_fwd_kernel(SeArgs a) {
  __shared__ float red[SE_T * SE_CH];
  __shared__ float sm[SE_CMAX], sh[SE_RMAX], ss[SE_CMAX];
  extern __shared__ __attribute__((aligned(16))) char se_lds[];   // x image [T][C]
  __shared__ hst sw1[SE_RMAX * SE_CMAX], sw2[SE_CMAX * SE_RMAX];
  const int b = blockIdx.x, T = a.T, C = a.C, R = a.R;
  const uint4* ximg = reinterpret_cast<const uint4*>(se_lds);
  head_stage(se_lds, a.x + (int64_t)b * T * C, T, C);
  for (int i = threadIdx.x; i < R * C; i += SE_T) {
    sw1[i] = a.w1[i];
    sw2[i] = a.w2[i];
  }
  __syncthreads();
  se_colsum(red, sm, T, C, [&](int t, int q, float* acc) {
    float v[SE_CH];
    se_unpack(ximg[t * (C / SE_CH) + q], v);
#pragma unroll
    for (int k = 0; k < SE_CH; ++k) acc[k] += v[k];
  });
  if (threadIdx.x < C) {
    const int c = threadIdx.x;
    const float mv = hround(sm[c] * (1.0f / (float)T));
    sm[c] = mv;
    a.m[(int64_t)b * C + c] = f2h(mv);
  }
  __syncthreads();
  {   // fc1 + relu: 16 lanes per output j (lane l takes c = l, l + 16, ...; the 16 partials added by a butterfly),
      // weights read from the image staged with x
    const int j = threadIdx.x >> 4, l = threadIdx.x & 15;
    float acc = 0.f;
    if (j < R)
      for (int c = l; c < C; c += 16) acc = fmaf(sm[c], h2f(sw1[j * C + c]), acc);
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) acc += __shfl_xor(acc, o, 64);
    if (j < R && l == 0) {
      const float hv = fmaxf(hround(acc), 0.f);
      sh[j] = hv;
      a.h[(int64_t)b * R + j] = f2h(hv);
    }
  }
  __syncthreads();
  if (threadIdx.x < C) {   // fc2 + sigmoid
    const int c = threadIdx.x;
    float acc = 0.f;
    for (int j = 0; j < R; ++j) acc = fmaf(sh[j], h2f(sw2[c * R + j]), acc);
    const float z = hround(acc);
    const float sv = hround(1.0f / (1.0f + __expf(-z)));
    ss[c] = sv;
    a.s[(int64_t)b * C + c] = f2h(sv);
  }
  __syncthreads();
  // y = x * s: 16-byte chunks, consecutive threads on consecutive chunks
  const int nq = C / SE_CH;
  hst* yb = a.y + (int64_t)b * T * C;
  for (int i = threadIdx.x; i < T * nq; i += SE_T) {
    const int t = i / nq, q = i % nq;
    float v[SE_CH];
    se_unpack(ximg[i], v);
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = hpack2(v[2 * j] * ss[q * SE_CH + 2 * j], v[2 * j + 1] * ss[q * SE_CH + 2 * j + 1]);
    *reinterpret_cast<uint4*>(yb + (int64_t)t * C + q * SE_CH) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

struct SeBwdArgs {
  const hst* dy;    // [B, T, C]
  const hst* x;
  const hst* w1;
  const hst* w2;
  const hst* m;
  const hst* h;
  const hst* s;
  hst* dx;          // [B, T, C]
  float* part;      // [B, R * C + C * R]: dW1 [R, C] then dW2 [C, R], per utterance
  int B, T, C, R;
};

__global__ __launch_bounds__(SE_T) void se_bwd_kernel(SeBwdArgs a) {
  __shared__ float red[SE_T * SE_CH];
  __shared__ float sds[SE_CMAX], sdz[SE_CMAX], sdh[SE_RMAX], sdm[SE_CMAX], ssv[SE_CMAX];
  extern __shared__ __attribute__((aligned(16))) char se_lds[];   // dy image [T][C], then x image [T][C]
  const int b = blockIdx.x, T = a.T, C = a.C, R = a.R;
  const uint4* dimg = reinterpret_cast<const uint4*>(se_lds);
  const uint4* ximg = reinterpret_cast<const uint4*>(se_lds + T * C * 2);
  __shared__ hst sw1[SE_RMAX * SE_CMAX], sw2[SE_CMAX * SE_RMAX];
  __shared__ float shv[SE_RMAX], smv[SE_CMAX];
  head_stage(se_lds, a.dy + (int64_t)b * T * C, T, C);
  head_stage(se_lds + T * C * 2, a.x + (int64_t)b * T * C, T, C);
  for (int i = threadIdx.x; i < R * C; i += SE_T) {
    sw1[i] = a.w1[i];
    sw2[i] = a.w2[i];
  }
  if (threadIdx.x < R) shv[threadIdx.x] = h2f(a.h[(int64_t)b * R + threadIdx.x]);
  if (threadIdx.x < C) smv[threadIdx.x] = h2f(a.m[(int64_t)b * C + threadIdx.x]);
  __syncthreads();
  // ds = sum_t round(dy * x)
  se_colsum(red, sds, T, C, [&](int t, int q, float* acc) {
    float d[SE_CH], v[SE_CH];
    se_unpack(dimg[t * (C / SE_CH) + q], d);
    se_unpack(ximg[t * (C / SE_CH) + q], v);
#pragma unroll
    for (int k = 0; k < SE_CH; ++k) acc[k] += hround(d[k] * v[k]);
  });
  float* prow = a.part + (int64_t)b * (2 * R * C);
  if (threadIdx.x < C) {   // sigmoid backward
    const int c = threadIdx.x;
    const float sv = h2f(a.s[(int64_t)b * C + c]);
    ssv[c] = sv;
    sdz[c] = hround(hround(sds[c]) * (sv * (1.0f - sv)));
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C * R; i += SE_T) prow[R * C + i] = sdz[i / R] * shv[i % R];   // dW2 [C, R] = dz h^T
  {   // fc2's input gradient, relu': 16 lanes per j, as the forward's fc1
    const int j = threadIdx.x >> 4, l = threadIdx.x & 15;
    float acc = 0.f;
    if (j < R)
      for (int c = l; c < C; c += 16) acc = fmaf(sdz[c], h2f(sw2[c * R + j]), acc);
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) acc += __shfl_xor(acc, o, 64);
    if (j < R && l == 0) sdh[j] = shv[j] > 0.f ? hround(acc) : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < R * C; i += SE_T) prow[i] = sdh[i / C] * smv[i % C];   // dW1 [R, C] = dh m^T
  if (threadIdx.x < C) {   // fc1's input gradient; the mean's backward
    const int c = threadIdx.x;
    float acc = 0.f;
    for (int j = 0; j < R; ++j) acc = fmaf(sdh[j], h2f(sw1[j * C + c]), acc);
    sdm[c] = hround(hround(acc) / (float)T);
  }
  __syncthreads();
  const int nq = C / SE_CH;
  hst* dxb = a.dx + (int64_t)b * T * C;
  for (int i = threadIdx.x; i < T * nq; i += SE_T) {
    const int t = i / nq, q = i % nq;
    float d[SE_CH];
    se_unpack(dimg[i], d);
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c0 = q * SE_CH + 2 * j;
      o[j] = hpack2(hround(d[2 * j] * ssv[c0]) + sdm[c0], hround(d[2 * j + 1] * ssv[c0 + 1]) + sdm[c0 + 1]);
    }
    *reinterpret_cast<uint4*>(dxb + (int64_t)t * C + q * SE_CH) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// grad[i] += sum_b part[b][i] (utterance order), i < n: dW1 into g1 [R * C], then dW2 into g2 [C * R]
__global__ __launch_bounds__(256) void se_wgrad_kernel(const float* __restrict__ part, int B, int n1, int n2,
                                                       float* __restrict__ g1, float* __restrict__ g2) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n1 + n2) return;
  float sum = 0.f;
#pragma unroll 8
  for (int b = 0; b < B; ++b) sum += part[(int64_t)b * (n1 + n2) + i];   // in order; 8 loads in flight
  if (i < n1) g1[i] += sum;
  else g2[i - n1] += sum;
}


// ---- Attention pooling of the head (src/models/DualStreamSEMamba.py:700-770, Model.forward's tail) under autocast:
//   z = round(f w^T + b) [B, T] (attention_pool, a 1-output linear), a = softmax_t(z) in fp32, a16 = round(a),
//   feat = round(a16^T f) [B, C] (autocast's bmm on the 16-bit attention weights).
// One workgroup per utterance, f [T, C] read twice (scores, then the weighted sum). Backward from dfeat [B, C]:
//   da = round(f dfeat) [T], df1 = round(a16 dfeat^T); dz = round(a (da - sum_t a da)) (softmax backward in fp32 on the
//   fp32 output, then the cast back to z's dtype); df2 = round(dz w); df = round(df1 + df2) (the two branches' 16-bit
//   add); dw = sum dz f, db = sum dz in fp32, per-utterance partials summed in utterance order into .grad.
constexpr int AP_T = 256;
constexpr int AP_TMAX = 1024;

struct ApArgs {
  const hst* f;      // [B, T, C]
  const hst* w;      // [C] (16-bit)
  const hst* bias;   // [1] (16-bit) or null
  hst* feat;         // [B, C]
  float* a;          // [B, T] fp32 softmax (saved)
  int B, T, C;
};

__device__ __forceinline__ float ap_block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < AP_T / 64; ++i) s += red[i];
  return s;
}
__device__ __forceinline__ float ap_block_max(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = red[0];
#pragma unroll
  for (int i = 1; i < AP_T / 64; ++i) s = fmaxf(s, red[i]);
  return s;
}

// f [T, C] of the utterance staged in LDS once (every 16-byte load of a batch in flight before its stores), then
// read from there by the score pass (a thread per row) and the weighted sum (a thread per (8-channel chunk, row
// group), the groups' partial sums added in group order): the global reads were one dependent round trip per row
// and per step of a per-channel loop over T.
constexpr int AP_LDS_MAX = 128 * 1024;   // f image bytes
static_assert(AP_LDS_MAX + 2 * 1024 * 4 + 2 * 1024 * 4 + 8 * 256 * 4 + 64 <= 160 * 1024, "LDS budget");
// sum over t of wt(t) * f[t, chunk q] for this thread's (chunk, row group), the groups' partials through `red`
// ([G][C] floats) added in group order into out[c] (thread c < C)
template <class Wt>
__device__ __forceinline__ void ap_colsum(const char* img, float* red, float* out, int T, int C, Wt wt) {
  const int nq = C / 8, G = AP_T / nq;
  const int q = threadIdx.x % nq, g = threadIdx.x / nq;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (g < G)
    for (int t = g; t < T; t += G) {
      float v[8];
      se_unpack(reinterpret_cast<const uint4*>(img)[t * nq + q], v);
      const float wv = wt(t);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = fmaf(wv, v[k], acc[k]);
    }
  __syncthreads();
  if (g < G)
#pragma unroll
    for (int k = 0; k < 8; ++k) red[g * C + 8 * q + k] = acc[k];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += AP_T) {
    float sum = 0.f;
    for (int gg = 0; gg < G; ++gg) sum += red[gg * C + c];
    out[c] = sum;
  }
  __syncthreads();
}
// dynamic LDS: f image [T][C] 16-bit | per-row floats x 2 [AP_TMAX] | per-channel floats x 2 [1024] | the row
// groups' partials [G][C] (G C = 8 G nq <= 8 AP_T floats) | block-reduction scratch
__host__ __device__ constexpr int ap_lds_bytes(int T, int C) {
  return T * C * 2 + 2 * AP_TMAX * 4 + 2 * 1024 * 4 + 8 * AP_T * 4 + 64;
}

__global__ __launch_bounds__(AP_T) void attn_pool_fwd_kernel(ApArgs a) {
  extern __shared__ __attribute__((aligned(16))) char ap_lds[];
  const int b = blockIdx.x, T = a.T, C = a.C;
  char* img = ap_lds;
  float* sz = reinterpret_cast<float*>(ap_lds + T * C * 2);
  float* sw = sz + 2 * AP_TMAX;
  float* sout = sw + 1024;
  float* red2 = sout + 1024;
  float* red = red2 + 8 * AP_T;
  head_stage(img, a.f + (int64_t)b * T * C, T, C);
  for (int c = threadIdx.x; c < C; c += AP_T) sw[c] = h2f(a.w[c]);
  const float bias = a.bias ? h2f(a.bias[0]) : 0.f;
  __syncthreads();
  const int nq = C / 8;
  for (int t = threadIdx.x; t < T; t += AP_T) {   // scores: a thread per row
    float acc = 0.f;
    for (int q = 0; q < nq; ++q) {
      float v[8];
      se_unpack(reinterpret_cast<const uint4*>(img)[t * nq + q], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc = fmaf(v[k], sw[8 * q + k], acc);
    }
    sz[t] = hround(acc + bias);
  }
  __syncthreads();
  float mx = -INFINITY;
  for (int t = threadIdx.x; t < T; t += AP_T) mx = fmaxf(mx, sz[t]);
  mx = ap_block_max(mx, red);
  float sum = 0.f;
  for (int t = threadIdx.x; t < T; t += AP_T) {
    const float e = __expf(sz[t] - mx);
    sz[t] = e;
    sum += e;
  }
  sum = ap_block_sum(sum, red);
  const float inv = 1.0f / sum;
  __syncthreads();
  for (int t = threadIdx.x; t < T; t += AP_T) {
    const float av = sz[t] * inv;
    a.a[(int64_t)b * T + t] = av;
    sz[t] = hround(av);
  }
  __syncthreads();
  ap_colsum(img, red2, sout, T, C, [&](int t) { return sz[t]; });
  for (int c = threadIdx.x; c < C; c += AP_T) a.feat[(int64_t)b * C + c] = f2h(sout[c]);
}

struct ApBwdArgs {
  const hst* f;
  const hst* w;
  const float* a;
  const hst* dfeat;   // [B, C]
  hst* df;            // [B, T, C]
  float* part;        // [B, C + 1]: dw then db per utterance
  int B, T, C;
};

__global__ __launch_bounds__(AP_T) void attn_pool_bwd_kernel(ApBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char ap_lds[];
  const int b = blockIdx.x, T = a.T, C = a.C, nq = C / 8;
  char* img = ap_lds;
  float* sa = reinterpret_cast<float*>(ap_lds + T * C * 2);
  float* sdz = sa + AP_TMAX;
  float* sdf = sdz + AP_TMAX;
  float* sw = sdf + 1024;
  float* red2 = sw + 1024;
  float* red = red2 + 8 * AP_T;
  head_stage(img, a.f + (int64_t)b * T * C, T, C);
  for (int c = threadIdx.x; c < C; c += AP_T) {
    sdf[c] = h2f(a.dfeat[(int64_t)b * C + c]);
    sw[c] = h2f(a.w[c]);
  }
  for (int t = threadIdx.x; t < T; t += AP_T) sa[t] = a.a[(int64_t)b * T + t];
  __syncthreads();
  for (int t = threadIdx.x; t < T; t += AP_T) {   // da = round(f dfeat): a thread per row
    float acc = 0.f;
    for (int q = 0; q < nq; ++q) {
      float v[8];
      se_unpack(reinterpret_cast<const uint4*>(img)[t * nq + q], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc = fmaf(v[k], sdf[8 * q + k], acc);
    }
    sdz[t] = hround(acc);
  }
  __syncthreads();
  float dot = 0.f;
  for (int t = threadIdx.x; t < T; t += AP_T) dot = fmaf(sa[t], sdz[t], dot);
  dot = ap_block_sum(dot, red);
  __syncthreads();
  float dbs = 0.f;
  for (int t = threadIdx.x; t < T; t += AP_T) {
    const float dz = hround(sa[t] * (sdz[t] - dot));
    sdz[t] = dz;
    dbs += dz;
  }
  dbs = ap_block_sum(dbs, red);
  __syncthreads();
  // df = round(round(a16 dfeat) + round(dz w)): 16-byte chunks, every (row, chunk) in parallel
  hst* dfb = a.df + (int64_t)b * T * C;
  for (int i = threadIdx.x; i < T * nq; i += AP_T) {
    const int t = i / nq, q = i - t * nq;
    const float a16 = hround(sa[t]), dz = sdz[t];
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = 8 * q + 2 * k;
      o[k] = hpack2(hround(a16 * sdf[c]) + hround(dz * sw[c]), hround(a16 * sdf[c + 1]) + hround(dz * sw[c + 1]));
    }
    reinterpret_cast<uint4*>(dfb)[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
  // dw = sum_t dz f (row groups added in group order), db = sum_t dz
  float* prow = a.part + (int64_t)b * (C + 1);
  ap_colsum(img, red2, prow, T, C, [&](int t) { return sdz[t]; });
  if (threadIdx.x == 0) prow[C] = dbs;
}

__global__ __launch_bounds__(256) void ap_wgrad_kernel(const float* __restrict__ part, int B, int C,
                                                       float* __restrict__ dw, float* __restrict__ db) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i > C) return;
  float s = 0.f;
#pragma unroll 8
  for (int b = 0; b < B; ++b) s += part[(int64_t)b * (C + 1) + i];   // in order; 8 loads in flight
  if (i < C) dw[i] += s;
  else if (db) db[0] += s;
}

// ---- DualStreamFusion's time alignment and concatenation (src/models/DualStreamSEMamba.py:537-637) under autocast:
//   out[b, t] = [fw[b, t, :] | fs[b, idx(t), :]],  idx(t) = min(floor(t * (T2 / T1)), T2 - 1)  (F.interpolate's
// 'nearest' index, the scale in fp32 as torch computes it; the fp32 round trip autocast makes through the upsample is
// exact for 16-bit values). One launch instead of the casts, the upsample and the cat. Backward of the SincNet half:
//   dfs[b, t2, c] = round(sum_{t: idx(t) = t2} dout[b, t, C + c]) (fp32 sum, one rounding: the upsample's backward
//   in fp32 and autocast's cast back); the WavLM half's gradient is a view of dout.
__device__ __forceinline__ int up_idx(int t, float scale, int T2) {
  const int i = (int)floorf((float)t * scale);
  return i < T2 - 1 ? i : T2 - 1;
}

__global__ __launch_bounds__(256) void upcat_fwd_kernel(const hst* __restrict__ fw, const hst* __restrict__ fs,
                                                        hst* __restrict__ out, int B, int T1, int T2, int C,
                                                        float scale) {
  const int nq = C / 8;                      // 16-byte chunks per half row
  const int64_t n = (int64_t)B * T1 * 2 * nq;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int q2 = (int)(i % (2 * nq));
    const int64_t bt = i / (2 * nq);
    const int t = (int)(bt % T1), b = (int)(bt / T1);
    const hst* src = q2 < nq ? fw + bt * C + q2 * 8
                             : fs + ((int64_t)b * T2 + up_idx(t, scale, T2)) * C + (q2 - nq) * 8;
    *reinterpret_cast<uint4*>(out + bt * 2 * C + q2 * 8) = *reinterpret_cast<const uint4*>(src);
  }
}

__global__ __launch_bounds__(256) void upcat_bwd_kernel(const hst* __restrict__ dout, hst* __restrict__ dfs, int B,
                                                        int T1, int T2, int C, float scale) {
  const int64_t n = (int64_t)B * T2 * C;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    const int64_t bt2 = i / C;
    const int t2 = (int)(bt2 % T2), b = (int)(bt2 / T2);
    // the t with idx(t) == t2: a run around t2 * T1 / T2 (checked with the forward's own index arithmetic)
    int t0 = (int)((int64_t)t2 * T1 / T2) - 4;
    t0 = t0 < 0 ? 0 : t0;
    float acc = 0.f;
    for (int t = t0; t < T1; ++t) {
      const int k = up_idx(t, scale, T2);
      if (k > t2) break;
      if (k == t2) acc += h2f(dout[((int64_t)b * T1 + t) * 2 * C + C + c]);
    }
    dfs[i] = f2h(acc);
  }
}

}  // namespace rdx

using namespace rdx;

constexpr int SE_IMG_MAX = 64 * 1024;   // bytes of one [T][C] image (the backward stages two)
static bool se_shape_ok(int B, int T, int C, int R) {
  return B > 0 && T > 0 && C > 0 && C % SE_CH == 0 && C <= SE_CMAX && R > 0 && R <= SE_RMAX && C / SE_CH <= 32 &&
         (int64_t)T * C * 2 <= SE_IMG_MAX;
}
static int se_set_lds() {
  static bool done = false;
  if (!done) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&se_fwd_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, SE_IMG_MAX);
    if (e == hipSuccess)
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(&se_bwd_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * SE_IMG_MAX);
    if (e != hipSuccess) return (int)e;
    done = true;
  }
  return RDX_OK;
}

extern "C" int rdx_se_fwd(const void* x, const void* w1, const void* w2, void* y, void* m, void* h, void* s, int B,
                          int T, int C, int R, void* stream) {
  RDX_REQUIRE(x && w1 && w2 && y && m && h && s && se_shape_ok(B, T, C, R));
  RDX_REQUIRE((((uintptr_t)x | (uintptr_t)y) & 15) == 0);
  SeArgs a{(const hst*)x, (const hst*)w1, (const hst*)w2, (hst*)y, (hst*)m, (hst*)h, (hst*)s, B, T, C, R};
  if (const int e = se_set_lds()) return e;
  hipLaunchKernelGGL(se_fwd_kernel, dim3((unsigned)B), dim3(SE_T), T * C * 2, as_stream(stream), a);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int64_t rdx_se_bwd_part_floats(int B, int C, int R) { return (int64_t)B * 2 * R * C; }

extern "C" int rdx_se_bwd(const void* dy, const void* x, const void* w1, const void* w2, const void* m, const void* h,
                          const void* s, void* dx, float* part, float* dw1, float* dw2, int B, int T, int C, int R,
                          void* stream) {
  RDX_REQUIRE(dy && x && w1 && w2 && m && h && s && dx && part && dw1 && dw2 && se_shape_ok(B, T, C, R));
  RDX_REQUIRE((((uintptr_t)dy | (uintptr_t)x | (uintptr_t)dx) & 15) == 0);
  SeBwdArgs a{(const hst*)dy, (const hst*)x, (const hst*)w1, (const hst*)w2, (const hst*)m, (const hst*)h,
              (const hst*)s, (hst*)dx, part, B, T, C, R};
  if (const int e = se_set_lds()) return e;
  hipLaunchKernelGGL(se_bwd_kernel, dim3((unsigned)B), dim3(SE_T), 2 * T * C * 2, as_stream(stream), a);
  RDX_LAUNCH_CHECK();
  const int n = 2 * R * C;
  hipLaunchKernelGGL(se_wgrad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), part, B,
                     R * C, R * C, dw1, dw2);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

static bool ap_shape_ok(int B, int T, int C) {
  return B > 0 && T > 0 && T <= AP_TMAX && C > 0 && C <= 1024 && C % 8 == 0 && (int64_t)T * C * 2 <= AP_LDS_MAX;
}
static int ap_set_lds() {
  static bool done = false;
  if (!done) {
    for (const void* fn : {reinterpret_cast<const void*>(&attn_pool_fwd_kernel),
                           reinterpret_cast<const void*>(&attn_pool_bwd_kernel)}) {
      // the largest image (AP_LDS_MAX) with the fixed parts: 152 KB
      const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               ap_lds_bytes(1, AP_LDS_MAX / 2));
      if (e != hipSuccess) return (int)e;
    }
    done = true;
  }
  return RDX_OK;
}

extern "C" int rdx_attn_pool_fwd(const void* f, const void* w, const void* bias, void* feat, float* a, int B, int T,
                                 int C, void* stream) {
  RDX_REQUIRE(f && w && feat && a && ap_shape_ok(B, T, C) && ((uintptr_t)f & 15) == 0);
  if (const int e = ap_set_lds()) return e;
  ApArgs g{(const hst*)f, (const hst*)w, (const hst*)bias, (hst*)feat, a, B, T, C};
  hipLaunchKernelGGL(attn_pool_fwd_kernel, dim3((unsigned)B), dim3(AP_T), ap_lds_bytes(T, C), as_stream(stream), g);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_attn_pool_bwd(const void* f, const void* w, const float* a, const void* dfeat, void* df, float* part,
                                 float* dw, float* db, int B, int T, int C, void* stream) {
  RDX_REQUIRE(f && w && a && dfeat && df && part && dw && ap_shape_ok(B, T, C));
  RDX_REQUIRE((((uintptr_t)f | (uintptr_t)df) & 15) == 0);
  if (const int e = ap_set_lds()) return e;
  ApBwdArgs g{(const hst*)f, (const hst*)w, a, (const hst*)dfeat, (hst*)df, part, B, T, C};
  hipLaunchKernelGGL(attn_pool_bwd_kernel, dim3((unsigned)B), dim3(AP_T), ap_lds_bytes(T, C), as_stream(stream), g);
  RDX_LAUNCH_CHECK();
  hipLaunchKernelGGL(ap_wgrad_kernel, dim3((unsigned)((C + 1 + 255) / 256)), dim3(256), 0, as_stream(stream), part, B,
                     C, dw, db);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_upcat_fwd(const void* fw, const void* fs, void* out, int B, int T1, int T2, int C, void* stream) {
  RDX_REQUIRE(fw && fs && out && B > 0 && T1 > 0 && T2 > 0 && C > 0 && C % 8 == 0);
  RDX_REQUIRE((((uintptr_t)fw | (uintptr_t)fs | (uintptr_t)out) & 15) == 0);
  const int64_t n = (int64_t)B * T1 * (C / 4);
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(upcat_fwd_kernel, dim3((unsigned)grid), dim3(256), 0, as_stream(stream), (const hst*)fw,
                     (const hst*)fs, (hst*)out, B, T1, T2, C, (float)T2 / (float)T1);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_upcat_bwd(const void* dout, void* dfs, int B, int T1, int T2, int C, void* stream) {
  RDX_REQUIRE(dout && dfs && B > 0 && T1 > 0 && T2 > 0 && C > 0);
  const int64_t n = (int64_t)B * T2 * C;
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(upcat_bwd_kernel, dim3((unsigned)grid), dim3(256), 0, as_stream(stream), (const hst*)dout,
                     (hst*)dfs, B, T1, T2, C, (float)T2 / (float)T1);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
