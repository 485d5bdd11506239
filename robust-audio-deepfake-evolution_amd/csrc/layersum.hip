// WavLM layer-weighted sum (25 hidden states) for gfx950.
//
// Reference: WavLMFrontend.forward (src/models/DualStreamSEMamba.py:427-437):
//   stacked = torch.stack(hidden_states)            # materialises 25 x [B, T, 1024]
//   out = (softmax(layer_weights).view(-1,1,1,1) * stacked).sum(0)
// Here the states are read in place through a pointer table (no stack copy), the softmax of the
// 25 weights is taken in-kernel, and every lane streams 16 B per state per step (HBM-bound).
#include "common.h"

namespace rdx {

constexpr int LWS_MAXL = 64;
constexpr int LWS_THREADS = 256;
constexpr int LWS_NBLK = 1024;  // fixed grid for the backward partial dots (grid-stride)

struct PtrTable {
  const void* p[LWS_MAXL];
};
struct MutPtrTable {
  void* p[LWS_MAXL];
};

template <typename T> struct Vec4;
template <> struct Vec4<float> {
  using type = float4;
  static __device__ __forceinline__ void load(const float* p, int64_t i, float v[4]) {
    float4 q = *reinterpret_cast<const float4*>(p + i);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
  static __device__ __forceinline__ void store(float* p, int64_t i, const float v[4]) {
    *reinterpret_cast<float4*>(p + i) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct Vec4<hst> {
  static __device__ __forceinline__ void load(const hst* p, int64_t i, float v[4]) {
    uint2 q = *reinterpret_cast<const uint2*>(p + i);
    v[0] = hlo(q.x); v[1] = hhi(q.x);
    v[2] = hlo(q.y); v[3] = hhi(q.y);
  }
  static __device__ __forceinline__ void store(hst* p, int64_t i, const float v[4]) {
    hst b0 = f2h(v[0]), b1 = f2h(v[1]);
    hst b2 = f2h(v[2]), b3 = f2h(v[3]);
    uint2 q;
    q.x = (uint32_t)(*reinterpret_cast<uint16_t*>(&b0)) | ((uint32_t)(*reinterpret_cast<uint16_t*>(&b1)) << 16);
    q.y = (uint32_t)(*reinterpret_cast<uint16_t*>(&b2)) | ((uint32_t)(*reinterpret_cast<uint16_t*>(&b3)) << 16);
    *reinterpret_cast<uint2*>(p + i) = q;
  }
};

__device__ __forceinline__ void softmax_into(const float* __restrict__ w, int nl, float* s_p) {
  if (threadIdx.x < 64) {
    float v = (threadIdx.x < nl) ? w[threadIdx.x] : -INFINITY;
    float m = v;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float e = (threadIdx.x < nl) ? __expf(v - m) : 0.f;
    float s = wave_sum(e);
    if (threadIdx.x < nl) s_p[threadIdx.x] = e / s;
  }
  __syncthreads();
}

template <typename T>
__global__ __launch_bounds__(LWS_THREADS) void lws_fwd_kernel(PtrTable hs, int nl, const float* __restrict__ w,
                                                              T* __restrict__ out, int64_t n) {
  __shared__ float s_p[LWS_MAXL];
  softmax_into(w, nl, s_p);
  const int64_t nv = n / 4;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += (int64_t)gridDim.x * blockDim.x) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    // 8 layers' loads in flight, then their FMAs in layer order (one round trip per layer before); a layer past nl
    // re-reads the last one and is not added
    for (int l0 = 0; l0 < nl; l0 += 8) {
      float h[8][4];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        Vec4<T>::load(reinterpret_cast<const T*>(hs.p[l0 + k < nl ? l0 + k : nl - 1]), v * 4, h[k]);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (l0 + k < nl) {
          const float p = s_p[l0 + k];
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] = fmaf(p, h[k][j], acc[j]);
        }
      }
    }
    Vec4<T>::store(out, v * 4, acc);
  }
  // tail (n % 4)
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    int64_t i = (n & ~(int64_t)3) + threadIdx.x;
    float acc = 0.f;
    for (int l = 0; l < nl; ++l) acc = fmaf(s_p[l], ld(reinterpret_cast<const T*>(hs.p[l]), i), acc);
    st(out, i, acc);
  }
}

template <typename T>
__global__ __launch_bounds__(LWS_THREADS) void lws_bwd_kernel(PtrTable hs, MutPtrTable dhs, int nl,
                                                              const float* __restrict__ w,
                                                              const T* __restrict__ g,
                                                              float* __restrict__ dot_part, int64_t n) {
  __shared__ float s_p[LWS_MAXL];
  __shared__ float s_red[LWS_THREADS / 64][LWS_MAXL];
  softmax_into(w, nl, s_p);
  const int64_t nv = n / 4;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // v outer, layers inner in batches of 8 (g loaded once per v, 8 layers' h loads in flight before their dots and
  // dh stores); each layer's dot still sums this thread's v in the grid-stride order, as one loop per layer did
  float dot[LWS_MAXL];
#pragma unroll
  for (int l = 0; l < LWS_MAXL; ++l) dot[l] = 0.f;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += (int64_t)gridDim.x * blockDim.x) {
    float gv[4];
    Vec4<T>::load(g, v * 4, gv);
#pragma unroll
    for (int l0 = 0; l0 < LWS_MAXL; l0 += 8) {
      if (l0 >= nl) continue;   // (continue, not break: the loop stays fully unrolled, dot[] in registers)
      float hv[8][4];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        Vec4<T>::load(reinterpret_cast<const T*>(hs.p[l0 + k < nl ? l0 + k : nl - 1]), v * 4, hv[k]);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (l0 + k < nl) {
#pragma unroll
          for (int j = 0; j < 4; ++j) dot[l0 + k] = fmaf(gv[j], hv[k][j], dot[l0 + k]);
          T* dh = reinterpret_cast<T*>(dhs.p[l0 + k]);
          if (dh) {
            const float p = s_p[l0 + k];
            const float o[4] = {p * gv[0], p * gv[1], p * gv[2], p * gv[3]};
            Vec4<T>::store(dh, v * 4, o);
          }
        }
      }
    }
  }
#pragma unroll
  for (int l = 0; l < LWS_MAXL; ++l) {
    if (l >= nl) continue;
    float d = dot[l];
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {   // tail (n % 4)
      const T* h = reinterpret_cast<const T*>(hs.p[l]);
      T* dh = reinterpret_cast<T*>(dhs.p[l]);
      const int64_t i = (n & ~(int64_t)3) + threadIdx.x;
      const float gg = ld(g, i);
      d = fmaf(gg, ld(h, i), d);
      if (dh) st(dh, i, s_p[l] * gg);
    }
    d = wave_sum(d);
    if (lane == 0) s_red[wid][l] = d;
  }
  __syncthreads();
  if (threadIdx.x < nl) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < LWS_THREADS / 64; ++k) s += s_red[k][threadIdx.x];
    dot_part[(int64_t)blockIdx.x * nl + threadIdx.x] = s;
  }
}

}  // namespace rdx

using namespace rdx;

#define LWS_DISPATCH(dtype, ...)                                    \
  do {                                                              \
    if ((dtype) == RDX_F32) {                                       \
      using T = float;                                              \
      __VA_ARGS__;                                                  \
    } else if ((dtype) == RDX_BF16) {                               \
      using T = hst;                                     \
      __VA_ARGS__;                                                  \
    } else {                                                        \
      return RDX_EINVAL;                                            \
    }                                                               \
  } while (0)

extern "C" int rdx_layer_wsum_nblk(int64_t n) {
  int64_t nv = (n / 4 + LWS_THREADS - 1) / LWS_THREADS;
  if (nv < 1) nv = 1;
  return (int)(nv < LWS_NBLK ? nv : LWS_NBLK);
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

extern "C" int rdx_layer_wsum_fwd(int dtype, int nl, const void* const* hs, const float* w, void* out,
                                  int64_t n, void* stream) {
  RDX_REQUIRE(hs && w && out && n > 0 && nl > 0);
  if (nl > LWS_MAXL) return RDX_EUNSUPPORTED;
  PtrTable t{};
  for (int l = 0; l < nl; ++l) {
    RDX_REQUIRE(hs[l] != nullptr);
    if (!aligned16(hs[l])) return RDX_EUNSUPPORTED;
    t.p[l] = hs[l];
  }
  if (!aligned16(out)) return RDX_EUNSUPPORTED;
  int nblk = rdx_layer_wsum_nblk(n);
  LWS_DISPATCH(dtype, hipLaunchKernelGGL(lws_fwd_kernel<T>, dim3(nblk), dim3(LWS_THREADS), 0,
                                         as_stream(stream), t, nl, w, (T*)out, n));
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

extern "C" int rdx_layer_wsum_bwd(int dtype, int nl, const void* const* hs, const float* w, const void* g,
                                  void* const* dhs, float* dot_part, int64_t n, void* stream) {
  RDX_REQUIRE(hs && dhs && w && g && dot_part && n > 0 && nl > 0);
  if (nl > LWS_MAXL) return RDX_EUNSUPPORTED;
  PtrTable t{};
  MutPtrTable dt{};
  for (int l = 0; l < nl; ++l) {
    RDX_REQUIRE(hs[l] != nullptr);   // dhs[l] == nullptr: that state's gradient p_l * g is not written
    if (!aligned16(hs[l]) || (dhs[l] && !aligned16(dhs[l]))) return RDX_EUNSUPPORTED;
    t.p[l] = hs[l];
    dt.p[l] = dhs[l];
  }
  if (!aligned16(g)) return RDX_EUNSUPPORTED;
  int nblk = rdx_layer_wsum_nblk(n);
  LWS_DISPATCH(dtype, hipLaunchKernelGGL(lws_bwd_kernel<T>, dim3(nblk), dim3(LWS_THREADS), 0,
                                         as_stream(stream), t, dt, nl, w, (const T*)g, dot_part, n));
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

// ---- fp32 -> 16-bit casts of up to RDX_CAST_MAX tensors in one launch (the window's per-window cast of the
// detector head's fp32 weights to the autocast dtype, radhip/window.py: one launch instead of one per tensor)
constexpr int RDX_CAST_MAX = 64;
struct CastTable {
  const float* src[RDX_CAST_MAX];
  hst* dst[RDX_CAST_MAX];
  int64_t n[RDX_CAST_MAX];
};

__global__ __launch_bounds__(256) void cast_many_kernel(CastTable t) {
  const int k = blockIdx.y;
  const float* __restrict__ s = t.src[k];
  hst* __restrict__ d = t.dst[k];
  const int64_t n = t.n[k];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) d[i] = f2h(s[i]);
}

extern "C" int rdx_cast_f32_many(int n, const float* const* src, void* const* dst, const int64_t* numel,
                                 void* stream) {
  RDX_REQUIRE(n >= 0 && (n == 0 || (src && dst && numel)));
  if (n > RDX_CAST_MAX) return RDX_EUNSUPPORTED;
  if (n == 0) return RDX_OK;
  CastTable t{};
  int64_t mx = 1;
  for (int k = 0; k < n; ++k) {
    RDX_REQUIRE(numel[k] >= 0 && (numel[k] == 0 || (src[k] && dst[k])));   // an empty tensor may be null
    t.src[k] = src[k];
    t.dst[k] = reinterpret_cast<hst*>(dst[k]);
    t.n[k] = numel[k];
    mx = numel[k] > mx ? numel[k] : mx;
  }
  const int64_t bx = (mx + 255) / 256;
  hipLaunchKernelGGL(cast_many_kernel, dim3((unsigned)(bx < 64 ? bx : 64), (unsigned)n), dim3(256), 0,
                     as_stream(stream), t);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

// ---- dst[k] += src[k] (or dst[k] = src[k]) over up to RDX_ADDM_MAX fp32 tensors in one launch: the window's per-pass
// hand-over of autograd's parameter gradients into the flat gradient buffer and the feature_projection copies
// (radhip/window.py). torch's multi-tensor add gives each workgroup a 64 K-element chunk, so a pass's few hundred
// thousand elements run on a dozen workgroups at ~0.15 TB/s; here a workgroup owns 4096 elements (16 per lane, every
// load of the lane issued before its stores) and the tensors' chunks are laid end to end over the grid.
constexpr int RDX_ADDM_MAX = 64;
constexpr int RDX_ADDM_CHUNK = 4096;
struct AddManyTable {
  float* dst[RDX_ADDM_MAX];
  const float* src[RDX_ADDM_MAX];
  int64_t n[RDX_ADDM_MAX];
  int start[RDX_ADDM_MAX + 1];  // first workgroup of each tensor; start[nt] = the grid size
};

template <bool kCopy>
__global__ __launch_bounds__(256) void add_many_kernel(AddManyTable t, int nt) {
  const int b = blockIdx.x;
  int k = 0;
  while (k + 1 < nt && t.start[k + 1] <= b) ++k;   // workgroup-uniform
  const int64_t base = (int64_t)(b - t.start[k]) * RDX_ADDM_CHUNK + threadIdx.x;
  const int64_t n = t.n[k];
  float* __restrict__ d = t.dst[k];
  const float* __restrict__ s = t.src[k];
  constexpr int kPer = RDX_ADDM_CHUNK / 256;
  float a[kPer], c[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t i = base + j * 256;
    a[j] = i < n ? s[i] : 0.f;
    if (!kCopy) c[j] = i < n ? d[i] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t i = base + j * 256;
    if (i < n) d[i] = kCopy ? a[j] : c[j] + a[j];
  }
}

extern "C" int rdx_add_f32_many(int n, void* const* dst, const float* const* src, const int64_t* numel, int copy,
                                void* stream) {
  RDX_REQUIRE(n >= 0 && (n == 0 || (src && dst && numel)) && (copy == 0 || copy == 1));
  if (n > RDX_ADDM_MAX) return RDX_EUNSUPPORTED;
  AddManyTable t{};
  int64_t blocks = 0;
  for (int k = 0; k < n; ++k) {
    RDX_REQUIRE(numel[k] >= 0 && (numel[k] == 0 || (src[k] && dst[k])));
    t.dst[k] = reinterpret_cast<float*>(dst[k]);
    t.src[k] = src[k];
    t.n[k] = numel[k];
    t.start[k] = (int)blocks;
    blocks += (numel[k] + RDX_ADDM_CHUNK - 1) / RDX_ADDM_CHUNK;
    if (blocks > (int64_t)INT32_MAX) return RDX_EUNSUPPORTED;
  }
  t.start[n] = (int)blocks;
  if (blocks == 0) return RDX_OK;
  if (copy)
    hipLaunchKernelGGL(add_many_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), t, n);
  else
    hipLaunchKernelGGL(add_many_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), t, n);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}

// ---- Column sums of row-partial buffers: out[c] = sum_r in[r * ld + c] for up to CS_MAXP problems per launch (the
// per-(direction, utterance, chunk) partial rows of the scan backward and of the depthwise conv backward: one launch
// instead of a torch reduction each). A 256-thread block owns 32 columns x 8 row groups; a thread sums every 8th row
// in row order, the 8 group sums are added in group order (fixed order: deterministic).
namespace rdx {
constexpr int CS_MAXP = 4;
struct ColSumTable {
  const float* in[CS_MAXP];
  float* out[CS_MAXP];
  int64_t ld[CS_MAXP];
  int rows[CS_MAXP];
  int cols[CS_MAXP];
};
__global__ __launch_bounds__(256) void colsum_many_kernel(ColSumTable t) {
  __shared__ float red[8][33];
  const int pb = blockIdx.y;
  const int c = blockIdx.x * 32 + (threadIdx.x & 31), g = threadIdx.x >> 5;
  if (blockIdx.x * 32 >= t.cols[pb]) return;   // block-uniform
  const float* in = t.in[pb];
  const int rows = t.rows[pb];
  const int64_t ld = t.ld[pb];
  float s = 0.f;
  if (c < t.cols[pb]) {
    int r = g;
    for (; r + 24 < rows; r += 32) {   // four rows of this group in flight per step, added in row order
      const float a0 = in[(int64_t)r * ld + c], a1 = in[(int64_t)(r + 8) * ld + c];
      const float a2 = in[(int64_t)(r + 16) * ld + c], a3 = in[(int64_t)(r + 24) * ld + c];
      s = (((s + a0) + a1) + a2) + a3;
    }
    for (; r < rows; r += 8) s += in[(int64_t)r * ld + c];
  }
  red[g][threadIdx.x & 31] = s;
  __syncthreads();
  if (g == 0 && c < t.cols[pb]) {
    float tot = red[0][threadIdx.x];
#pragma unroll
    for (int k = 1; k < 8; ++k) tot += red[k][threadIdx.x];
    t.out[pb][c] = tot;
  }
}
}  // namespace rdx

extern "C" int rdx_colsum_many(int n, const float* const* in, const int* rows, const int* cols, const int64_t* ld,
                               float* const* out, void* stream) {
  RDX_REQUIRE(n > 0 && n <= rdx::CS_MAXP && in && rows && cols && ld && out);
  rdx::ColSumTable t{};
  int maxc = 0;
  for (int k = 0; k < n; ++k) {
    RDX_REQUIRE(in[k] && out[k] && rows[k] > 0 && cols[k] > 0 && ld[k] >= cols[k]);
    t.in[k] = in[k];
    t.out[k] = out[k];
    t.ld[k] = ld[k];
    t.rows[k] = rows[k];
    t.cols[k] = cols[k];
    maxc = cols[k] > maxc ? cols[k] : maxc;
  }
  hipLaunchKernelGGL(rdx::colsum_many_kernel, dim3((unsigned)((maxc + 31) / 32), (unsigned)n), dim3(256), 0,
                     as_stream(stream), t);
  RDX_LAUNCH_CHECK();
  return RDX_OK;
}
