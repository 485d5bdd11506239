// Diagnostic: per-phase cycle stamps of the fused attention backward (csrc/attention.hip built with
// RDX_ATTN_PROBE), at the Phase-6 shape (T = 201, H = 16, dropout 0.1) and B from argv[1].
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DRDX_ATTN_PROBE -o tools/attn_probe tools/attn_probe.cpp
//   tools/attn_probe 8
// Prints the kernel time (HIP events) and, per phase, the median / max over workgroups of the slowest
// wave's s_memtime cycles: 0-1 staging, 1-2 key-stationary loop, 2-3 dK/dV stores + K image, 3-4 dQ loop.
#include "../robust-audio-deepfake-evolution_amd/csrc/attention.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

template <typename Tp>
static Tp* dev_rand(size_t n, float scale, unsigned seed, bool bf = false) {
  std::vector<float> h(n);
  unsigned x = seed;
  for (auto& v : h) {
    x = x * 1664525u + 1013904223u;
    v = scale * (((x >> 8) & 0xffff) / 32768.f - 1.f);
  }
  Tp* d;
  CK(hipMalloc(&d, n * sizeof(Tp)));
  if (bf) {
    std::vector<__hip_bfloat16> b(n);
    for (size_t i = 0; i < n; ++i) b[i] = __float2bfloat16(h[i]);
    CK(hipMemcpy(d, b.data(), n * sizeof(Tp), hipMemcpyHostToDevice));
  } else {
    CK(hipMemcpy(d, h.data(), n * sizeof(Tp), hipMemcpyHostToDevice));
  }
  return d;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 8, T = 201, H = 16, E = H * 64, ld = 3 * E;
  auto* qkv = dev_rand<__hip_bfloat16>((size_t)B * T * ld, 0.5f, 1, true);
  auto* dO = dev_rand<__hip_bfloat16>((size_t)B * T * E, 0.5f, 2, true);
  auto* gate = dev_rand<float>((size_t)B * T * H, 0.5f, 3);
  auto* rel = dev_rand<float>((size_t)H * (2 * T - 1), 0.5f, 4);
  int64_t seed_h = 12345, *seed;
  CK(hipMalloc(&seed, 8));
  CK(hipMemcpy(seed, &seed_h, 8, hipMemcpyHostToDevice));
  __hip_bfloat16 *o, *dq;
  float *lse, *D, *dgate;
  uint32_t* mask;
  CK(hipMalloc(&o, (size_t)B * T * E * 2));
  CK(hipMalloc(&dq, (size_t)B * T * ld * 2));
  CK(hipMalloc(&lse, (size_t)B * H * T * 4));
  CK(hipMalloc(&D, (size_t)B * H * T * 4));
  CK(hipMalloc(&dgate, (size_t)B * T * H * 4));
  CK(hipMalloc(&mask, rdx_attn_keep_mask_words(B, T, H) * 4));
  if (rdx_attn_fwd(qkv, ld, qkv + E, ld, qkv + 2 * E, ld, gate, rel, seed, 3, 0.1f, 0.125f, o, E, lse, mask, B, T,
                   H, 64, nullptr))
    return 2;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e9f;
  for (int it = 0; it < 10; ++it) {
    CK(hipEventRecord(e0));
    if (rdx_attn_bwd_fused(qkv, ld, qkv + E, ld, qkv + 2 * E, ld, gate, rel, mask, 0.1f, 0.125f, o, E, lse, dO,
                           E, D, dq, dq + E, dq + 2 * E, ld, dgate, B, T, H, 64, nullptr))
      return 3;
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms);
  }
  std::vector<uint64_t> st(1 << 16);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(rdx_probe), st.size() * 8));
  const int nwg = B * H, nw = 7;
  printf("B=%d kernel %.1f us (best of 10)\n", B, best * 1e3);
  const char* names[] = {"stage", "key loop", "dK/dV + K img", "dQ loop", "tail"};
  for (int ph = 0; ph < 5; ++ph) {
    std::vector<double> v;
    for (int wg = 0; wg < nwg; ++wg) {
      double mx = 0;
      for (int w = 0; w < nw; ++w) {
        const uint64_t* p = &st[((size_t)wg * 8 + w) * 8];
        mx = std::max(mx, (double)(p[ph + 1] - p[ph]));
      }
      v.push_back(mx);
    }
    std::sort(v.begin(), v.end());
    printf("  phase %d %-14s median %8.0f  max %8.0f cycles\n", ph, names[ph], v[v.size() / 2], v.back());
  }
  auto sub = [&](int a, int b, const char* nm) {
    std::vector<double> v;
    for (int wg = 0; wg < nwg; ++wg) {
      double mx = 0;
      for (int w = 0; w < nw; ++w) {
        const uint64_t* p = &st[((size_t)wg * 8 + w) * 8];
        mx = std::max(mx, (double)(p[b] - p[a]));
      }
      v.push_back(mx);
    }
    std::sort(v.begin(), v.end());
    printf("  %-34s median %8.0f  max %8.0f cycles\n", nm, v[v.size() / 2], v.back());
  };
  sub(0, 6, "phase 0a loads + LDS writes");
  sub(6, 1, "phase 0b barrier + D + barrier");
  sub(2, 7, "phase 2a dK/dV stores");
  sub(7, 3, "phase 2b barrier + K img + barrier");
  // whole-WG span and start skew
  std::vector<double> span, start;
  uint64_t t0 = ~0ull;
  for (int wg = 0; wg < nwg; ++wg) t0 = std::min(t0, st[(size_t)wg * 64]);
  for (int wg = 0; wg < nwg; ++wg) {
    uint64_t a = ~0ull, b = 0;
    for (int w = 0; w < nw; ++w) {
      a = std::min(a, st[((size_t)wg * 8 + w) * 8]);
      b = std::max(b, st[((size_t)wg * 8 + w) * 8 + 5]);
    }
    span.push_back((double)(b - a));
    start.push_back((double)(a - t0));
  }
  std::sort(span.begin(), span.end());
  std::sort(start.begin(), start.end());
  printf("  WG span median %.0f max %.0f cycles; start skew max %.0f cycles\n", span[span.size() / 2], span.back(),
         start.back());
  return 0;
}
