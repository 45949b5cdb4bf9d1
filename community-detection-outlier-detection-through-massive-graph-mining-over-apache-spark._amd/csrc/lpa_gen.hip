// Synthetic inputs generated in HBM: R-MAT (configs C3/C4),
// the planted-partition SBM (C2) and the Chung-Lu power-law graph (C5).  Every draw is a pure function of
// (seed, edge index, slot) through a splitmix64 counter RNG, so the device
// output is bit-identical to the CPU restatement in oracle/lpa_oracle.c.
#include <math.h>

#include <vector>

#include "lpa_internal.h"

namespace lpa {
namespace {

__device__ __forceinline__ u64 sm64(u64 x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__host__ __device__ inline u64 sm64_h(u64 x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ u32 below(u32 r, u32 n) { return (u32)(((u64)r * n) >> 32); }

constexpr u32 kTA = 2448131358u;  // floor(.57 * 2^32)
constexpr u32 kTB = 3264175144u;  // floor(.76 * 2^32)
constexpr u32 kTC = 4080218931u;  // floor(.95 * 2^32)

__device__ __forceinline__ u64 scramble(u64 x, u64 mask, int sh, u64 m1, u64 m2, u64 c1) {
  x = (x * m1 + c1) & mask;
  x ^= x >> sh;
  x = (x * m2) & mask;
  x ^= x >> sh;
  x = (x * m1 + c1) & mask;
  return x;
}

__global__ void k_rmat(int scale, int64_t m, u64 seed_mixed, int do_scramble, u64 m1, u64 m2,
                       u64 c1, int32_t* __restrict__ src, int32_t* __restrict__ dst) {
  const u64 mask = (1ull << scale) - 1ull;
  const int sh = scale / 2 + 1;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m;
       e += (int64_t)gridDim.x * blockDim.x) {
    u64 u = 0, v = 0, r = 0;
    for (int l = 0; l < scale; ++l) {
      if ((l & 1) == 0) r = sm64(seed_mixed + (u64)e * 32ull + (u64)(l >> 1));
      const u32 r32 = (l & 1) ? (u32)r : (u32)(r >> 32);
      const u64 bu = r32 >= kTB ? 1ull : 0ull;
      const u64 bv = (r32 >= kTA && r32 < kTB) || r32 >= kTC ? 1ull : 0ull;
      u = (u << 1) | bu;
      v = (v << 1) | bv;
    }
    if (do_scramble) {
      u = scramble(u, mask, sh, m1, m2, c1);
      v = scramble(v, mask, sh, m1, m2, c1);
    }
    src[e] = (int32_t)u;
    dst[e] = (int32_t)v;
  }
}

__global__ void k_sbm(u32 V, u32 blocks, int64_t m, u32 p_in, u64 seed_mixed,
                      int32_t* __restrict__ src, int32_t* __restrict__ dst) {
  const u32 bs = V / blocks;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m;
       e += (int64_t)gridDim.x * blockDim.x) {
    const u64 r0 = sm64(seed_mixed + (u64)e * 32ull + 0ull);
    const u64 r1 = sm64(seed_mixed + (u64)e * 32ull + 1ull);
    const u32 u = below((u32)(r0 >> 32), V);
    u32 b = u / bs;
    if (b >= blocks) b = blocks - 1;
    const u32 lo = b * bs;
    const u32 hi = (b == blocks - 1) ? V : lo + bs;
    u32 v;
    if ((u32)r0 < p_in) {
      v = lo + below((u32)(r1 >> 32), hi - lo);
    } else {
      const u32 w = below((u32)(r1 >> 32), V - (hi - lo));
      v = w < lo ? w : w + (hi - lo);
    }
    src[e] = (int32_t)u;
    dst[e] = (int32_t)v;
  }
}

// Chung-Lu (C5): both endpoints of an edge drawn independently with P(i) ~ w_i =
// (i + i0)^(-1/(gamma-1)) over weight ranks i, then mapped to vertex ids by the
// seeded affine permutation id = (mul i + add) mod V.  The sampler is integer-only
// on the device: a 62-bit uniform draw, binary search of the quantized cumulative
// weight table Q[0..V] (Q[0] = 0, Q[V] = 2^62, built on the host).
__global__ void k_chunglu(const u64* __restrict__ Q, u32 V, int64_t m, u64 seed_mixed, u64 mul,
                          u64 add, int32_t* __restrict__ src, int32_t* __restrict__ dst) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m;
       e += (int64_t)gridDim.x * blockDim.x) {
    u32 id[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const u64 r = sm64(seed_mixed + (u64)e * 32ull + (u64)k) >> 2;
      u32 lo = 0, hi = V;  // Q[lo] <= r < Q[hi]
      while (hi - lo > 1) {
        const u32 mid = lo + ((hi - lo) >> 1);
        if (Q[mid] <= r) lo = mid; else hi = mid;
      }
      id[k] = (u32)((mul * (u64)lo + add) % (u64)V);
    }
    src[e] = (int32_t)id[0];
    dst[e] = (int32_t)id[1];
  }
}

inline unsigned gen_grid(int64_t m) {
  int64_t b = (m + 255) / 256;
  if (b < 1) b = 1;
  if (b > 262144) b = 262144;
  return (unsigned)b;
}

}  // namespace

int gen_rmat(int32_t scale, int64_t m, uint64_t seed, int32_t do_scramble, int32_t* d_src,
             int32_t* d_dst, hipStream_t s) {
  if (scale < 1 || scale > 31 || m < 0) {
    set_error("gen_rmat: scale must be in [1, 31] and m >= 0 (got %d, %lld)", scale, (long long)m);
    return LPA_EINVAL;
  }
  const u64 m1 = sm64_h(seed ^ 0x1234567ull) | 1ull;
  const u64 m2 = sm64_h(seed ^ 0x89abcdefull) | 1ull;
  const u64 c1 = sm64_h(seed ^ 0x5555ull);
  if (m == 0) return LPA_OK;
  hipLaunchKernelGGL(k_rmat, dim3(gen_grid(m)), dim3(256), 0, s, scale, m, sm64_h(seed),
                     do_scramble, m1, m2, c1, d_src, d_dst);
  LPA_HIP(hipGetLastError());
  return LPA_OK;
}

// Host half of the Chung-Lu sampler (restated in oracle/lpa_oracle.c: the same
// double arithmetic in the same order, so both build the identical table).
// i0 is set by bisection so that the expected maximum degree 2 m w_0 / W equals
// max_deg, with W from the integral approximation; the table itself uses the
// exact sequential sum.
void chunglu_table(int32_t V, int64_t m, double gamma, double max_deg, uint64_t seed, u64* Q,
                   u64* mul_out, u64* add_out) {
  const double a = 1.0 / (gamma - 1.0);
  double i0 = 1.0;
  if (max_deg > 0.0) {
    auto expmax = [&](double x) {
      const double S = (pow((double)V + x, 1.0 - a) - pow(x, 1.0 - a)) / (1.0 - a) + 0.5 * pow(x, -a);
      return 2.0 * (double)m * pow(x, -a) / S;
    };
    double lo = log(1e-3), hi = log((double)V);
    for (int it = 0; it < 200; ++it) {
      const double mid = 0.5 * (lo + hi);
      if (expmax(exp(mid)) > max_deg) lo = mid; else hi = mid;
    }
    i0 = exp(0.5 * (lo + hi));
  }
  double W = 0.0;
  for (int32_t i = 0; i < V; ++i) W += pow((double)i + i0, -a);
  const double two62 = 4611686018427387904.0;
  double c = 0.0;
  for (int32_t i = 0; i < V; ++i) {
    Q[i] = (u64)(c / W * two62);
    c += pow((double)i + i0, -a);
  }
  Q[V] = 1ull << 62;
  u64 mul = V > 1 ? sm64_h(seed ^ 0xC0FFEEull) % (u64)V : 1ull;
  auto gcd = [](u64 x, u64 y) { while (y) { u64 t = x % y; x = y; y = t; } return x; };
  if (mul == 0) mul = 1;
  while (V > 1 && gcd(mul, (u64)V) != 1) mul = mul + 1 == (u64)V ? 1 : mul + 1;
  *mul_out = mul;
  *add_out = V > 1 ? sm64_h(seed ^ 0xADDull) % (u64)V : 0ull;
}

int gen_chunglu(int32_t V, int64_t m, double gamma, double max_deg, uint64_t seed, int32_t* d_src,
                int32_t* d_dst, hipStream_t s) {
  if (V < 1 || m < 0 || !(gamma > 1.0 && gamma < 10.0)) {
    set_error("gen_chunglu: need V >= 1, m >= 0 and 1 < gamma < 10");
    return LPA_EINVAL;
  }
  if (m == 0) return LPA_OK;
  std::vector<u64> Q;
  try {
    Q.resize((size_t)V + 1);
  } catch (...) {
    set_error("gen_chunglu: host table allocation failed");
    return LPA_ENOMEM;
  }
  u64 mul = 1, add = 0;
  chunglu_table(V, m, gamma, max_deg, seed, Q.data(), &mul, &add);
  u64* dQ = nullptr;
  LPA_HIP(hipMalloc(&dQ, Q.size() * sizeof(u64)));
  hipError_t e = hipMemcpyAsync(dQ, Q.data(), Q.size() * sizeof(u64), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_chunglu, dim3(gen_grid(m)), dim3(256), 0, s, dQ, (u32)V, m, sm64_h(seed),
                       mul, add, d_src, d_dst);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(dQ);
  LPA_HIP(e);
  return LPA_OK;
}

int gen_sbm(int32_t V, int32_t blocks, int64_t m, uint32_t p_in_q32, uint64_t seed, int32_t* d_src,
            int32_t* d_dst, hipStream_t s) {
  if (V < 1 || blocks < 1 || blocks > V || m < 0) {
    set_error("gen_sbm: need 1 <= blocks <= V and m >= 0");
    return LPA_EINVAL;
  }
  if (m == 0) return LPA_OK;
  hipLaunchKernelGGL(k_sbm, dim3(gen_grid(m)), dim3(256), 0, s, (u32)V, (u32)blocks, m, p_in_q32,
                     sm64_h(seed), d_src, d_dst);
  LPA_HIP(hipGetLastError());
  return LPA_OK;
}

}  // namespace lpa
